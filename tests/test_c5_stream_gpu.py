"""BASELINE config 5 on the GPU: the ordered mixed contains/add stream with C5's own kernel
instantiation -- 64-byte fixed keys (KLEN = 64) on tryInit(1e6, 1e-3) tenants (m = 14,377,587,
k = 10, so KMAX = 16) and on k = 7 tenants (KMAX = 8) -- replayed command by command on the
oracle (oracle.bloom_stream = orc_bloom_stream: each command is add(T) / contains(T),
M/RedissonBloomFilter.java:99-102,198-201, executed one after another).

Per-command replies, both counts and every tenant bitmap (the Redis string, `GET name`) must be
bit-identical.  Tenants are Zipf(s = 1)-skewed, 10% adds, the filters start at their design fill
(random bitmaps imported as Redis strings, as bench.py's C5 leg does), and keys repeat so adds hit
present keys and contains hit keys added earlier in the same chunk.
"""
import numpy as np
import pytest

from oracle import oracle as O
from redisson_amd import BloomHandle, bloom_stream
from redisson_amd import _lib as L

pytestmark = pytest.mark.gpu



def _zipf_tenants(rng, nt, n, s=1.0):
    w = 1.0 / np.arange(1, nt + 1, dtype=np.float64) ** s
    cdf = np.cumsum(w)
    cdf /= cdf[-1]
    return np.minimum(np.searchsorted(cdf, rng.random(n)), nt - 1).astype(np.uint32)


def _c5_case(client, fresh, seed, nt, expected, fpp, n, chunk=0, klen=64, table8=None, hot_last=False, geometry=None):
    """expected: one tryInit size for every tenant, or a per-tenant list.  hot_last: the Zipf-hottest
    tenant is the LAST handle (the largest filter id of the call) instead of the first.  geometry:
    the (bb, fbits, pb, chunk) the call must have run with (rbx_bench_stream_geometry)."""
    rng = np.random.default_rng(seed)
    names = [f"{fresh}-{t}" for t in range(nt)]
    refs, handles = [], []
    sizes = [expected] * nt if np.isscalar(expected) else list(expected)
    for nm, ex in zip(names, sizes):
        f = client.getBloomFilter(nm)
        assert f.tryInit(ex, fpp)
        nb = (f.getSize() + 7) // 8
        bm = rng.integers(0, 256, size=nb, dtype=np.uint8)  # design fill 0.5
        f.importBitmap(bm.tobytes())
        r = O.OracleBloom(f.getSize(), f.getHashIterations())
        r.bitmap[:nb] = bm
        r.redis_len = nb
        refs.append(r)
        handles.append(BloomHandle(client, nm))
    kf = _zipf_tenants(rng, nt, n)
    if hot_last:
        first, last = kf == 0, kf == nt - 1
        kf[first], kf[last] = nt - 1, 0
    if nt > 1 << 16:  # ids past 2^16 (the tag's filter-id field) really occur
        assert int(kf.max()) >= 1 << 16 and np.count_nonzero(kf >= 1 << 8) > n // 4
    op = (rng.random(n) < 0.1).astype(np.uint8)
    pool = rng.integers(0, 256, size=(n // 4, klen), dtype=np.uint8)
    keys = pool[rng.integers(0, len(pool), size=n)]
    # a contains right after the add of the same key on the same tenant, every 101 commands
    idx = np.arange(0, n - 1, 101)
    op[idx], op[idx + 1] = 1, 0
    kf[idx + 1] = kf[idx]
    keys[idx + 1] = keys[idx]
    assert L.lib().rbx_tune(b"stream_chunk", chunk) == 0
    if table8 is not None:
        assert L.lib().rbx_tune(b"stream_table8", table8) == 0
    try:
        out, counts = bloom_stream(client, handles, kf, op, _fixed(keys))
        if geometry is not None:
            g = np.zeros(4, np.uint64)
            assert L.lib().rbx_bench_stream_geometry(client.ctx, g.ctypes.data_as(L.u64p)) == 0
            assert tuple(int(x) for x in g) == tuple(geometry), (g, geometry)
    finally:
        L.lib().rbx_tune(b"stream_chunk", 0)
        L.lib().rbx_tune(b"stream_table8", 1)
    want, wc = O.bloom_stream(refs, kf, op, keys, None, stride=klen)
    bad = np.flatnonzero(out != want)
    assert bad.size == 0, (bad.size, bad[:10], out[bad[:10]], want[bad[:10]], kf[bad[:10]], op[bad[:10]])
    assert [int(counts[0]), int(counts[1])] == wc
    # the stream did real work: present contains and new adds on the hot tenants
    assert wc[0] > 0 and wc[1] > 0
    for nm, r in zip(names, refs):
        assert client.getBloomFilter(nm).exportBitmap() == r.redis_string(), nm
    for h in handles:
        h.close()
    for nm in names:
        client.getBloomFilter(nm).delete()
    return wc


def _fixed(keys):
    from redisson_amd import Arena

    return Arena.fixed(keys)


def test_c5_instantiation_two_full_chunks(client, fresh):
    """C5 exactly: tryInit(1e6, 1e-3) tenants (14,377,587 bits, k = 10 -> k_stream_*<64, 16>), 64-byte
    keys, 14M commands = two chunks at the production chunk size (8-byte table: 2^27 / 10 rounded to
    128 = 13,421,696 commands for 200 tenants; C5's 100k tenants get 2^23 - 128)."""
    f = client.getBloomFilter(fresh + "-probe")
    f.tryInit(1_000_000, 1e-3)
    assert (f.getSize(), f.getHashIterations()) == (14_377_587, 10)
    f.delete()
    _c5_case(client, fresh, seed=0x5EED0005, nt=200, expected=1_000_000, fpp=1e-3, n=14_000_000)


def test_c5_kmax8_many_chunks(client, fresh):
    """k = 7 tenants (tryInit(1e6, 0.01): 9,585,058 bits -> k_stream_*<64, 8>), 64-byte keys, 2M commands
    in 300k-command chunks."""
    _c5_case(client, fresh, seed=77, nt=64, expected=1_000_000, fpp=0.01, n=2_000_000, chunk=300_000)


def test_c5_shared_bits_and_claimed_lookups(client, fresh):
    """Add replies from the slot of each add's first zero-bit claim (k_stream_final8, before the walk)
    and first-setter lookups as rounds of the slot contains kernel.  Keys repeat (a quarter of the
    stream is distinct) and 80 Zipf tenants share bits within a chunk, so an add's first zero bit is
    often claimed by an earlier add (final8's slow path), occupied home slots make claims probe on, and
    many contains meet a bit claimed earlier in the chunk (the lookup round finds it)."""
    _c5_case(client, fresh, seed=929, nt=80, expected=1_000_000, fpp=1e-3, n=1_200_000, chunk=400_000)


@pytest.mark.parametrize("table8", [0, 1])
def test_c5_first_setter_tables_agree(client, fresh, table8):
    """The r03 16-byte epoch-tagged first-setter table (stream_table8 0) and the r04 8-byte table with
    the walk commit (1, default) on the same C5-shaped stream: both must equal the oracle."""
    _c5_case(client, fresh, seed=4242, nt=300, expected=1_000_000, fpp=1e-3, n=1_500_000, chunk=500_000,
             table8=table8)


def test_c5_k10_chunk_boundaries(client, fresh):
    """C5 tenants and keys in 303,031-command chunks (= 101 * 3000 + 1: the add at 303,030 and the
    contains of the same key at 303,031 sit on the two sides of the first boundary; the earlier
    chunk's commit must land before the next chunk probes)."""
    _c5_case(client, fresh, seed=91, nt=100, expected=1_000_000, fpp=1e-3, n=2_000_000, chunk=303_031)


@pytest.mark.parametrize("table8", [1, 0])
def test_c5_100k_tenants_filter_ids_past_2_17(client, fresh, table8):
    """C5's tenant count.  The first-setter entries carry the filter's index in the call
    (up to 2^17 here), so the bench leg's id range is checked against the oracle too: 100,000
    tryInit(1000, 1e-3) tenants (14,377 bits, k = 10 -> the same <64, 16> instantiation as C5, 1.8 KB
    each), Zipf(1.0) tenants, 10% adds, 64-byte keys, 2.1M commands in three chunks, on the 8-byte table
    (1) and the 16-byte fallback (0).  Per-command replies, both counts and every tenant's bitmap must be
    identical."""
    f = client.getBloomFilter(fresh + "-probe")
    f.tryInit(1000, 1e-3)
    assert (f.getSize(), f.getHashIterations()) == (14_377, 10)
    f.delete()
    wc = _c5_case(client, fresh, seed=0xC5100 + 23 * (1 - table8), nt=100_000, expected=1000, fpp=1e-3, n=2_100_000,
                  chunk=700_000, table8=table8)
    assert wc[1] > 10_000


@pytest.mark.parametrize("table8", [1, 0])
def test_stream_k20_variable_keys(client, fresh, table8):
    """The stream's KMAX = 32 instantiation and variable-length keys (KLEN = 0: the generic hash
    path of the probe, the slot contains kernel and both first-setter tables): tryInit(10_000, 1e-6) tenants
    (k = 20), keys of 0..90 bytes, adds and contains of the same keys interleaved, 3 chunks."""
    rng = np.random.default_rng(0xC520 + table8)
    from redisson_amd import Arena

    nt = 40
    names = [f"{fresh}-{t}" for t in range(nt)]
    refs, handles = [], []
    for nm in names:
        f = client.getBloomFilter(nm)
        assert f.tryInit(10_000, 1e-6)
        refs.append(O.OracleBloom(f.getSize(), f.getHashIterations()))
        handles.append(BloomHandle(client, nm))
    assert refs[0].k == 20
    n = 60_000
    pool = [rng.bytes(int(x)) for x in rng.integers(0, 91, size=n // 3)]
    keys = [pool[int(i)] for i in rng.integers(0, len(pool), size=n)]
    kf = _zipf_tenants(rng, nt, n)
    op = (rng.random(n) < 0.3).astype(np.uint8)
    assert L.lib().rbx_tune(b"stream_chunk", 20_000) == 0
    assert L.lib().rbx_tune(b"stream_table8", table8) == 0
    try:
        out, counts = bloom_stream(client, handles, kf, op, Arena(keys))
    finally:
        L.lib().rbx_tune(b"stream_chunk", 0)
        L.lib().rbx_tune(b"stream_table8", 1)
    buf, offs = O.arena(keys)
    want, wc = O.bloom_stream(refs, kf, op, buf, offs)
    assert np.array_equal(out, want) and [int(counts[0]), int(counts[1])] == wc
    assert wc[0] > 0 and wc[1] > 0
    for nm, r in zip(names, refs):
        assert client.getBloomFilter(nm).exportBitmap() == r.redis_string(), nm
    for h in handles:
        h.close()
    for nm in names:
        client.getBloomFilter(nm).delete()


def test_c5_production_entry_packing(client, fresh):
    """the bench leg's own 8-byte entry packing, ((fid << bb | bit) << pb) | position
    with bb = 24 (a 14,377,587-bit tenant), fbits = 17 (100,000 filter ids) and pb = 23, and the
    production chunk: min(2^23 - 1, 2^27 / 10) rounded down to 128 = 8,388,480 commands, with no
    stream_chunk override.  9.2M commands = one full chunk + a second one, so positions run to the
    top of the 23-bit field.  99,999 tryInit(1000, 1e-3) tenants (14,377 bits) + one tryInit(1e6,
    1e-3) tenant, all k = 10 (k_stream_*<64, 16>); the big tenant is the Zipf-hottest AND the last
    handle (filter id 99,999 >= 2^16), so its claims fill every field at once.  Replies, counts and
    all 100,000 bitmaps vs the oracle (M/RedissonBloomFilter.java:99-102,198-201)."""
    nt = 100_000
    sizes = [1000] * (nt - 1) + [1_000_000]
    chunk = ((1 << 23) - 1) & ~127
    assert chunk == 8_388_480 and chunk < (1 << 27) // 10
    wc = _c5_case(client, fresh, seed=0xC5B0023, nt=nt, expected=sizes, fpp=1e-3, n=9_200_000, hot_last=True,
                  geometry=(24, 17, 23, chunk))
    assert wc[1] > 100_000
