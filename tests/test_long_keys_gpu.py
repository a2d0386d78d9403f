"""Long keys through every Bloom kernel family on the GPU vs the oracle.

Codec bytes have any length (Hash.hash128 packetizes them: 32-byte packets, then the remainder,
M/misc/Hash.java:53-74 over M/misc/HighwayHash.java:93-285), so keys of many packets and every
remainder length reach the generic hash path (KLEN = 0) of the direct and partitioned contains/add,
the multi-tenant add (per-segment and chunked paths) and contains, and the ordered stream
(M/RedissonBloomFilter.java:104-186).  Keys of up to ~10 KB, including one longer than the host
staging buffer.  Per-key flags, counts and Redis bitmap bytes must equal the oracle's.
"""
import numpy as np
import pytest

from oracle import oracle as O
from redisson_amd import Arena, BloomHandle, bloom_add_multi, bloom_contains_multi, bloom_stream
from redisson_amd import _lib as L

pytestmark = pytest.mark.gpu

# packet and remainder boundaries of the 32-byte HighwayHash packets, and multi-KB keys
LENS = [0, 1, 15, 16, 17, 31, 32, 33, 63, 64, 65, 95, 96, 97, 127, 128, 129, 255, 256, 257, 1000, 1023, 1024,
        1025, 4095, 4096, 4097, 9999]


def _keys(rng, n, maxlen):
    lens = LENS + [int(x) for x in rng.integers(0, maxlen, size=n - len(LENS))]
    pool = [rng.bytes(x) for x in lens]
    # repeats: the same key twice in one batch (shared bits, in-order first setters)
    return pool + [pool[int(j)] for j in rng.integers(0, len(pool), size=n // 8)]


@pytest.mark.parametrize("part", [0, 1])
def test_long_keys_single_filter(client, fresh, part):
    """add() then contains() of long keys on one filter, the partitioned add and contains forced on
    (1) or off (0); a second add re-adds half the keys."""
    rng = np.random.default_rng(0x10C + part)
    keys = _keys(rng, 4000, 2500)
    first, second = keys[: len(keys) // 2], keys[len(keys) // 4:]
    probes = keys + [rng.bytes(int(x)) for x in rng.integers(0, 3000, size=1000)]
    f = client.getBloomFilter(fresh)
    f.tryInitRaw((1 << 26) + 7, 7)
    ref = O.OracleBloom((1 << 26) + 7, 7)
    assert L.lib().rbx_tune(b"add_partition", part) == 0
    assert L.lib().rbx_tune(b"contains_partition", part) == 0
    try:
        for batch in (first, second):
            cg, ng = f.addEach(Arena(batch))
            cr, nr = ref.add(*O.arena(batch), per_key=True)
            assert cg == cr and np.array_equal(ng, nr)
        cg, pg = f.containsEach(Arena(probes))
    finally:
        L.lib().rbx_tune(b"add_partition", 2)
        L.lib().rbx_tune(b"contains_partition", 2)
    cr, pr = ref.contains(*O.arena(probes), per_key=True)
    assert cg == cr and np.array_equal(pg, pr)
    assert f.exportBitmap() == ref.redis_string()
    assert f.count() == ref.count()
    f.delete()


def test_long_keys_host_staging_smaller_than_a_key(client, fresh):
    """Host-arena calls staged through a 4 KiB buffer: a 9,999-byte key is a chunk of its own."""
    rng = np.random.default_rng(0x57A6)
    keys = _keys(rng, 600, 6000)
    f = client.getBloomFilter(fresh)
    f.tryInit(100_000, 0.01)
    ref = O.OracleBloom(f.getSize(), f.getHashIterations())
    assert L.lib().rbx_set_staging(client.ctx, 4096) == 0
    try:
        cg, ng = f.addEach(Arena(keys))
        cc, pc = f.containsEach(Arena(keys[::-1]))
    finally:
        assert L.lib().rbx_set_staging(client.ctx, 64 << 20) == 0
    cr, nr = ref.add(*O.arena(keys), per_key=True)
    assert cg == cr and np.array_equal(ng, nr)
    ccr, pcr = ref.contains(*O.arena(keys[::-1]), per_key=True)
    assert cc == ccr and np.array_equal(pc, pcr)
    assert f.exportBitmap() == ref.redis_string()
    f.delete()


@pytest.mark.parametrize("segment", [1, 0])
def test_long_keys_multi_tenant(client, fresh, segment):
    """add(Collection) per tenant over long keys, one segment per filter (the per-segment kernel, 1)
    or the chunked optimistic path (0), then contains per tenant."""
    rng = np.random.default_rng(0x3A7 + segment)
    nt = 12
    names = [f"{fresh}-{t}" for t in range(nt)]
    refs = []
    for t, nm in enumerate(names):
        m, k = int(rng.integers(5_000, 300_000)), int(rng.integers(3, 17))
        client.getBloomFilter(nm).tryInitRaw(m, k)
        refs.append(O.OracleBloom(m, k))
    handles = [BloomHandle(client, nm) for nm in names]
    keys, segs = [], [0]
    for t in range(nt):
        keys += _keys(rng, 300, 1500)
        segs.append(len(keys))
    segs = np.array(segs, np.uint64)
    assert L.lib().rbx_tune(b"add_multi_segment", segment) == 0
    try:
        counts, flags = bloom_add_multi(client, handles, segs, Arena(keys), per_key=True)
    finally:
        L.lib().rbx_tune(b"add_multi_segment", 1)
    for t in range(nt):
        a, b = int(segs[t]), int(segs[t + 1])
        c, fl = refs[t].add(*O.arena(keys[a:b]), per_key=True)
        assert counts[t] == c and np.array_equal(flags[a:b], fl), t
    pc, pf = bloom_contains_multi(client, handles[::-1], np.concatenate([[0], np.cumsum(np.diff(segs)[::-1])]).astype(
        np.uint64), Arena(sum((keys[int(segs[t]):int(segs[t + 1])] for t in range(nt - 1, -1, -1)), [])), per_key=True)
    pos = 0
    for s, t in enumerate(range(nt - 1, -1, -1)):
        sub = keys[int(segs[t]):int(segs[t + 1])]
        c, fl = refs[t].contains(*O.arena(sub), per_key=True)
        assert pc[s] == c and np.array_equal(pf[pos:pos + len(sub)], fl), t
        pos += len(sub)
    for nm, r in zip(names, refs):
        assert client.getBloomFilter(nm).exportBitmap() == r.redis_string(), nm
    for h in handles:
        h.close()
    for nm in names:
        client.getBloomFilter(nm).delete()


def test_long_keys_ordered_stream(client, fresh):
    """The ordered mixed stream over long keys: adds and contains of the same keys interleaved on
    8 tenants, two chunks."""
    rng = np.random.default_rng(0x57E)
    nt = 8
    names = [f"{fresh}-{t}" for t in range(nt)]
    refs, handles = [], []
    for nm in names:
        f = client.getBloomFilter(nm)
        assert f.tryInit(20_000, 1e-4)
        refs.append(O.OracleBloom(f.getSize(), f.getHashIterations()))
        handles.append(BloomHandle(client, nm))
    pool = _keys(rng, 1200, 3000)
    n = 6000
    keys = [pool[int(i)] for i in rng.integers(0, len(pool), size=n)]
    kf = rng.integers(0, nt, size=n).astype(np.uint32)
    op = (rng.random(n) < 0.4).astype(np.uint8)
    assert L.lib().rbx_tune(b"stream_chunk", 3000) == 0
    try:
        out, counts = bloom_stream(client, handles, kf, op, Arena(keys))
    finally:
        L.lib().rbx_tune(b"stream_chunk", 0)
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


def test_long_elements_hll(client, fresh):
    """PFADD of long elements (MurmurHash64A over many 8-byte blocks and every tail length, [redis-7.2]
    hllPatLen): a sparse HLL (the string as Redis builds it, element by element) and a dense one
    (registers and PFCOUNT)."""
    rng = np.random.default_rng(0x411)
    lens = [0, 1, 7, 8, 9, 15, 16, 17, 63, 64, 65, 1000, 4095, 4096, 4097, 9999]
    few = [rng.bytes(x) for x in lens] + [rng.bytes(int(x)) for x in rng.integers(0, 3000, size=150)]
    ref = O.RedisHll()
    ref.pfadd(*O.arena(few))
    h = client.getHyperLogLog(fresh)
    assert h.addAll(Arena(few)) is True
    s = h.exportString()
    assert s[4] == 1 and s == ref.string(h.exportDense()[8:16])
    assert h.count() == O.hll_count(ref.regs)
    many = few + [rng.bytes(int(x)) for x in rng.integers(0, 2500, size=20000)]
    g = client.getHyperLogLog(fresh + "d")
    assert g.addAll(Arena(many)) is True
    regs = O.hll_new()
    O.hll_pfadd(regs, *O.arena(many))
    d = g.exportDense()
    assert np.array_equal(O.hll_dense_unpack(d[16:]), regs)
    assert g.count() == O.hll_count(regs)
    h.delete()
    g.delete()
