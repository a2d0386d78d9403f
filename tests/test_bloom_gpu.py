"""RBloomFilter on the GPU (librbx.so) vs the CPU oracle: bit-exact parity.

Mirrors T/RedissonBloomFilterTest.java (T/ = redisson/src/test/java/org/redisson/) and adds
per-key parity of contains/add flags, Redis bitmap bytes and count() over many (size, k)
shapes and key layouts (fast 16/32/64-byte path, unaligned and variable-length generic path).
"""
import json
import os

import numpy as np
import pytest

from oracle import oracle as O
from redisson_amd import (Arena, ArithmeticException, BloomHandle, IllegalArgumentException,
                          IllegalStateException, RedisException, bloom_add_multi, bloom_contains_multi)
from redisson_amd import _lib as L

pytestmark = pytest.mark.gpu
G = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "golden.json")))


# ---- T/RedissonBloomFilterTest.java replays ----------------------------------------------
def test_contains_all(client, fresh):
    f = client.getBloomFilter(fresh)
    f.tryInit(100, 0.03)
    lst = ["1", "2", "3"]
    assert f.contains(lst) == 0
    assert f.add(lst) == 3
    assert f.contains(lst) == 3
    assert f.contains(["1", "5"]) == 1


def test_add_all(client, fresh):
    f = client.getBloomFilter(fresh)
    f.tryInit(100, 0.03)
    lst = ["1", "2", "3"]
    assert f.add(lst) == 3
    assert f.add(lst) == 0
    assert f.count() == 3
    assert f.add(["1", "5"]) == 1
    assert f.count() == 4
    for s in lst:
        assert f.contains(s) is True


@pytest.mark.parametrize("n,p", [(1, -1), (1, 2), (1, 1)])
def test_illegal_arguments(client, fresh, n, p):
    with pytest.raises(IllegalArgumentException):
        client.getBloomFilter(fresh).tryInit(n, p)


def test_config(client, fresh):
    f = client.getBloomFilter(fresh)
    f.tryInit(100, 0.03)
    assert f.getExpectedInsertions() == 100
    assert f.getFalseProbability() == 0.03
    assert f.getHashIterations() == 5
    assert f.getSize() == 729


def test_init(client, fresh):
    f = client.getBloomFilter(fresh)
    assert f.tryInit(55000000, 0.03) is True
    assert f.tryInit(55000001, 0.03) is False
    f.delete()
    assert f.isExists() is False
    assert f.tryInit(55000001, 0.03) is True
    f.delete()


@pytest.mark.parametrize("op", ["getExpectedInsertions", "contains", "add"])
def test_not_initialized(client, fresh, op):
    f = client.getBloomFilter(fresh)
    with pytest.raises(IllegalStateException):
        if op == "getExpectedInsertions":
            f.getExpectedInsertions()
        else:
            getattr(f, op)("32")


def test_empty_rename(client, fresh):
    f = client.getBloomFilter(fresh)
    f.tryInit(1000, 0.01)
    f.rename(fresh + "1")
    assert f.isExists()
    assert client.getBloomFilter(fresh).isExists() is False
    f.delete()


def _test_body(f):  # RedissonBloomFilterTest.test(RBloomFilter)
    assert f.contains("123") is False
    assert f.add("123") is True
    assert f.contains("123") is True
    assert f.add("123") is False
    assert f.count() == 1
    assert f.contains("hflgs;jl;ao1-32471320o31803-24") is False
    assert f.add("hflgs;jl;ao1-32471320o31803-24") is True
    assert f.contains("hflgs;jl;ao1-32471320o31803-24") is True
    assert f.count() == 2


def test_large_filters(client, fresh):
    f = client.getBloomFilter(fresh)
    f.tryInit(550000000, 0.5)
    _test_body(f)
    f.delete()
    assert f.tryInit(550000000, 0.03) is True
    _test_body(f)
    f.delete()


def test_rename(client, fresh):
    f = client.getBloomFilter(fresh)
    f.tryInit(550000000, 0.03)
    assert f.add("123") is True
    f.rename(fresh + "new")
    f2 = client.getBloomFilter(fresh + "new")
    assert f2.count() == 1
    assert client.getBloomFilter(fresh).isExists() is False
    f2.delete()


def test_renamenx(client, fresh):
    f = client.getBloomFilter(fresh)
    f.tryInit(550000000, 0.03)
    assert f.add("123") is True
    assert f.contains("123") is True
    f2 = client.getBloomFilter(fresh + "2")
    f2.tryInit(550000000, 0.03)
    assert f2.add("234") is True
    assert f.renamenx(fresh + "2") is False
    assert f.count() == 1
    assert f.renamenx(fresh + "new") is True
    assert client.getBloomFilter(fresh).isExists() is False
    nf = client.getBloomFilter(fresh + "new")
    assert nf.count() == 1
    assert nf.contains("123") is True
    nf.delete()
    f2.delete()


# ---- reference error behaviour ------------------------------------------------------------
def test_empty_collection_arithmetic(client, fresh):
    f = client.getBloomFilter(fresh)
    f.tryInit(100, 0.03)
    with pytest.raises(ArithmeticException):
        f.add([])
    with pytest.raises(ArithmeticException):
        f.contains([])
    f.delete()


def test_config_changed(client, fresh):
    f = client.getBloomFilter(fresh)
    f.tryInit(100, 0.03)
    f.add(["a"])
    other = client.getBloomFilter(fresh)
    other.delete()
    other.tryInit(1000, 0.01)
    with pytest.raises(RedisException, match="config has been changed"):
        f.add(["b"])
    with pytest.raises(RedisException, match="config has been changed"):
        f.contains(["b"])
    other.delete()


def test_wrongtype(client, fresh):
    h = client.getHyperLogLog(fresh)
    h.add("x")
    f = client.getBloomFilter(fresh)
    f.tryInit(100, 0.03)
    with pytest.raises(RedisException, match="WRONGTYPE"):
        f.add(["a"])
    f.delete()


# ---- parity against the oracle -----------------------------------------------------------------
def _oargs(a):
    """oracle (bytes, offsets) for a list of keys or an Arena."""
    if isinstance(a, list):
        return O.arena(a)
    if a.offsets is None:
        stride = a.struct.stride
        return a.bytes, np.arange(a.n + 1, dtype=np.uint64) * np.uint64(stride)
    return a.bytes, a.offsets


def _parity(client, name, size, k, batches, probes):
    f = client.getBloomFilter(name)
    assert f.tryInitRaw(size, k)
    ref = O.OracleBloom(size, k)
    for b in batches:
        cg, ng = f.addEach(Arena(b) if isinstance(b, list) else b)
        cr, nr = ref.add(*_oargs(b), per_key=True)
        assert cg == cr
        assert np.array_equal(ng, nr)
    for p in probes:
        cg, pg = f.containsEach(Arena(p) if isinstance(p, list) else p)
        cr, pr = ref.contains(*_oargs(p), per_key=True)
        assert cg == cr
        assert np.array_equal(pg, pr)
    assert f.exportBitmap() == ref.redis_string()
    assert f.bitcount() == ref.bitcount()
    f.delete()


SHAPES = [(729, 5), (64, 7), (9585, 7), (95850583, 7), (14377587, 10), (1 << 20, 7), (1000003, 1),
          (100003, 17), (100003, 33), (50021, 40), (4294967293, 7), (1 << 32, 7), (3, 3), (1, 4)]


@pytest.mark.parametrize("size,k", SHAPES)
def test_parity_variable_length(client, fresh, size, k):
    rng = np.random.default_rng(size * 31 + k)
    base = [rng.bytes(int(L)) for L in rng.integers(0, 100, size=3000)]
    batches = [[base[int(j)] for j in rng.integers(0, len(base), size=2000)] for _ in range(3)]
    probes = [base[:1500] + [rng.bytes(int(L)) for L in rng.integers(0, 100, size=1500)]]
    _parity(client, fresh, size, k, batches, probes)


@pytest.mark.parametrize("L", [16, 32, 64, 24, 48, 8])
@pytest.mark.parametrize("size,k", [(95850583, 7), (14377587, 10), (1 << 32, 7), (1000, 40)])
def test_parity_fixed_length(client, fresh, L, size, k):
    rng = np.random.default_rng(L * 1000 + k)
    mat = rng.integers(0, 256, size=(20000, L), dtype=np.uint8)
    mat[5000:5100] = mat[0:100]  # duplicates inside the batch
    a1 = Arena.fixed(mat[:12000])
    a2 = Arena.fixed(mat[8000:])
    probe = Arena.fixed(np.concatenate([mat[:3000], rng.integers(0, 256, size=(3000, L), dtype=np.uint8)]))
    _parity(client, fresh, size, k, [a1, a2], [probe])


def test_parity_unaligned_device_keys(client, fresh):
    """32-byte keys at an odd device address (generic unaligned path) and variable-length
    keys through the device offsets arena."""
    import torch

    from redisson_amd import device_keys

    rng = np.random.default_rng(77)
    n = 4000
    raw = rng.integers(0, 256, size=(1 + n * 32), dtype=np.uint8)
    mat = np.ascontiguousarray(raw[1:].reshape(n, 32))
    d = torch.from_numpy(raw).cuda()
    f = client.getBloomFilter(fresh)
    f.tryInitRaw(95850583, 7)
    h = BloomHandle(client, fresh)
    out = torch.zeros(n, dtype=torch.uint8, device="cuda")
    cnt = torch.zeros(2, dtype=torch.int64, device="cuda")
    h.add_dev(device_keys(d.data_ptr() + 1, n, 32), cnt.data_ptr(), out.data_ptr())
    client.synchronize()
    ref = O.OracleBloom(95850583, 7)
    cr, nr = ref.add(*O.fixed_arena(mat), per_key=True)
    assert cnt[0].item() == cr and np.array_equal(out.cpu().numpy(), nr)
    # variable-length keys through device offsets
    keys = [rng.bytes(int(L)) for L in rng.integers(0, 90, size=n)]
    b, o = O.arena(keys)
    db = torch.from_numpy(np.concatenate([np.zeros(3, np.uint8), b])).cuda()
    do = torch.from_numpy((o + 3).astype(np.int64)).cuda()
    h.contains_dev(device_keys(db.data_ptr(), n, 0, do.data_ptr()), cnt.data_ptr() + 8, out.data_ptr())
    client.synchronize()
    cr, pr = ref.contains(b, o, per_key=True)
    assert cnt[1].item() == cr and np.array_equal(out.cpu().numpy(), pr)
    h.close()
    f.delete()


def test_golden_sequences_on_gpu(client, fresh):
    for i, s in enumerate(G["bloom_sequences"]):
        f = client.getBloomFilter(f"{fresh}-{i}")
        f.tryInitRaw(s["size"], s["k"])
        for b in s["batches"]:
            c, flags = f.addEach([bytes.fromhex(x) for x in b["keys"]])
            assert c == b["count"] and flags.tolist() == b["new"]
        c, pres = f.containsEach([bytes.fromhex(x) for x in s["probes"]])
        assert c == s["contains"] and pres.tolist() == s["present"]
        assert f.exportBitmap().hex() == s["bitmap"]
        assert f.count() == s["count"]
        f.delete()


def test_export_import_roundtrip(client, fresh):
    rng = np.random.default_rng(11)
    keys = [rng.bytes(20) for _ in range(5000)]
    f = client.getBloomFilter(fresh)
    f.tryInit(10000, 0.01)
    f.add(keys)
    blob = f.exportBitmap()
    g = client.getBloomFilter(fresh + "b")
    g.tryInit(10000, 0.01)
    g.importBitmap(blob)
    assert g.contains(keys) == len(keys)
    assert g.exportBitmap() == blob
    assert g.count() == f.count()
    f.delete()
    g.delete()


@pytest.mark.parametrize("order", [[0, 1, 2, 3, 4, 5, 6, 3, 0], [6, 5, 3, 2, 1, 0]])
@pytest.mark.parametrize("small", [2, 1, 0])
def test_multi_tenant_parity(client, fresh, small, order):
    """Multi-tenant add/contains from a host arena (segments in order; a tenant repeated, or every filter
    once with k <= 16: the per-segment add), per key vs the oracle; small 2: keys, segment offsets and
    flags in coherent pinned memory (r06 tiny path, counts from the flags), 1: the one-transfer staging
    (counts, segment offsets and keys in one upload), 0: the separate uploads."""
    rng = np.random.default_rng(12)
    assert L.lib().rbx_tune(b"host_small_batches", min(small, 1)) == 0
    assert L.lib().rbx_tune(b"host_tiny_keys", 16384 if small == 2 else 0) == 0
    names = [f"{fresh}-{t}" for t in range(7)]
    shapes = [(14377587, 10), (729, 5), (9585, 7), (64, 7), (1000, 40), (1 << 20, 3), (100003, 17)]
    refs = []
    for n, (m, k) in zip(names, shapes):
        client.getBloomFilter(n).tryInitRaw(m, k)
        refs.append(O.OracleBloom(m, k))
    handles = [BloomHandle(client, n) for n in names]
    # segments: tenant order with a repeated tenant (sequential semantics across segments)
    sizes = [int(x) for x in rng.integers(1, 400, size=len(order))]
    keys, segs = [], [0]
    for t, sz in zip(order, sizes):
        pool = [rng.bytes(int(L)) for L in rng.integers(0, 40, size=sz // 2 + 1)]
        keys += [pool[int(j)] for j in rng.integers(0, len(pool), size=sz)]
        segs.append(len(keys))
    segs = np.array(segs, np.uint64)
    counts, flags = bloom_add_multi(client, [handles[t] for t in order], segs, Arena(keys), per_key=True)
    for s, t in enumerate(order):
        sub = keys[int(segs[s]):int(segs[s + 1])]
        c, fl = refs[t].add(*O.arena(sub), per_key=True)
        assert counts[s] == c
        assert np.array_equal(flags[int(segs[s]):int(segs[s + 1])], fl)
    probes_c, probes_f = bloom_contains_multi(client, [handles[t] for t in order], segs, Arena(keys), per_key=True)
    L.lib().rbx_tune(b"host_small_batches", 1)
    L.lib().rbx_tune(b"host_tiny_keys", 16384)
    for s, t in enumerate(order):
        sub = keys[int(segs[s]):int(segs[s + 1])]
        c, fl = refs[t].contains(*O.arena(sub), per_key=True)
        assert probes_c[s] == c and np.array_equal(probes_f[int(segs[s]):int(segs[s + 1])], fl)
    for n, r in zip(names, refs):
        assert client.getBloomFilter(n).exportBitmap() == r.redis_string()
    for h in handles:
        h.close()
    for n in names:
        client.getBloomFilter(n).delete()


@pytest.mark.parametrize("table8,clog2", [(2, 17), (2, 6), (0, 17)])
@pytest.mark.parametrize("chunk", [0, 700])
def test_multi_tenant_add_first_setter_tables(client, fresh, table8, clog2, chunk):
    """r05: multi-tenant add(Collection) by optimistic SETBITs with conflict repair (add_multi_table8 2,
    default; a 64-entry conflict table (clog2 6) overflows and the chunk falls back to the full
    first-setter table), on the 8-byte first-setter table (1: one CAS per zero bit, replies from the
    first claim's slot, walk commit) and on the r03 16-byte table (0).  Shapes with k up to 17 (KMAX
    32), variable-length keys (KLEN 0), repeated tenants and keys repeated inside and across segments
    (shared zero bits); chunk 700 runs the chunked paths in many chunks (the in-order fold across
    chunk boundaries)."""
    rng = np.random.default_rng(1200 + table8 + chunk + clog2)
    names = [f"{fresh}-{t}" for t in range(6)]
    shapes = [(14377587, 10), (729, 5), (9585, 7), (64, 7), (1 << 20, 3), (100003, 17)]
    refs = []
    for n, (m, k) in zip(names, shapes):
        client.getBloomFilter(n).tryInitRaw(m, k)
        refs.append(O.OracleBloom(m, k))
    handles = [BloomHandle(client, n) for n in names]
    order = [0, 1, 2, 3, 4, 5, 3, 0, 2, 2]
    sizes = [int(x) for x in rng.integers(1, 600, size=len(order))]
    shared = [rng.bytes(int(L)) for L in rng.integers(0, 40, size=50)]
    keys, segs = [], [0]
    for t, sz in zip(order, sizes):
        pool = [rng.bytes(int(L)) for L in rng.integers(0, 40, size=sz // 2 + 1)] + shared
        keys += [pool[int(j)] for j in rng.integers(0, len(pool), size=sz)]
        segs.append(len(keys))
    segs = np.array(segs, np.uint64)
    assert L.lib().rbx_tune(b"add_multi_table8", table8) == 0
    assert L.lib().rbx_tune(b"add_multi_conflict_log2", clog2) == 0
    assert L.lib().rbx_tune(b"stream_chunk", chunk) == 0
    try:
        counts, flags = bloom_add_multi(client, [handles[t] for t in order], segs, Arena(keys), per_key=True)
    finally:
        L.lib().rbx_tune(b"add_multi_table8", ADD_MULTI_DEFAULT)
        L.lib().rbx_tune(b"add_multi_conflict_log2", 17)
        L.lib().rbx_tune(b"stream_chunk", 0)
    for s, t in enumerate(order):
        sub = keys[int(segs[s]):int(segs[s + 1])]
        c, fl = refs[t].add(*O.arena(sub), per_key=True)
        assert counts[s] == c, s
        assert np.array_equal(flags[int(segs[s]):int(segs[s + 1])], fl), s
    for n, r in zip(names, refs):
        assert client.getBloomFilter(n).exportBitmap() == r.redis_string()
    for h in handles:
        h.close()
    for n in names:
        client.getBloomFilter(n).delete()


ADD_MULTI_DEFAULT = 2
ADD_MULTI_SEG_GRID_DEFAULT = 8192


@pytest.mark.parametrize("segmax,grid", [(16384, 8192), (300, 8192), (1, 8192), (16384, 64)])
@pytest.mark.parametrize("fixed", [True, False])
def test_multi_tenant_add_one_segment_per_filter(client, fresh, segmax, grid, fixed):
    """A multi-tenant add whose filters are all distinct runs one workgroup per segment (k_madd_seg: tiles
    of <= 256 keys in order, LDS first setters, plain word stores, the next tile's hash before the store
    wait); segments longer than add_multi_segmax keys go to the chunked path in the same call (segmax
    300: both paths; 1: every non-trivial segment chunked); grid 64: workgroups walk many segments.
    40 filters with k = 3..16 (KMAX 8 and 16; tiles of 160..256 keys), 1..1,500 keys per segment, keys
    repeated within a segment and across tile boundaries (shared zero bits), fixed 16-byte or
    variable-length keys.  Per-key flags, per-segment counts and every bitmap vs the oracle; then the
    same batch again (every key already present)."""
    rng = np.random.default_rng(1300 + segmax + grid + int(fixed))
    nt = 40
    names = [f"{fresh}-{t}" for t in range(nt)]
    refs = []
    for t, n in enumerate(names):
        m, k = int(rng.integers(2_000, 400_000)), int(rng.integers(3, 17))
        client.getBloomFilter(n).tryInitRaw(m, k)
        refs.append(O.OracleBloom(m, k))
    handles = [BloomHandle(client, n) for n in names]
    sizes = [int(x) for x in rng.integers(1, 1500, size=nt)]  # (an empty add is an error: "/ by zero")
    sizes[3] = 1
    segs = np.zeros(nt + 1, np.uint64)
    segs[1:] = np.cumsum(sizes)
    n = int(segs[-1])
    if fixed:
        pool = rng.integers(0, 256, size=(max(1, n // 3), 16), dtype=np.uint8)
        mat = pool[rng.integers(0, len(pool), size=n)]
        keys, arena, sub = mat, Arena.fixed(mat), (lambda a, b: O.fixed_arena(mat[a:b]))
    else:
        pool = [rng.bytes(int(L)) for L in rng.integers(0, 40, size=max(1, n // 3))]
        keys = [pool[int(j)] for j in rng.integers(0, len(pool), size=n)]
        arena, sub = Arena(keys), (lambda a, b: O.arena(keys[a:b]))
    assert L.lib().rbx_tune(b"add_multi_segmax", segmax) == 0
    assert L.lib().rbx_tune(b"add_multi_seg_grid", grid) == 0
    try:
        for rep in range(2):
            counts, flags = bloom_add_multi(client, handles, segs, arena, per_key=True)
            for t in range(nt):
                a, b = int(segs[t]), int(segs[t + 1])
                c, fl = refs[t].add(*sub(a, b), per_key=True)
                assert counts[t] == c and np.array_equal(flags[a:b], fl), (rep, t, sizes[t])
            if rep == 0:
                assert int(counts.sum()) > n // 4
    finally:
        L.lib().rbx_tune(b"add_multi_segmax", 16384)
        L.lib().rbx_tune(b"add_multi_seg_grid", ADD_MULTI_SEG_GRID_DEFAULT)
    for nm, r in zip(names, refs):
        assert client.getBloomFilter(nm).exportBitmap() == r.redis_string(), nm
    for h in handles:
        h.close()
    for nm in names:
        client.getBloomFilter(nm).delete()


@pytest.mark.parametrize("fill", [0.5, 0.0])
def test_multi_tenant_add_segment_tile_boundaries(client, fresh, fill):
    """k = 10 (tryInit(1e6, 1e-3): 14,377,587 bits) tenants whose segments hold
    exactly 1, 255, 256, 257, 511, 512, 513, 1024, 1025 and 16,384 keys (the per-segment kernel's tile
    is 256 keys at k = 10; 16,384 = add_multi_segmax, the longest segment it takes), fresh 16-byte keys
    plus repeats of keys from earlier tiles of the same segment.  fill 0.5: bitmaps at design fill (~5
    zero bits per key); fill 0: empty bitmaps (10 zero bits per key: the LDS tables at their 0.625 load
    bound).  Per-key flags, counts and every bitmap vs the oracle (M/RedissonBloomFilter.java:104-137)."""
    import torch

    rng = np.random.default_rng(0x5E6B + int(fill * 10))
    sizes = [1, 255, 256, 257, 511, 512, 513, 1024, 1025, 16384]
    names = [f"{fresh}:{t}" for t in range(len(sizes))]
    nb = (14_377_587 + 7) // 8
    refs, handles = [], []
    try:
        for nm in names:
            f = client.getBloomFilter(nm)
            assert f.tryInit(1_000_000, 1e-3)
            r = O.OracleBloom(14_377_587, 10)
            if fill:
                bm = rng.integers(0, 256, size=nb, dtype=np.uint8)
                d = torch.from_numpy(bm).cuda()
                assert L.lib().rbx_bloom_import_dev(client.ctx, nm.encode(), d.data_ptr(), nb, None) == 0
                torch.cuda.synchronize()
                del d
                r.bitmap[:nb] = bm
                r.redis_len = nb
            refs.append(r)
            handles.append(BloomHandle(client, nm))
        segs = np.zeros(len(sizes) + 1, np.uint64)
        segs[1:] = np.cumsum(sizes)
        n = int(segs[-1])
        keys = rng.integers(0, 256, size=(n, 16), dtype=np.uint8)
        for t, sz in enumerate(sizes):  # repeats: a key of an earlier round again (and one inside a round)
            a = int(segs[t])
            for p in range(1, sz, 97):
                keys[a + p] = keys[a + int(rng.integers(0, p))]
        counts, flags = bloom_add_multi(client, handles, segs, Arena.fixed(keys), per_key=True)
        for t in range(len(sizes)):
            a, b = int(segs[t]), int(segs[t + 1])
            c, fl = refs[t].add(*O.fixed_arena(keys[a:b]), per_key=True)
            assert counts[t] == c and np.array_equal(flags[a:b], fl), (t, sizes[t])
        for nm, r in zip(names, refs):
            assert client.getBloomFilter(nm).exportBitmap() == r.redis_string(), nm
    finally:
        for h in handles:
            h.close()
        for nm in names:
            client.getBloomFilter(nm).delete()


@pytest.mark.parametrize("segment", [1, 0])
def test_multi_tenant_add_segment_path_at_c3_shape(client, fresh, segment):
    """The bench's C3 add shape at 20,000 tenants (tryInit(1e6, 1e-3): 14,377,587 bits, k = 10) at design
    fill: one add_multi of 1,000 fresh 16-byte keys per tenant, on the per-segment path (1) and on the
    chunked optimistic path (0); per-key flags and counts vs the oracle for 300 sampled tenants, every
    count checked against the flags."""
    import torch

    nt, per = 20_000, 1000
    rng = np.random.default_rng(0xC3ADD + segment)
    pool = rng.integers(0, 256, size=16 << 20, dtype=np.uint8)
    dpool = torch.from_numpy(pool).cuda()
    names = [f"{fresh}:{t:05d}" for t in range(nt)]
    offs = np.zeros(nt, np.int64)
    handles = []
    nb = (14_377_587 + 7) // 8
    try:
        for t, nm in enumerate(names):
            assert client.getBloomFilter(nm).tryInit(1_000_000, 1e-3)
            offs[t] = int(rng.integers(0, (pool.size - nb) // 256)) * 256
            assert L.lib().rbx_bloom_import_dev(client.ctx, nm.encode(), dpool.data_ptr() + int(offs[t]), nb,
                                                None) == 0
            handles.append(BloomHandle(client, nm))
        keys = rng.integers(0, 256, size=(nt * per, 16), dtype=np.uint8)
        seg = np.arange(nt + 1, dtype=np.uint64) * np.uint64(per)
        assert L.lib().rbx_tune(b"add_multi_segment", segment) == 0
        try:
            counts, flags = bloom_add_multi(client, handles, seg, Arena.fixed(keys), per_key=True)
        finally:
            L.lib().rbx_tune(b"add_multi_segment", 1)
        sample = rng.choice(nt, size=300, replace=False)
        for t in sample:
            t = int(t)
            r = O.OracleBloom(14_377_587, 10)
            r.bitmap[:nb] = pool[offs[t]:offs[t] + nb]
            r.redis_len = nb
            c, fl = r.add(*O.fixed_arena(keys[t * per:(t + 1) * per]), per_key=True)
            assert counts[t] == c and np.array_equal(flags[t * per:(t + 1) * per], fl), t
            assert client.getBloomFilter(names[t]).exportBitmap() == r.redis_string(), t
        assert int(counts.sum()) == int(flags.sum()) and int(counts.sum()) > nt * per * 0.99
    finally:
        for h in handles:
            h.close()
        for nm in names:
            client.getBloomFilter(nm).delete()
        del dpool
        torch.cuda.empty_cache()


@pytest.mark.parametrize("table8", [2, 0])
def test_multi_tenant_add_filter_ids_past_2_17(client, fresh, table8):
    """per-key add parity of a multi-tenant add batch whose filter ids reach 2^17:
    100,000 tryInit(1000, 1e-3) tenants (14,377 bits, k = 10) at design fill, one add_multi batch of
    ~24 16-byte keys per tenant (a tenant's keys repeat, so shared bits occur), every tenant once in
    tenant order except the last 1,000 segments, which revisit earlier tenants.  Per-key flags,
    per-segment counts and all 100,000 bitmaps vs the oracle (M/RedissonBloomFilter.java:104-137)."""
    nt = 100_000
    rng = np.random.default_rng(0xADD17 + table8)
    names = [f"{fresh}:{t:06d}" for t in range(nt)]
    refs, handles = [], []
    try:
        for nm in names:
            f = client.getBloomFilter(nm)
            assert f.tryInit(1000, 1e-3)
            nb = (f.getSize() + 7) // 8
            bm = rng.integers(0, 256, size=nb, dtype=np.uint8)
            f.importBitmap(bm.tobytes())
            r = O.OracleBloom(f.getSize(), f.getHashIterations())
            r.bitmap[:nb] = bm
            r.redis_len = nb
            refs.append(r)
            handles.append(BloomHandle(client, nm))
        assert (refs[0].size, refs[0].k) == (14_377, 10)
        order = list(range(nt)) + [int(x) for x in rng.integers(0, nt, size=1000)]
        sizes = rng.integers(1, 48, size=len(order))
        segs = np.zeros(len(order) + 1, np.uint64)
        segs[1:] = np.cumsum(sizes)
        n = int(segs[-1])
        pool = rng.integers(0, 256, size=(n // 2, 16), dtype=np.uint8)
        keys = pool[rng.integers(0, len(pool), size=n)]
        # and a key added to one tenant twice in one segment, for a few thousand segments
        for s in range(0, len(order), 37):
            a, b = int(segs[s]), int(segs[s + 1])
            if b - a >= 2:
                keys[b - 1] = keys[a]
        assert L.lib().rbx_tune(b"add_multi_table8", table8) == 0
        try:
            counts, flags = bloom_add_multi(client, [handles[t] for t in order], segs, Arena.fixed(keys),
                                            per_key=True)
        finally:
            L.lib().rbx_tune(b"add_multi_table8", ADD_MULTI_DEFAULT)
        for s, t in enumerate(order):
            a, b = int(segs[s]), int(segs[s + 1])
            c, fl = refs[t].add(*O.fixed_arena(keys[a:b]), per_key=True)
            assert counts[s] == c and np.array_equal(flags[a:b], fl), (s, t)
        assert int(counts.sum()) > n // 2
        for nm, r in zip(names, refs):
            assert client.getBloomFilter(nm).exportBitmap() == r.redis_string(), nm
    finally:
        for h in handles:
            h.close()
        for nm in names:
            client.getBloomFilter(nm).delete()


def test_device_path_matches_host_path(client, fresh):
    import torch

    rng = np.random.default_rng(13)
    mat = rng.integers(0, 256, size=(100000, 32), dtype=np.uint8)
    f = client.getBloomFilter(fresh)
    f.tryInitRaw(1 << 24, 7)
    h = BloomHandle(client, fresh)
    d = torch.from_numpy(mat).cuda()
    cnt = torch.zeros(2, dtype=torch.int64, device="cuda")
    from redisson_amd import device_keys

    dk = device_keys(d.data_ptr(), 50000, 32)
    h.add_dev(dk, cnt.data_ptr(), stream=torch.cuda.current_stream().cuda_stream)
    dk2 = device_keys(d.data_ptr(), 100000, 32)
    h.contains_dev(dk2, cnt.data_ptr() + 8, stream=torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    ref = O.OracleBloom(1 << 24, 7)
    ca = ref.add(*O.fixed_arena(mat[:50000]))
    cc = ref.contains(*O.fixed_arena(mat))
    assert cnt.tolist() == [ca, cc]
    h.close()
    f.delete()


def test_full_size_2pow32_property(client, fresh):
    """C2 geometry (m = 2^32, k = 7) at 4.2M 32-byte keys (above the 2^22-key threshold of the
    default partitioned contains): add counts and per-key flags equal the oracle, no false
    negatives, false-positive rate near theory, per-key contains flags of fresh keys equal the
    oracle's, bitmap bytes identical."""
    rng = np.random.default_rng(0x5EED0002)
    n = 4_200_000
    mat = rng.integers(0, 256, size=(n, 32), dtype=np.uint8)
    f = client.getBloomFilter(fresh)
    f.tryInitRaw(1 << 32, 7)
    ref = O.OracleBloom(1 << 32, 7)
    a = Arena.fixed(mat)
    cg, ng = f.addEach(a)
    cr, nr = ref.add(*O.fixed_arena(mat), per_key=True)
    assert cg == cr == n and np.array_equal(ng, nr)
    assert f.contains(a) == n
    fmat = rng.integers(0, 256, size=(n, 32), dtype=np.uint8)
    fp, pg = f.containsEach(Arena.fixed(fmat))
    theory = (1 - np.exp(-7 * n / 2**32)) ** 7
    assert fp <= max(10, 5 * theory * n)
    cr, pr = ref.contains(*O.fixed_arena(fmat), per_key=True)
    assert fp == cr and np.array_equal(pg, pr)
    assert f.exportBitmap() == ref.redis_string()
    f.delete()


def test_partitioned_contains_miss_record_overflow(client, fresh):
    """A half-full filter with k = 16 probed by absent keys: ~3.75 clear bits per key, so the
    probe's per-region LDS record list (4096) and the per-range record capacity (2 per key)
    both overflow into the direct atomicOr path.  Per-key answers equal the oracle's."""
    from redisson_amd import _lib as L_

    rng = np.random.default_rng(31)
    size, k = 1 << 27, 16
    blob = rng.integers(0, 256, size=size // 8, dtype=np.uint8)
    f = client.getBloomFilter(fresh)
    f.tryInitRaw(size, k)
    f.importBitmap(blob.tobytes())
    ref = O.OracleBloom(size, k)
    ref.bitmap[: size // 8] = blob
    ref.redis_len = size // 8
    probe = rng.integers(0, 256, size=(1_500_000, 16), dtype=np.uint8)
    assert L_.lib().rbx_tune(b"contains_partition", 1) == 0
    try:
        cg, pg = f.containsEach(Arena.fixed(probe))
    finally:
        L_.lib().rbx_tune(b"contains_partition", 2)
    cr, pr = ref.contains(*O.fixed_arena(probe), per_key=True)
    assert cg == cr and np.array_equal(pg, pr)
    f.delete()


def test_partitioned_contains_bucket_overflow(client, fresh):
    """Batches that overflow the partitioned path's fixed bucket capacities (a few keys repeated
    hundreds of thousands of times put all pairs into k-1 buckets): the overflowing pairs are
    probed directly and every per-key answer still equals the oracle's."""
    from redisson_amd import _lib as L_

    rng = np.random.default_rng(77)
    base = rng.integers(0, 256, size=(40, 32), dtype=np.uint8)
    f = client.getBloomFilter(fresh)
    f.tryInitRaw(1 << 30, 7)
    ref = O.OracleBloom(1 << 30, 7)
    f.add(Arena.fixed(base[:20]))
    ref.add(*O.fixed_arena(base[:20]))
    probe = np.concatenate([base[rng.integers(0, 40, size=400_000)], rng.integers(0, 256, size=(50_000, 32),
                                                                                 dtype=np.uint8)])
    assert L_.lib().rbx_tune(b"contains_partition", 1) == 0
    try:
        cg, pg = f.containsEach(Arena.fixed(probe))
    finally:
        L_.lib().rbx_tune(b"contains_partition", 2)
    cr, pr = ref.contains(*O.fixed_arena(probe), per_key=True)
    assert cg == cr and np.array_equal(pg, pr)
    f.delete()


def test_import_dev_many_tenants_parity(client, fresh):
    """Slab-allocated tenant bitmaps loaded from a device buffer (SET from device memory),
    then one multi-tenant contains batch checked per key against the oracle."""
    import torch

    rng = np.random.default_rng(21)
    nt = 300
    names = [f"{fresh}-{i}" for i in range(nt)]
    pool = rng.integers(0, 256, size=(1 << 22), dtype=np.uint8)
    dpool = torch.from_numpy(pool).cuda()
    refs = []
    from redisson_amd import _lib as L

    for i, nm in enumerate(names):
        f = client.getBloomFilter(nm)
        f.tryInit(10000, 0.01)
        nb = (f.getSize() + 7) // 8
        off = int(rng.integers(0, (pool.size - nb) // 256)) * 256
        assert L.lib().rbx_bloom_import_dev(client.ctx, nm.encode(), dpool.data_ptr() + off, nb, None) == 0
        r = O.OracleBloom(f.getSize(), f.getHashIterations())
        r.bitmap[:nb] = pool[off:off + nb]
        r.redis_len = nb
        refs.append(r)
        if i % 50 == 0:
            assert f.exportBitmap() == pool[off:off + nb].tobytes()
    handles = [BloomHandle(client, nm) for nm in names]
    per = [int(x) for x in rng.integers(1, 60, size=nt)]
    keys, segs = [], [0]
    for p in per:
        keys += [rng.bytes(16) for _ in range(p)]
        segs.append(len(keys))
    segs = np.array(segs, np.uint64)
    counts, flags = bloom_contains_multi(client, handles, segs, Arena(keys), per_key=True)
    for s in range(nt):
        sub = keys[int(segs[s]):int(segs[s + 1])]
        c, fl = refs[s].contains(*O.arena(sub), per_key=True)
        assert counts[s] == c and np.array_equal(flags[int(segs[s]):int(segs[s + 1])], fl)
    for h in handles:
        h.close()
    for nm in names:  # free-list reuse afterwards
        client.getBloomFilter(nm).delete()
    f = client.getBloomFilter(fresh + "again")
    f.tryInit(10000, 0.01)
    assert f.add(["x", "y"]) == 2 and f.contains(["x", "y", "z"]) >= 2
    f.delete()


@pytest.mark.parametrize("sched", [0, 1, 2, 3, 4, 5])
def test_contains_schedules_identical(client, fresh, sched):
    """Every early-exit schedule returns exactly the oracle's per-key answers."""
    from redisson_amd import _lib as L

    rng = np.random.default_rng(31)
    for size, k in [(14377587, 10), (95850583, 7), (4099, 7), (100003, 13)]:
        mat = rng.integers(0, 256, size=(60000, 16), dtype=np.uint8)
        f = client.getBloomFilter(f"{fresh}-{size}")
        f.tryInitRaw(size, k)
        ref = O.OracleBloom(size, k)
        f.add(Arena.fixed(mat[:30000]))
        ref.add(*O.fixed_arena(mat[:30000]))
        assert L.lib().rbx_tune(b"contains_stage1", sched) == 0
        try:
            cg, pg = f.containsEach(Arena.fixed(mat))
        finally:
            L.lib().rbx_tune(b"contains_stage1", 4)
        cr, pr = ref.contains(*O.fixed_arena(mat), per_key=True)
        assert cg == cr and np.array_equal(pg, pr)
        f.delete()


@pytest.mark.parametrize("sched", [4, 5])
@pytest.mark.parametrize("varlen", [False, True])
def test_contains_multi_schedules_identical(client, fresh, sched, varlen):
    """Multi-tenant contains under the staged (4) and per-lane slot (5) kernels: per-key flags and
    per-tenant counts equal the oracle's, with 1-key, sub-range and multi-range tenant segments."""
    from redisson_amd import _lib as L
    from redisson_amd import BloomHandle, bloom_contains_multi

    rng = np.random.default_rng(77 + varlen)
    shapes = [(14377587, 10), (729, 5), (100003, 17), (4099, 1), (95850583, 7)]
    seg_lens = [1, 300, 5000, 129, 128, 2, 70000, 1, 257, 3]  # an empty one raises "/ by zero" (:121)
    names, refs, handles = [], [], []
    for i in range(len(seg_lens)):
        size, k = shapes[i % len(shapes)]
        nm = f"{fresh}-{i}"
        f = client.getBloomFilter(nm)
        f.tryInitRaw(size, k)
        ref = O.OracleBloom(size, k)
        add = [rng.bytes(int(rng.integers(0, 40)) if varlen else 16) for _ in range(2000)]
        f.add(Arena(add))
        ref.add(*O.arena(add))
        names.append(nm)
        refs.append((ref, add))
        handles.append(BloomHandle(client, nm))
    keys, segs = [], [0]
    for i, n in enumerate(seg_lens):
        add = refs[i][1]
        for _ in range(n):  # half present, half random
            keys.append(add[int(rng.integers(0, len(add)))] if rng.random() < 0.5 else
                        rng.bytes(int(rng.integers(0, 40)) if varlen else 16))
        segs.append(len(keys))
    segs = np.array(segs, np.uint64)
    assert L.lib().rbx_tune(b"contains_stage1", sched) == 0
    try:
        arena = Arena(keys) if varlen else Arena.fixed(np.frombuffer(b"".join(keys), np.uint8).reshape(-1, 16))
        counts, flags = bloom_contains_multi(client, handles, segs, arena, per_key=True)
    finally:
        L.lib().rbx_tune(b"contains_stage1", 4)
    for s in range(len(seg_lens)):
        sub = keys[int(segs[s]):int(segs[s + 1])]
        c, fl = refs[s][0].contains(*O.arena(sub), per_key=True) if sub else (0, np.zeros(0, np.uint8))
        assert counts[s] == c and np.array_equal(flags[int(segs[s]):int(segs[s + 1])], fl)
    for h in handles:
        h.close()
    for nm in names:
        client.getBloomFilter(nm).delete()


@pytest.mark.parametrize("seed", [1, 2])
def test_mixed_stream_in_order_semantics(client, fresh, seed):
    """C5 shape: an ordered stream of single-key contains/add commands over tenants with a
    skewed tenant choice; every answer equals the one-after-another oracle replay, including
    contains right after an add of the same key and adds racing on shared bits."""
    _stream_case(client, fresh, seed)


def _stream_case(client, fresh, seed):
    from redisson_amd import bloom_stream

    rng = np.random.default_rng(seed)
    shapes = [(64, 7), (729, 5), (9585, 7), (14377587, 10), (100003, 17)]
    names = [f"{fresh}-{i}" for i in range(len(shapes))]
    refs = []
    for n, (m, k) in zip(names, shapes):
        client.getBloomFilter(n).tryInitRaw(m, k)
        refs.append(O.OracleBloom(m, k))
    handles = [BloomHandle(client, n) for n in names]
    handles.append(handles[1])  # the same filter under a second index
    alias = {len(shapes): 1}
    nkeys = 6000
    pool = [rng.bytes(int(L)) for L in rng.integers(0, 40, size=800)]
    kf = np.minimum(rng.zipf(1.3, size=nkeys) - 1, len(handles) - 1).astype(np.uint32)
    op = (rng.random(nkeys) < 0.3).astype(np.uint8)
    keys = [pool[int(j)] for j in rng.integers(0, len(pool), size=nkeys)]
    for i in range(0, nkeys, 97):  # contains of a key right after its add
        if i + 1 < nkeys:
            op[i], op[i + 1] = 1, 0
            kf[i + 1] = kf[i]
            keys[i + 1] = keys[i]
    out, counts = bloom_stream(client, handles, kf, op, Arena(keys))
    want = np.zeros(nkeys, np.uint8)
    for i in range(nkeys):
        r = refs[alias.get(int(kf[i]), int(kf[i]))]
        b, o = O.arena([keys[i]])
        want[i] = r.add(b, o) if op[i] else r.contains(b, o)
    assert np.array_equal(out, want)
    assert counts[0] == int(want[op == 0].sum()) and counts[1] == int(want[op == 1].sum())
    for n, r in zip(names, refs):
        assert client.getBloomFilter(n).exportBitmap() == r.redis_string()
    for h in handles[:-1]:
        h.close()
    for n in names:
        client.getBloomFilter(n).delete()


def test_mixed_stream_multi_chunk(client, fresh):
    """A 5M-command stream with k = 32 (chunks of 2^26 / 32 = 2M commands, so three chunks and a
    multi-block add compaction in each): runs of adds and contains on two filters, replayed on
    the oracle run by run (filters are independent, and a run of one command type on one filter
    is exactly one ordered batch)."""
    from redisson_amd import bloom_stream

    rng = np.random.default_rng(5)
    shapes = [(50_000_017, 32), (1_000_003, 20)]
    names = [f"{fresh}-{i}" for i in range(len(shapes))]
    refs = []
    for nm, (m, k) in zip(names, shapes):
        client.getBloomFilter(nm).tryInitRaw(m, k)
        refs.append(O.OracleBloom(m, k))
    handles = [BloomHandle(client, nm) for nm in names]
    n = 5_000_000
    pool = rng.integers(0, 256, size=(400_000, 16), dtype=np.uint8)
    keys = pool[rng.integers(0, len(pool), size=n)]
    kf = np.zeros(n, np.uint32)
    op = np.zeros(n, np.uint8)
    runs, i = [], 0
    while i < n:
        ln = min(int(rng.integers(1, 40_000)), n - i)
        f, o = int(rng.integers(0, 2)), int(rng.random() < 0.3)
        kf[i:i + ln], op[i:i + ln] = f, o
        runs.append((i, ln, f, o))
        i += ln
    out, counts = bloom_stream(client, handles, kf, op, Arena.fixed(keys))
    want = np.zeros(n, np.uint8)
    for s, ln, f, o in runs:
        buf, offs = O.fixed_arena(keys[s:s + ln])
        _, fl = (refs[f].add if o else refs[f].contains)(buf, offs, per_key=True)
        want[s:s + ln] = fl
    assert np.array_equal(out, want)
    assert counts[0] == int(want[op == 0].sum()) and counts[1] == int(want[op == 1].sum())
    for nm, r in zip(names, refs):
        assert client.getBloomFilter(nm).exportBitmap() == r.redis_string()
    for h in handles:
        h.close()
    for nm in names:
        client.getBloomFilter(nm).delete()


@pytest.mark.parametrize("mode", [0, 1, 2])
@pytest.mark.parametrize("size,k,L", [(1 << 32, 7, 32), (4294967293, 7, 32), (300_000_007, 10, 16),
                                      (14377587, 2, 64), (95850583, 16, 0), (8388608 * 3 + 5, 5, 24)])
def test_partitioned_contains_parity(client, fresh, mode, size, k, L):
    """The region-bucketed contains (forced on, mode 1) and the direct kernel (mode 0) give the
    oracle's per-key answers; sizes that are not a multiple of the 1 MiB region included."""
    from redisson_amd import _lib as L_

    rng = np.random.default_rng(size % 1000 + k * 7 + L)
    n = 300_000
    if L:
        mat = rng.integers(0, 256, size=(n, L), dtype=np.uint8)
        a_add, a_probe = Arena.fixed(mat[: n // 2]), Arena.fixed(mat)
        o_add, o_probe = O.fixed_arena(mat[: n // 2]), O.fixed_arena(mat)
    else:
        keys = [rng.bytes(int(x)) for x in rng.integers(0, 90, size=n)]
        a_add, a_probe = Arena(keys[: n // 2]), Arena(keys)
        o_add, o_probe = O.arena(keys[: n // 2]), O.arena(keys)
    f = client.getBloomFilter(fresh)
    f.tryInitRaw(size, k)
    ref = O.OracleBloom(size, k)
    f.add(a_add)
    ref.add(*o_add)
    assert L_.lib().rbx_tune(b"contains_partition", mode) == 0
    try:
        cg, pg = f.containsEach(a_probe)
        c2 = f.contains(a_probe)
    finally:
        L_.lib().rbx_tune(b"contains_partition", 2)
    cr, pr = ref.contains(*o_probe, per_key=True)
    assert cg == cr == c2
    assert np.array_equal(pg, pr)
    f.delete()


@pytest.mark.parametrize("staging", [4096, 65536])
def test_host_path_pipelined_chunks(client, fresh, staging):
    """Host-buffer batches cut into many double-buffered upload chunks (tiny staging window):
    add order across chunks, variable-length keys split mid-arena, fixed strides."""
    from redisson_amd import _lib as L_

    rng = np.random.default_rng(staging)
    keys = [rng.bytes(int(x)) for x in rng.integers(0, 120, size=20000)]
    keys += keys[:3000]  # duplicates in later chunks
    mat = rng.integers(0, 256, size=(30000, 32), dtype=np.uint8)
    f = client.getBloomFilter(fresh)
    f.tryInitRaw(95850583, 7)
    ref = O.OracleBloom(95850583, 7)
    assert L_.lib().rbx_set_staging(client.ctx, staging) == 0
    try:
        cg, ng = f.addEach(Arena(keys))
        cr, nr = ref.add(*O.arena(keys), per_key=True)
        assert cg == cr and np.array_equal(ng, nr)
        cg, ng = f.addEach(Arena.fixed(mat))
        cr, nr = ref.add(*O.fixed_arena(mat), per_key=True)
        assert cg == cr and np.array_equal(ng, nr)
        probe = keys[::3] + [rng.bytes(int(x)) for x in rng.integers(0, 120, size=5000)]
        cg, pg = f.containsEach(Arena(probe))
        cr, pr = ref.contains(*O.arena(probe), per_key=True)
        assert cg == cr and np.array_equal(pg, pr)
    finally:
        L_.lib().rbx_set_staging(client.ctx, 64 << 20)
    assert f.exportBitmap() == ref.redis_string()
    f.delete()


@pytest.mark.parametrize("small", [1, 0])
def test_host_small_batches(client, fresh, small):
    """r05: host batches within host_small_bytes (here 256 KiB; default 4 MiB) take the one-transfer path (bloom_host_small:
    pinned copy, one upload with the zeroed count, one readback); with it on (1) and off (0): single
    keys, batches of 256 KiB and 256 KiB + 16 bytes, variable-length keys under and over the
    limit, empty keys, and a large pipelined batch in between -- add and contains, per-key flags and
    counts, then the bitmap, vs the oracle."""
    from redisson_amd import _lib as L_

    rng = np.random.default_rng(0x5A11 + small)
    f = client.getBloomFilter(fresh)
    f.tryInit(100_000, 0.01)
    ref = O.OracleBloom(f.getSize(), f.getHashIterations())
    mats = [rng.integers(0, 256, size=(n, 16), dtype=np.uint8) for n in (1, 1, 4096, 16384, 16385, 200_000)]
    var = [[rng.bytes(int(x)) for x in rng.integers(0, 91, size=500)],
           [rng.bytes(int(x)) for x in rng.integers(66, 76, size=4000)],  # ~280 KB: past the limit
           [b""] * 100]
    batches = [(Arena.fixed(m), O.fixed_arena(m)) for m in mats[:2]] + [(Arena(v), O.arena(v)) for v in var] + \
              [(Arena.fixed(m), O.fixed_arena(m)) for m in mats[2:]] + [(Arena.fixed(mats[0]), O.fixed_arena(mats[0]))]
    assert L_.lib().rbx_tune(b"host_small_batches", small) == 0
    assert L_.lib().rbx_tune(b"host_small_bytes", 256 << 10) == 0  # the batches straddle this limit
    try:
        for a, o in batches:
            cg, ng = f.addEach(a)
            cr, nr = ref.add(*o, per_key=True)
            assert cg == cr and np.array_equal(ng, nr)
            assert f.add(a) == ref.add(*o)  # again: every key present, count only
            cg, pg = f.containsEach(a)
            cr, pr = ref.contains(*o, per_key=True)
            assert cg == cr and np.array_equal(pg, pr)
        one = [bytes(mats[4][7]), b"never-added-key"]
        for key in one:  # contains(T) / add(T) shapes: one key per call
            assert f.contains(Arena([key])) == ref.contains(*O.arena([key]))
    finally:
        L_.lib().rbx_tune(b"host_small_batches", 1)
        L_.lib().rbx_tune(b"host_small_bytes", 4 << 20)
    assert f.exportBitmap() == ref.redis_string()
    assert f.count() == ref.count()
    f.delete()


@pytest.mark.parametrize("tiny,seg,one,spin", [(16384, 256, 1, 1), (16384, 256, 1, 0), (16384, 256, 0, 1),
                                               (16384, 16384, 1, 1), (0, 256, 1, 1), (0, 0, 0, 0)])
@pytest.mark.parametrize("k_fpp", [(100_000, 0.01), (10_000, 1e-6)])  # k = 7 and k = 20 (past k = 16: fallbacks)
def test_host_tiny_batches(client, fresh, tiny, seg, one, spin, k_fpp):
    """r06: host batches of <= host_tiny_keys keys and <= 64 KiB of key bytes run from coherent pinned memory
    (bloom_host_tiny: the kernel reads the keys over the host link and writes the flags back), and
    single-filter adds of <= add_single_seg_keys keys run the per-segment kernel on one segment, and one-key
    adds k_bloom_add_one (add_one_key), and small host calls spin on a completion word (host_tiny_spin);
    each on and off: single keys, a key repeated inside one batch (only its first occurrence is new), 255 / 256 / 4,096
    (= 64 KiB) / 4,097 keys, 16,384 short keys, variable-length and empty keys -- per-key flags and counts,
    then the bitmap and the Redis string length, vs the oracle."""
    from redisson_amd import _lib as L_

    rng = np.random.default_rng(0x7171 + tiny + k_fpp[0])
    f = client.getBloomFilter(fresh)
    f.tryInit(*k_fpp)
    ref = O.OracleBloom(f.getSize(), f.getHashIterations())
    dup = rng.integers(0, 256, size=(64, 16), dtype=np.uint8)
    dup[40] = dup[3]
    dup[63] = dup[3]
    mats = [rng.integers(0, 256, size=(n, 16), dtype=np.uint8) for n in (1, 2, 17, 63, 64, 65, 255, 256, 4096, 4097)] + [dup] + \
           [rng.integers(0, 256, size=(16384, 4), dtype=np.uint8)]
    var = [[rng.bytes(int(x)) for x in rng.integers(0, 91, size=300)], [b""] * 5,
           [b"k-%d" % (i % 7) for i in range(50)]]  # repeats inside the batch
    batches = [(Arena.fixed(m), O.fixed_arena(m)) for m in mats] + [(Arena(v), O.arena(v)) for v in var]
    assert L_.lib().rbx_tune(b"host_tiny_keys", tiny) == 0
    assert L_.lib().rbx_tune(b"add_single_seg_keys", seg) == 0
    assert L_.lib().rbx_tune(b"add_one_key", one) == 0
    assert L_.lib().rbx_tune(b"host_tiny_spin", spin) == 0
    try:
        for a, o in batches:
            cg, pg = f.containsEach(a)
            cr, pr = ref.contains(*o, per_key=True)
            assert cg == cr and np.array_equal(pg, pr)
            cg, ng = f.addEach(a)
            cr, nr = ref.add(*o, per_key=True)
            assert cg == cr and np.array_equal(ng, nr)
            assert f.add(a) == ref.add(*o)  # again: nothing new, count only
            assert f.contains(a) == ref.contains(*o)
        for key in [bytes(mats[8][9]), b"never-added-key", b""] + [rng.bytes(int(x)) for x in rng.integers(0, 80, 40)]:
            assert f.contains(Arena([key])) == ref.contains(*O.arena([key]))
            assert f.add(Arena([key])) == ref.add(*O.arena([key]))
    finally:
        L_.lib().rbx_tune(b"host_tiny_keys", 16384)
        L_.lib().rbx_tune(b"add_single_seg_keys", 256)
        L_.lib().rbx_tune(b"add_one_key", 1)
        L_.lib().rbx_tune(b"host_tiny_spin", 1)
    assert f.exportBitmap() == ref.redis_string()
    assert f.count() == ref.count()
    f.delete()


def test_pinned_host_arena(client, fresh):
    """Keys in rbx_host_alloc (pinned) memory go through the same path."""
    import ctypes as C

    from redisson_amd import _lib as L_
    from redisson_amd.keys import Arena as A

    rng = np.random.default_rng(5)
    n, L = 50000, 16
    p = C.c_void_p()
    assert L_.lib().rbx_host_alloc(n * L, C.byref(p)) == 0
    try:
        buf = np.ctypeslib.as_array((C.c_uint8 * (n * L)).from_address(p.value))
        buf[:] = rng.integers(0, 256, size=n * L, dtype=np.uint8)
        a = A.fixed(buf.reshape(n, L))
        f = client.getBloomFilter(fresh)
        f.tryInit(100000, 0.01)
        ref = O.OracleBloom(f.getSize(), f.getHashIterations())
        assert f.add(a) == ref.add(*O.fixed_arena(buf.reshape(n, L)))
        assert f.contains(a) == n
        f.delete()
    finally:
        L_.lib().rbx_host_free(p)


@pytest.mark.parametrize("mode,records", [(0, 2), (1, 2), (1, 0), (1, 1), (1, 3)])
@pytest.mark.parametrize("size,k,L", [(1 << 32, 7, 32), (4294967293, 7, 32), (300_000_007, 10, 16),
                                      ((1 << 29) + 3, 16, 0), (1 << 20, 3, 24), (100_003, 2, 64)])
def test_partitioned_add_parity(client, fresh, mode, records, size, k, L):
    """add() through the LDS-region partitioned pipeline (mode 1, forced) and the first-setter table
    (mode 0): per-key new flags, the count, the Redis bitmap bytes and length equal the oracle's
    in-order SETBIT fold, for a second batch that repeats keys within itself and re-adds keys of
    the first batch.  records: how the region kernel reports new keys -- 0 owner bits,
    1 non-owner counters, 3 owner records, 2 chosen from the sampled fill (the small filters are
    more than half full for batch two)."""
    from redisson_amd import _lib as L_

    rng = np.random.default_rng(size % 997 + 31 * k + L)
    n = 200_000
    if L:
        mat = rng.integers(0, 256, size=(n, L), dtype=np.uint8)
        first = mat[: n // 4]
        second = np.concatenate([mat[n // 8: n // 2], mat[rng.integers(0, n // 2, size=n // 4)], mat[n // 2:]])
        arenas = [(Arena.fixed(first), O.fixed_arena(first)), (Arena.fixed(second), O.fixed_arena(second))]
    else:
        keys = [rng.bytes(int(x)) for x in rng.integers(0, 90, size=n)]
        first = keys[: n // 4]
        second = keys[n // 8: n // 2] + [keys[i] for i in rng.integers(0, n // 2, size=n // 4)] + keys[n // 2:]
        arenas = [(Arena(first), O.arena(first)), (Arena(second), O.arena(second))]
    f = client.getBloomFilter(fresh)
    f.tryInitRaw(size, k)
    ref = O.OracleBloom(size, k)
    assert L_.lib().rbx_tune(b"add_partition", mode) == 0
    assert L_.lib().rbx_tune(b"add_records", records) == 0
    try:
        for a, o in arenas:
            cg, ng = f.addEach(a)
            cr, nr = ref.add(*o, per_key=True)
            assert cg == cr and np.array_equal(ng, nr)
    finally:
        L_.lib().rbx_tune(b"add_partition", 2)
        L_.lib().rbx_tune(b"add_records", 2)
    assert f.exportBitmap() == ref.redis_string()
    assert f.count() == ref.count()
    f.delete()


@pytest.mark.parametrize("records", [0, 1, 3])
def test_partitioned_add_collision_table_rounds(client, fresh, records):
    """Every key twice in one 2^16-bit region: ~3000 bits are met by two pairs, about six times the
    region kernel's 512-slot collision table, so the table is cleared and refilled for further
    rounds.  Flags, count and bitmap equal the oracle's in-order fold."""
    from redisson_amd import _lib as L_

    rng = np.random.default_rng(77)
    base = rng.integers(0, 256, size=(420, 24), dtype=np.uint8)
    batch = np.concatenate([base, base[::-1], rng.integers(0, 256, size=(3, 24), dtype=np.uint8)])
    f = client.getBloomFilter(fresh)
    f.tryInitRaw(1 << 16, 7)
    ref = O.OracleBloom(1 << 16, 7)
    assert L_.lib().rbx_tune(b"add_partition", 1) == 0
    assert L_.lib().rbx_tune(b"add_records", records) == 0
    try:
        cg, ng = f.addEach(Arena.fixed(batch))
        cg2, ng2 = f.addEach(Arena.fixed(batch[::3]))
    finally:
        L_.lib().rbx_tune(b"add_partition", 2)
        L_.lib().rbx_tune(b"add_records", 2)
    cr, nr = ref.add(*O.fixed_arena(batch), per_key=True)
    cr2, nr2 = ref.add(*O.fixed_arena(batch[::3]), per_key=True)
    assert cg == cr and np.array_equal(ng, nr)
    assert cg2 == cr2 and np.array_equal(ng2, nr2)
    assert f.exportBitmap() == ref.redis_string()
    f.delete()


@pytest.mark.parametrize("tune", [(b"add_rec_lds_limit", 0), (b"add_rec_lds_limit", 64)])
@pytest.mark.parametrize("records", [1, 3])
def test_partitioned_add_region_variants(client, fresh, tune, records):
    """The region pass's other branches give the oracle's answers too: owner records past the
    block's LDS record space (add_rec_lds_limit 0 / 64: every region, or most, reports its owners by
    direct atomics instead of record runs).  Two batches, the second re-adding and repeating keys;
    flags, counts, bitmap bytes and count() equal the in-order SETBIT fold."""
    from redisson_amd import _lib as L_

    rng = np.random.default_rng(4242 + records)
    n = 300_000
    mat = rng.integers(0, 256, size=(n, 32), dtype=np.uint8)
    second = np.concatenate([mat[n // 8: n // 2], mat[rng.integers(0, n // 2, size=n // 4)], mat[n // 2:]])
    f = client.getBloomFilter(fresh)
    f.tryInitRaw(1 << 28, 7)
    ref = O.OracleBloom(1 << 28, 7)
    key, val = tune
    assert L_.lib().rbx_tune(b"add_partition", 1) == 0
    assert L_.lib().rbx_tune(b"add_records", records) == 0
    assert L_.lib().rbx_tune(key, val) == 0
    try:
        for batch in (mat[: n // 4], second):
            cg, ng = f.addEach(Arena.fixed(batch))
            cr, nr = ref.add(*O.fixed_arena(batch), per_key=True)
            assert cg == cr and np.array_equal(ng, nr)
    finally:
        L_.lib().rbx_tune(b"add_partition", 2)
        L_.lib().rbx_tune(b"add_records", 2)
        L_.lib().rbx_tune(b"add_rec_lds_limit", 7168)
    assert f.exportBitmap() == ref.redis_string()
    assert f.count() == ref.count()
    f.delete()


def test_partitioned_add_overflow_falls_back(client, fresh):
    """A batch that overflows the partitioned add's bucket capacities (40 keys repeated 400k
    times) reruns on the first-setter table: flags, count and bitmap still equal the oracle's."""
    from redisson_amd import _lib as L_

    rng = np.random.default_rng(5)
    base = rng.integers(0, 256, size=(40, 32), dtype=np.uint8)
    batch = np.concatenate([base[rng.integers(0, 40, size=400_000)], rng.integers(0, 256, size=(30_000, 32),
                                                                                 dtype=np.uint8)])
    f = client.getBloomFilter(fresh)
    f.tryInitRaw(1 << 30, 7)
    ref = O.OracleBloom(1 << 30, 7)
    assert L_.lib().rbx_tune(b"add_partition", 1) == 0
    assert L_.lib().rbx_tune(b"add_records", 1) == 0
    try:
        cg, ng = f.addEach(Arena.fixed(batch))
    finally:
        L_.lib().rbx_tune(b"add_partition", 2)
        L_.lib().rbx_tune(b"add_records", 2)
    cr, nr = ref.add(*O.fixed_arena(batch), per_key=True)
    assert cg == cr and np.array_equal(ng, nr)
    assert f.exportBitmap() == ref.redis_string()
    f.delete()


def test_cross_stream_calls_run_in_call_order(client, fresh):
    """Device-path calls issued on different streams run in call order (the context's scratch and
    the bitmap are ordered by an event chain): add on stream A, then contains of the same keys on
    stream B sees every key, and a second add on B sees none as new; partitioned and table paths."""
    import torch

    from redisson_amd import device_keys

    n = 4_300_000  # above the partitioned paths' 2^22-key threshold
    g = torch.Generator(device="cuda")
    g.manual_seed(11)
    keys = torch.randint(0, 256, (n, 32), dtype=torch.uint8, device="cuda", generator=g)
    sa, sb = torch.cuda.Stream(), torch.cuda.Stream()
    for size in (1 << 32, 95850583):
        name = f"{fresh}-{size}"
        f = client.getBloomFilter(name)
        f.tryInitRaw(size, 7)
        h = BloomHandle(client, name)
        cnt = torch.zeros(4, dtype=torch.int64, device="cuda")
        torch.cuda.synchronize()
        dk = device_keys(keys.data_ptr(), n, 32)
        h.add_dev(dk, cnt.data_ptr(), stream=sa.cuda_stream)
        h.contains_dev(dk, cnt.data_ptr() + 8, stream=sb.cuda_stream)
        h.add_dev(dk, cnt.data_ptr() + 16, stream=sb.cuda_stream)
        h.contains_dev(dk, cnt.data_ptr() + 24, stream=sa.cuda_stream)
        torch.cuda.synchronize()
        c = cnt.tolist()
        assert c[1] == n and c[2] == 0 and c[3] == n, (size, c)
        assert c[0] >= n * 0.999  # in-batch false positives of the smaller filter (~1e-4 at its end fill)
        h.close()
        f.delete()


def test_default_partitioned_paths_device_keys(client, fresh):
    """Default dispatch on device-resident keys at C2 geometry (2^32 bits, k = 7), 4.5M 32-byte
    keys -- above both partitioned paths' thresholds: per-key add flags and contains flags from
    the partitioned pipelines equal the oracle's, and so do the exported bitmap bytes."""
    import torch

    from redisson_amd import device_keys

    rng = np.random.default_rng(0x5EED00C2)
    n = 4_500_000
    first = rng.integers(0, 256, size=(n, 32), dtype=np.uint8)
    probe = np.concatenate([first[: n // 2], rng.integers(0, 256, size=(n - n // 2, 32), dtype=np.uint8)])
    f = client.getBloomFilter(fresh)
    f.tryInitRaw(1 << 32, 7)
    h = BloomHandle(client, fresh)
    ref = O.OracleBloom(1 << 32, 7)
    cnt = torch.zeros(2, dtype=torch.int64, device="cuda")
    d_first = torch.from_numpy(first).cuda()
    d_probe = torch.from_numpy(probe).cuda()
    d_new = torch.zeros(n, dtype=torch.uint8, device="cuda")
    d_pres = torch.zeros(n, dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()  # the uploads ran on torch's stream, the engine uses its own
    h.add_dev(device_keys(d_first.data_ptr(), n, 32), cnt.data_ptr(), d_out=d_new.data_ptr())
    h.contains_dev(device_keys(d_probe.data_ptr(), n, 32), cnt.data_ptr() + 8, d_out=d_pres.data_ptr())
    torch.cuda.synchronize()
    cr, nr = ref.add(*O.fixed_arena(first), per_key=True)
    pr_c, pr = ref.contains(*O.fixed_arena(probe), per_key=True)
    assert int(cnt[0].item()) == cr and np.array_equal(d_new.cpu().numpy(), nr)
    assert int(cnt[1].item()) == pr_c and np.array_equal(d_pres.cpu().numpy(), pr)
    assert f.exportBitmap() == ref.redis_string()
    h.close()
    f.delete()


def test_multi_filter_table_cache_follows_handles(client, fresh):
    """Repeated multi-tenant calls reuse the device filter table; a different handle at any
    position (even one allocated where a closed handle was) or a keyspace change rebuilds it."""
    from redisson_amd import BloomHandle, bloom_contains_multi

    rng = np.random.default_rng(5)
    sets = {}
    for nm, size in (("a", 100003), ("b", 729), ("c", 95850583)):
        f = client.getBloomFilter(f"{fresh}-{nm}")
        f.tryInitRaw(size, 7)
        keys = [rng.bytes(16) for _ in range(3000)]
        f.add(Arena(keys))
        ref = O.OracleBloom(size, 7)
        ref.add(*O.arena(keys))
        sets[nm] = (ref, keys)
    probe = sets["a"][1][:1000] + sets["b"][1][:1000] + sets["c"][1][:1000]
    segs = np.array([0, 1000, 2000, 3000], np.uint64)

    def expect(names):
        return [sets[n][0].contains(*O.arena(probe[1000 * i:1000 * (i + 1)])) if n else 0
                for i, n in enumerate(names)]

    ha, hb, hc = (BloomHandle(client, f"{fresh}-{n}") for n in "abc")
    for _ in range(2):  # the second call takes the cached table
        assert list(bloom_contains_multi(client, [ha, hb, hc], segs, Arena(probe))) == expect("abc")
    hb.close()
    hb2 = BloomHandle(client, f"{fresh}-c")  # may reuse hb's address
    assert list(bloom_contains_multi(client, [ha, hb2, hc], segs, Arena(probe))) == expect("acc")
    assert list(bloom_contains_multi(client, [hc, hb2, ha], segs, Arena(probe))) == expect("cca")
    client.getBloomFilter(f"{fresh}-a").delete()  # keyspace change: the cached table is not reused
    with pytest.raises(RedisException, match="config has been changed"):  # addConfigCheck (:207-213)
        bloom_contains_multi(client, [ha, hb2, hc], segs, Arena(probe))
    for h in (ha, hb2, hc):
        h.close()
    for n in "bc":
        client.getBloomFilter(f"{fresh}-{n}").delete()


def test_partitioned_contains_deterministic_at_c2_scale(client, fresh):
    """100M keys at C2 geometry: every partitioned call answers exactly what the direct kernel
    answers, key by key (a lost or stray region pair would flip a few keys' flags), and the
    counts agree with the flags."""
    import torch

    from redisson_amd import _lib as L
    from redisson_amd import device_keys

    n = 100_000_000
    g = torch.Generator(device="cuda")
    g.manual_seed(11)
    keys = torch.randint(0, 256, (n, 32), dtype=torch.uint8, device="cuda", generator=g)
    f = client.getBloomFilter(fresh)
    f.tryInitRaw(1 << 32, 7)
    h = BloomHandle(client, fresh)
    cnt = torch.zeros(8, dtype=torch.int64, device="cuda")
    h.add_dev(device_keys(keys.data_ptr(), n // 2, 32), cnt.data_ptr())
    dk = device_keys(keys.data_ptr(), n, 32)
    ref = torch.zeros(n, dtype=torch.uint8, device="cuda")
    out = torch.zeros(n, dtype=torch.uint8, device="cuda")
    try:
        L.lib().rbx_tune(b"contains_partition", 0)
        h.contains_dev(dk, cnt.data_ptr() + 8, ref.data_ptr())
        L.lib().rbx_tune(b"contains_partition", 1)
        for i in range(4):
            out.fill_(7)
            h.contains_dev(dk, cnt.data_ptr() + 16 + 8 * i, out.data_ptr())
            torch.cuda.synchronize()
            diff = int((out != ref).sum())
            assert diff == 0, (i, diff, torch.nonzero(out != ref)[:8].flatten().tolist())
    finally:
        L.lib().rbx_tune(b"contains_partition", 2)
    torch.cuda.synchronize()
    c = cnt.tolist()
    assert bool(ref[: n // 2].all()) and c[1] == int(ref.sum(dtype=torch.int64))
    assert c[2:6] == [c[1]] * 4, c
    h.close()
    f.delete()
    del keys, ref, out
    torch.cuda.empty_cache()


def test_partitioned_add_record_kinds_agree_at_c2_scale(client, fresh):
    """50M keys into a 2^32-bit filter (C2 add geometry), then the same 50M again: the
    first-setter table and the partitioned add reporting owner bits, non-owner counters and owner
    records return the same per-key new flags and counts and leave identical bitmaps."""
    import torch

    from redisson_amd import _lib as L
    from redisson_amd import device_keys

    n = 50_000_000
    g = torch.Generator(device="cuda")
    g.manual_seed(12)
    keys = torch.randint(0, 256, (n, 32), dtype=torch.uint8, device="cuda", generator=g)
    keys[n - 1000:] = keys[:1000]  # repeats inside the batch
    dk = device_keys(keys.data_ptr(), n, 32)
    # (add_partition, add_records)
    runs = [(0, 2), (1, 0), (1, 1), (1, 3)]
    flags, counts, bitmaps = [], [], []
    try:
        for i, (part, rec) in enumerate(runs):
            nm = f"{fresh}-{i}"
            f = client.getBloomFilter(nm)
            f.tryInitRaw(1 << 32, 7)
            h = BloomHandle(client, nm)
            cnt = torch.zeros(2, dtype=torch.int64, device="cuda")
            out = torch.zeros((2, n), dtype=torch.uint8, device="cuda")
            L.lib().rbx_tune(b"add_partition", part)
            L.lib().rbx_tune(b"add_records", rec)
            for j in range(2):  # second pass: every key already present
                h.add_dev(dk, cnt.data_ptr() + 8 * j, out[j].data_ptr())
            torch.cuda.synchronize()
            flags.append(out)
            counts.append(cnt.tolist())
            bitmaps.append(f.exportBitmap())
            h.close()
            f.delete()
    finally:
        L.lib().rbx_tune(b"add_partition", 2)
        L.lib().rbx_tune(b"add_records", 2)
    assert counts[0][1] == 0 and n - 1000 - 10 <= counts[0][0] <= n - 1000, counts[0]
    for i in range(1, len(runs)):
        assert counts[i] == counts[0], (runs[i], counts[i], counts[0])
        assert torch.equal(flags[i], flags[0]), runs[i]
        assert bitmaps[i] == bitmaps[0], runs[i]
    del keys, flags
    torch.cuda.empty_cache()


@pytest.mark.parametrize("case", range(4))
def test_bitset_vectors_on_gpu(client, fresh, case):
    """T/RedissonBitSetTest.java:140-186 on the engine: each test's SETBIT sequence replayed as an add()
    of keys that hit the chosen bits of a raw (64, 1) filter; the exported Redis string has the
    reference's size() = STRLEN * 8 and cardinality() = BITCOUNT, bits MSB-first."""
    from bitset_vectors import BITSET_VECTORS, key_for_bit

    bits, size_bits, card = BITSET_VECTORS[case]
    f = client.getBloomFilter(fresh)
    f.tryInitRaw(64, 1)
    assert f.exportBitmap() == b""  # size() 0 before any SETBIT
    keys = [key_for_bit(b) for b in bits]
    c, new = f.addEach(Arena(keys))
    assert c == len(bits) and new.all()
    s = f.exportBitmap()
    assert len(s) * 8 == size_bits and f.bitcount() == card
    assert [i for i in range(len(s) * 8) if s[i >> 3] & (0x80 >> (i & 7))] == sorted(bits)
    assert f.contains(Arena([key_for_bit(0)])) == (1 if 0 in bits else 0)
    ref = O.OracleBloom(64, 1)
    ref.add(*O.arena(keys))
    assert s == ref.redis_string()
    f.delete()


def test_c3_full_tenant_count_slot_kernel(client, fresh):
    """C3 at its real size: 100k tryInit(1e6, 1e-3) tenants (14,377,587 bits each, 179.7 GB of
    slab-allocated bitmaps imported from slices of a device pool, as bench.py's C3 leg builds them),
    then one contains_multi batch of 24 16-byte keys per tenant on the default kernel for that size
    (the per-lane slot kernel, > 64 MiB of bitmaps).  1,000 sampled tenants first get 8 keys each
    through add_multi (one 100k-filter batch, epoch-tagged first-setter table), mirrored on oracle
    filters rebuilt from the same pool slices; their per-key contains flags and counts must match."""
    import ctypes as C

    import torch

    from redisson_amd import _lib as L

    nt, per, nsample = 100_000, 24, 1000
    rng = np.random.default_rng(0x5EED0003)
    pool = rng.integers(0, 256, size=64 << 20, dtype=np.uint8)
    dpool = torch.from_numpy(pool).cuda()
    names = [f"{fresh}:{t:06d}" for t in range(nt)]
    offs = np.zeros(nt, np.int64)
    handles = []
    try:
        for t, nm in enumerate(names):
            f = client.getBloomFilter(nm)
            assert f.tryInit(1_000_000, 1e-3)
            nb = (14_377_587 + 7) // 8
            offs[t] = int(rng.integers(0, (pool.size - nb) // 256)) * 256
            assert L.lib().rbx_bloom_import_dev(client.ctx, nm.encode(), dpool.data_ptr() + int(offs[t]), nb,
                                                None) == 0
            handles.append(BloomHandle(client, nm))
        assert (handles[0].size, handles[0].k) == (14_377_587, 10)
        sample = np.sort(rng.choice(nt, size=nsample, replace=False))
        refs = {}
        for t in sample:
            r = O.OracleBloom(14_377_587, 10)
            nb = (14_377_587 + 7) // 8
            r.bitmap[:nb] = pool[offs[t]:offs[t] + nb]
            r.redis_len = nb
            refs[int(t)] = r
        # adds: 8 keys into each sampled tenant, one multi-tenant add batch
        add_keys = rng.integers(0, 256, size=(nsample * 8, 16), dtype=np.uint8)
        aseg = np.arange(nsample + 1, dtype=np.uint64) * np.uint64(8)
        acounts, aflags = bloom_add_multi(client, [handles[t] for t in sample], aseg, Arena.fixed(add_keys),
                                          per_key=True)
        for s, t in enumerate(sample):
            c, fl = refs[int(t)].add(*O.fixed_arena(add_keys[8 * s:8 * s + 8]), per_key=True)
            assert acounts[s] == c and np.array_equal(aflags[8 * s:8 * s + 8], fl)
        # contains: per keys per tenant, the sampled tenants' first 8 keys are their added ones
        keys = rng.integers(0, 256, size=(nt * per, 16), dtype=np.uint8)
        for s, t in enumerate(sample):
            keys[t * per:t * per + 8] = add_keys[8 * s:8 * s + 8]
        seg = np.arange(nt + 1, dtype=np.uint64) * np.uint64(per)
        counts, flags = bloom_contains_multi(client, handles, seg, Arena.fixed(keys), per_key=True)
        for t in sample:
            t = int(t)
            c, fl = refs[t].contains(*O.fixed_arena(keys[t * per:(t + 1) * per]), per_key=True)
            assert counts[t] == c and np.array_equal(flags[t * per:(t + 1) * per], fl), t
            assert c >= 8
        assert int(counts.sum()) == int(flags.sum())
    finally:
        for h in handles:
            h.close()
        for nm in names:
            client.getBloomFilter(nm).delete()
        del dpool
        torch.cuda.empty_cache()
