"""Host arenas whose offsets do not start at 0 (a view into a larger caller buffer: rbx_keys.offsets
points into the middle of an offsets array, offsets[0] > 0).  The engine must read key i as
bytes[offsets[i] .. offsets[i+1]) on every host path -- by-name add/contains (one-transfer and
pipelined uploads), multi-tenant add/contains, the ordered stream and PFADD -- and answer as the
oracle does on the keys themselves.
"""
import numpy as np
import pytest

from oracle import oracle as O
from redisson_amd import Arena, BloomHandle, bloom_add_multi, bloom_contains_multi, bloom_stream
from redisson_amd import _lib as L

pytestmark = pytest.mark.gpu


def _sliced(keys, rng):
    """An Arena over prefix + keys whose struct views only `keys` (offsets[0] = the prefix's bytes)."""
    prefix = [rng.bytes(int(x)) for x in rng.integers(1, 50, size=7)]
    a = Arena(prefix + keys)
    a.struct = L.RbxKeys(a.bytes.ctypes.data, a.offsets.ctypes.data + 8 * len(prefix), 0, len(keys))
    a.n = len(keys)
    assert int(a.offsets[len(prefix)]) > 0
    return a


@pytest.mark.parametrize("small", [2, 1, 0])  # 2: the tiny path (coherent pinned keys), 1: one transfer, 0: pipelined
def test_sliced_arena_bloom_and_hll(client, fresh, small):
    rng = np.random.default_rng(0x511CE + small)
    keys = [rng.bytes(int(x)) for x in rng.integers(0, 70, size=1500 if small == 2 else 3000)]  # tiny: <= 64 KiB
    assert L.lib().rbx_tune(b"host_small_batches", min(small, 1)) == 0
    assert L.lib().rbx_tune(b"host_tiny_keys", 16384 if small == 2 else 0) == 0
    na = len(keys) * 2 // 3
    try:
        f = client.getBloomFilter(fresh)
        f.tryInit(50_000, 0.01)
        ref = O.OracleBloom(f.getSize(), f.getHashIterations())
        cg, ng = f.addEach(_sliced(keys[:na], rng))
        cr, nr = ref.add(*O.arena(keys[:na]), per_key=True)
        assert cg == cr and np.array_equal(ng, nr)
        cg, pg = f.containsEach(_sliced(keys, rng))
        cr, pr = ref.contains(*O.arena(keys), per_key=True)
        assert cg == cr and np.array_equal(pg, pr)
        assert f.exportBitmap() == ref.redis_string()
        f.delete()
        h = client.getHyperLogLog(fresh + "h")
        assert h.addAll(_sliced(keys, rng)) is True
        regs = O.hll_new()
        O.hll_pfadd(regs, *O.arena(keys))
        assert h.count() == O.hll_count(regs)
        h.delete()
    finally:
        L.lib().rbx_tune(b"host_small_batches", 1)
        L.lib().rbx_tune(b"host_tiny_keys", 16384)


def test_sliced_arena_multi_tenant_and_stream(client, fresh):
    rng = np.random.default_rng(0x511CF)
    nt = 5
    names = [f"{fresh}-{t}" for t in range(nt)]
    refs = []
    for nm in names:
        client.getBloomFilter(nm).tryInitRaw(40_000, 5)
        refs.append(O.OracleBloom(40_000, 5))
    handles = [BloomHandle(client, nm) for nm in names]
    keys = [rng.bytes(int(x)) for x in rng.integers(0, 60, size=1500)]
    segs = np.array([0, 200, 500, 900, 1200, 1500], np.uint64)
    counts, flags = bloom_add_multi(client, handles, segs, _sliced(keys, rng), per_key=True)
    for t in range(nt):
        a, b = int(segs[t]), int(segs[t + 1])
        c, fl = refs[t].add(*O.arena(keys[a:b]), per_key=True)
        assert counts[t] == c and np.array_equal(flags[a:b], fl), t
    pc, pf = bloom_contains_multi(client, handles, segs, _sliced(keys, rng), per_key=True)
    for t in range(nt):
        a, b = int(segs[t]), int(segs[t + 1])
        c, fl = refs[t].contains(*O.arena(keys[a:b]), per_key=True)
        assert pc[t] == c and np.array_equal(pf[a:b], fl), t
    n = 3000
    skeys = [keys[int(i)] if i < 1500 else rng.bytes(20) for i in rng.integers(0, 2000, size=n)]
    kf = rng.integers(0, nt, size=n).astype(np.uint32)
    op = (rng.random(n) < 0.3).astype(np.uint8)
    out, cnt = bloom_stream(client, handles, kf, op, _sliced(skeys, rng))
    buf, offs = O.arena(skeys)
    want, wc = O.bloom_stream(refs, kf, op, buf, offs)
    assert np.array_equal(out, want) and [int(cnt[0]), int(cnt[1])] == wc
    for nm, r in zip(names, refs):
        assert client.getBloomFilter(nm).exportBitmap() == r.redis_string(), nm
    for h in handles:
        h.close()
    for nm in names:
        client.getBloomFilter(nm).delete()
