"""One process over the GPUs of a node (rbx_node_*): slot routing, scatter / concurrent run /
gather of multi-tenant batches, and cross-GPU PFCOUNT / PFMERGE -- per key against the oracle.

The box has one GPU, so the node is rehearsed with several contexts on device 0 (devices =
[0] * N): every context has its own keyspace, streams and scratch exactly as it would on its
own GPU, and the routing is the one an 8-GPU node uses (slot * N / 16384,
M/cluster/ClusterConnectionManager.java:777-830)."""
import numpy as np
import pytest

from oracle import oracle as O
from redisson_amd import Arena, IllegalStateException, RedissonClient
from redisson_amd import _lib as L
from redisson_amd.node import RedissonNode

pytestmark = pytest.mark.gpu
N = 4


@pytest.fixture(scope="module")
def node():
    nd = RedissonNode(N, devices=[0] * N)
    yield nd
    nd.shutdown()


def test_routing_matches_calc_slot(node, fresh):
    names = [f"{fresh}:{i}" for i in range(200)] + [f"{{{fresh}}}:{i}" for i in range(5)]
    for nm in names:
        assert node.gpu_of(nm) == O.calc_slot(nm.encode()) * N // 16384
    # hashtags pin a group to one GPU; the config hash shares its filter's slot
    assert len({node.gpu_of(f"{{{fresh}}}:{i}") for i in range(5)}) == 1
    assert node.gpu_of(fresh) == node.gpu_of("{" + fresh + "}:config")


def test_multitenant_batch_scatter_gather(node, fresh):
    rng = np.random.default_rng(41)
    T = 40
    names = [f"{fresh}-tenant:{t:03d}" for t in range(T)]
    gpus = {node.gpu_of(n) for n in names}
    assert len(gpus) > 1  # the batch really spans contexts
    ref = {}
    for nm in names:
        assert node.getBloomFilter(nm).tryInit(20_000, 0.01)
        cfg = node.getBloomFilter(nm)
        ref[nm] = O.OracleBloom(cfg.getSize(), cfg.getHashIterations())
    per = rng.integers(1, 300, size=T)
    seg = np.concatenate([[0], np.cumsum(per)]).astype(np.uint64)
    keys = [rng.bytes(int(L_)) for L_ in rng.integers(1, 48, size=int(seg[-1]))]
    # add, per key flags and counts in segment order
    counts, flags = node.bloom_add_multi(names, seg, Arena(keys), per_key=True)
    for s, nm in enumerate(names):
        c, f = ref[nm].add(*O.arena(keys[seg[s]:seg[s + 1]]), per_key=True)
        assert counts[s] == c and np.array_equal(flags[seg[s]:seg[s + 1]], f), nm
    # contains of the same keys plus fresh ones, repeated tenants in one batch (segment order)
    order = list(range(T)) + [3, 3, 17]
    ks, segs = [], [0]
    for s in order:
        ks += keys[seg[s]:seg[s + 1]] + [rng.bytes(20) for _ in range(50)]
        segs.append(len(ks))
    counts, pres = node.bloom_contains_multi([names[s] for s in order], segs, Arena(ks), per_key=True)
    for j, s in enumerate(order):
        c, p = ref[names[s]].contains(*O.arena(ks[segs[j]:segs[j + 1]]), per_key=True)
        assert counts[j] == c and np.array_equal(pres[segs[j]:segs[j + 1]], p)
    # each tenant lives only on its slot's context: its bitmap bytes equal the oracle's there
    for nm in names[:8]:
        g = node.gpu_of(nm)
        import ctypes as C

        ctx = C.c_void_p()
        assert L.lib().rbx_node_ctx(node.node, g, C.byref(ctx)) == 0
        n = C.c_uint64()
        buf = np.zeros((abs(ref[nm].size) + 7) // 8 + 1, np.uint8)
        assert L.lib().rbx_bloom_export(ctx, nm.encode(), buf.ctypes.data_as(L.u8p), buf.size, C.byref(n)) == 0
        assert buf[: n.value].tobytes() == ref[nm].redis_string()
        for other in range(N):
            if other == g:
                continue
            assert L.lib().rbx_node_ctx(node.node, other, C.byref(ctx)) == 0
            e = C.c_int()
            assert L.lib().rbx_bloom_is_exists(ctx, nm.encode(), C.byref(e)) == 0 and e.value == 0
    # fixed-stride arenas scatter too
    mat = rng.integers(0, 256, size=(600, 16), dtype=np.uint8)
    fseg = np.array([0, 100, 250, 600], np.uint64)
    fcounts = node.bloom_contains_multi(names[:3], fseg, Arena.fixed(mat))
    for s in range(3):
        assert fcounts[s] == ref[names[s]].contains(*O.fixed_arena(mat[fseg[s]:fseg[s + 1]]))
    assert node.delete(*names, *["{" + n + "}:config" for n in names]) == 2 * T


def test_uninitialized_tenant_raises(node, fresh):
    with pytest.raises(IllegalStateException):
        node.bloom_contains_multi([fresh + "-x"], [0, 1], Arena([b"k"]))


def test_config_recreated_with_other_parameters(node, fresh):
    """A cached per-GPU handle whose config was re-created with other (size, k) is replaced: the
    batch reads the new config like a freshly created RBloomFilter."""
    nm = fresh + "-re"
    keys = [b"a", b"b", b"c"]
    f = node.getBloomFilter(nm)
    f.tryInit(1000, 0.01)
    assert node.bloom_add_multi([nm], [0, 3], Arena(keys))[0] == 3
    node.delete(nm, "{" + nm + "}:config")
    f.tryInit(5000, 0.001)
    ref = O.OracleBloom(*O.bloom_optimal(5000, 0.001))
    assert node.bloom_add_multi([nm], [0, 3], Arena(keys))[0] == ref.add(*O.arena(keys))
    node.delete(nm, "{" + nm + "}:config")


def test_node_hll_routing_and_cross_gpu_union(node, fresh):
    rng = np.random.default_rng(42)
    names = [f"{fresh}-h{i}" for i in range(12)]
    assert len({node.gpu_of(n) for n in names}) > 1
    mats = [rng.integers(0, 256, size=(int(rng.integers(100, 4000)), 16), dtype=np.uint8) for _ in names]
    seg = np.concatenate([[0], np.cumsum([m.shape[0] for m in mats])]).astype(np.uint64)
    allm = np.concatenate(mats)
    ch = node.hll_add_multi(names, seg, Arena.fixed(allm))
    assert ch.tolist() == [1] * len(names)
    regs = []
    for m in mats:
        r = O.hll_new()
        O.hll_pfadd(r, *O.fixed_arena(m))
        regs.append(r)
    for nm, r in zip(names, regs):
        assert node.getHyperLogLog(nm).count() == O.hll_count(r)
    # PFCOUNT over names on different GPUs = count of the union
    u = O.hll_new()
    for r in regs:
        O.hll_merge(u, r)
    assert node.getHyperLogLog(names[0]).countWith(*names[1:]) == O.hll_count(u)
    # PFMERGE into a destination on yet another slot
    dest = fresh + "-dest"
    node.getHyperLogLog(dest).mergeWith(*names)
    assert node.getHyperLogLog(dest).count() == O.hll_count(u)
    # the staged temporaries are gone: only the test's keys remain
    assert node.delete(*names, dest) == len(names) + 1


def test_node_and_single_context_agree(node, fresh):
    """The same single-tenant calls through the node and through one plain context."""
    rng = np.random.default_rng(43)
    keys = [rng.bytes(24) for _ in range(5000)]
    nf = node.getBloomFilter(fresh)
    nf.tryInit(10_000, 0.01)
    with RedissonClient(0) as c:
        cf = c.getBloomFilter(fresh)
        cf.tryInit(10_000, 0.01)
        assert nf.add(keys) == cf.add(keys)
        probe = keys[:2000] + [rng.bytes(24) for _ in range(2000)]
        assert nf.containsEach(probe)[1].tolist() == cf.containsEach(probe)[1].tolist()
        assert nf.count() == cf.count()
    node.delete(fresh, "{" + fresh + "}:config")


def test_contains_on_empty_filter_creates_no_bitmap(node, fresh):
    """a node contains_multi on an initialized filter that was never added to reads all
    zeros and creates no bitmap key (GETBIT creates nothing): DEL then counts only the config hash."""
    import ctypes as C

    nm = fresh + "-empty"
    assert node.getBloomFilter(nm).tryInit(10_000, 0.01)
    counts, pres = node.bloom_contains_multi([nm, nm], [0, 2, 3], Arena([b"a", b"b", b"c"]), per_key=True)
    assert counts.tolist() == [0, 0] and not pres.any()
    ctx = C.c_void_p()
    assert L.lib().rbx_node_ctx(node.node, node.gpu_of(nm), C.byref(ctx)) == 0
    e = C.c_int()
    arr, keep = L.names_array([nm])  # EXISTS name (the bitmap key)
    assert L.lib().rbx_exists_n(ctx, arr, 1, C.byref(e)) == 0 and e.value == 0
    assert node.delete(nm, "{" + nm + "}:config") == 1
    # a single-context handle does not create it either
    with RedissonClient(0) as c:
        f = c.getBloomFilter(nm)
        f.tryInit(10_000, 0.01)
        from redisson_amd import BloomHandle

        h = BloomHandle(c, nm)
        assert f.contains(["a", "b"]) == 0
        assert f.delete() is True  # config only; the bitmap never existed
        h.close()


def test_delete_releases_cached_handle_memory(node, fresh):
    """the node caches one handle per (GPU, name); DEL evicts it, so a deleted tenant's
    bitmap (here 120 MB, its own allocation past the 64 MiB slab limit) goes back to the device."""
    import torch

    nm = fresh + "-big"
    assert node.getBloomFilter(nm).tryInit(100_000_000, 0.01)  # 958,505,837 bits = 120 MB
    assert node.bloom_add_multi([nm], [0, 2], Arena([b"x", b"y"]))[0] == 2
    torch.cuda.synchronize()
    free0, _ = torch.cuda.mem_get_info()
    assert node.delete(nm, "{" + nm + "}:config") == 2
    torch.cuda.synchronize()
    free1, _ = torch.cuda.mem_get_info()
    assert free1 - free0 >= 100 << 20, (free0, free1)
    # re-created with other parameters afterwards: a fresh handle is opened
    assert node.getBloomFilter(nm).tryInit(1000, 0.01)
    ref = O.OracleBloom(*O.bloom_optimal(1000, 0.01))
    assert node.bloom_add_multi([nm], [0, 2], Arena([b"x", b"y"]))[0] == ref.add(*O.arena([b"x", b"y"]))
    assert node.delete(nm, "{" + nm + "}:config") == 2


def _ctx(node, g):
    import ctypes as C

    ctx = C.c_void_p()
    assert L.lib().rbx_node_ctx(node.node, g, C.byref(ctx)) == 0
    return ctx


def _export(ctx, nm, nbytes):
    import ctypes as C

    buf = np.zeros(nbytes + 1, np.uint8)
    n = C.c_uint64()
    assert L.lib().rbx_bloom_export(ctx, nm.encode(), buf.ctypes.data_as(L.u8p), buf.size, C.byref(n)) == 0
    return buf[: n.value].tobytes()


def _digest(ctx, nm):
    import ctypes as C

    d = C.c_uint64()
    assert L.lib().rbx_bloom_digest(ctx, nm.encode(), C.byref(d)) == 0
    return d.value


def test_replicated_filter(node, fresh):
    """SURVEY 8e for C2 ("replicas only"): a filter replicated on every GPU of the node.  The copy is
    device to device (rbx_bloom_copy_to); afterwards every add reaches every replica and contains are
    split across them -- replies per key equal the oracle's, all replicas stay byte-identical (equal
    Redis strings and digests), multi-tenant batches naming the filter follow the same rules, and DEL
    removes every copy."""
    rng = np.random.default_rng(44)
    nm, other = fresh + "-rep", fresh + "-solo"
    f = node.getBloomFilter(nm)
    assert f.tryInit(200_000, 0.01)
    ref = O.OracleBloom(f.getSize(), f.getHashIterations())
    nbytes = (f.getSize() + 7) // 8
    k1 = [rng.bytes(int(x)) for x in rng.integers(1, 40, size=20_000)]
    assert f.add(k1) == ref.add(*O.arena(k1))  # home GPU only
    assert not f.isReplicated()
    f.replicate()
    assert f.isReplicated()

    def all_equal():
        want = ref.redis_string()
        digests = set()
        for g in range(N):
            assert _export(_ctx(node, g), nm, nbytes) == want, g
            digests.add(_digest(_ctx(node, g), nm))
        assert len(digests) == 1 and 0 not in digests

    all_equal()
    k2 = k1[:5000] + [rng.bytes(24) for _ in range(30_000)]
    c, new = f.addEach(k2)
    cr, nr = ref.add(*O.arena(k2), per_key=True)
    assert c == cr and np.array_equal(new, nr)
    all_equal()
    probe = k2[::3] + [rng.bytes(24) for _ in range(40_000)]
    cp, pres = f.containsEach(probe)
    crp, pr = ref.contains(*O.arena(probe), per_key=True)
    assert cp == crp and np.array_equal(pres, pr)
    # multi-tenant batches naming the replicated filter (adds to every replica, contains spread)
    assert node.getBloomFilter(other).tryInit(10_000, 0.01)
    oref = O.OracleBloom(*O.bloom_optimal(10_000, 0.01))
    k3 = [rng.bytes(16) for _ in range(3000)]
    seg = np.array([0, 1000, 1500, 3000], np.uint64)
    counts, flags = node.bloom_add_multi([nm, other, nm], seg, Arena(k3), per_key=True)
    for s, r in enumerate([ref, oref, ref]):
        cc, ff = r.add(*O.arena(k3[seg[s]:seg[s + 1]]), per_key=True)
        assert counts[s] == cc and np.array_equal(flags[seg[s]:seg[s + 1]], ff)
    all_equal()
    names = [nm, other] + [nm] * 6
    seg = np.arange(len(names) + 1, dtype=np.uint64) * np.uint64(500)
    k4 = [k3[int(i)] if rng.random() < 0.5 else rng.bytes(16) for i in rng.integers(0, 3000, size=int(seg[-1]))]
    counts, flags = node.bloom_contains_multi(names, seg, Arena(k4), per_key=True)
    for s, n_ in enumerate(names):
        r = ref if n_ == nm else oref
        cc, ff = r.contains(*O.arena(k4[seg[s]:seg[s + 1]]), per_key=True)
        assert counts[s] == cc and np.array_equal(flags[seg[s]:seg[s + 1]], ff)
    assert f.count() == ref.count()
    # DEL removes every copy and ends the replication
    assert node.delete(nm, "{" + nm + "}:config", other, "{" + other + "}:config") == 4
    assert not f.isReplicated()
    import ctypes as C

    for g in range(N):
        e = C.c_int()
        names_, keep = L.names_array([nm, "{" + nm + "}:config"])
        assert L.lib().rbx_exists_n(_ctx(node, g), names_, 2, C.byref(e)) == 0 and e.value == 0, g


def test_bloom_copy_between_contexts_and_digest(fresh):
    """rbx_bloom_copy_to between two contexts (the replica-sync primitive): config hash (all four
    fields) and bitmap string arrive byte-identical; the digest tells equal from different."""
    import ctypes as C

    rng = np.random.default_rng(45)
    with RedissonClient(0) as a, RedissonClient(0) as b:
        fa = a.getBloomFilter(fresh)
        assert fa.tryInit(1_000_000, 1e-3)
        keys = [rng.bytes(32) for _ in range(50_000)]
        fa.add(keys)
        assert b.getBloomFilter(fresh).digest() == 0  # missing key
        nm = L.name_struct(fresh)
        assert L.lib().rbx_bloom_copy_to(a.ctx, b.ctx, nm[0]) == 0
        fb = b.getBloomFilter(fresh)
        assert (fb.getSize(), fb.getHashIterations(), fb.getExpectedInsertions(), fb.getFalseProbability()) == \
            (fa.getSize(), fa.getHashIterations(), 1_000_000, 1e-3)
        assert fb.exportBitmap() == fa.exportBitmap() and fb.digest() == fa.digest() != 0
        assert fb.contains(keys) == len(keys)
        fb.add([b"only-on-b"])
        assert fb.digest() != fa.digest()
        assert L.lib().rbx_bloom_copy_to(a.ctx, b.ctx, nm[0]) == 0  # re-sync in place
        assert fb.digest() == fa.digest()
        assert L.lib().rbx_bloom_copy_to(a.ctx, a.ctx, nm[0]) == L.RBX_E_ILLEGAL_ARGUMENT
        missing = L.name_struct(fresh + "-none")
        assert L.lib().rbx_bloom_copy_to(a.ctx, b.ctx, missing[0]) == L.RBX_E_ILLEGAL_STATE
        fa.delete()
        fb.delete()


def test_cross_gpu_hll_union_keeps_encodings(node, fresh):
    """Cross-GPU PFCOUNT / PFMERGE stage remote HLLs by device copies (rbx_hll_copy_to): a merge of
    sparse-only inputs stays sparse and one dense input makes it dense, as Redis PFMERGE does."""
    import ctypes as C

    rng = np.random.default_rng(46)
    names = [f"{fresh}-s{i}" for i in range(6)]
    assert len({node.gpu_of(n) for n in names}) > 1
    regs = []
    for i, nm in enumerate(names):
        el = rng.integers(0, 256, size=(50 if i < 5 else 20_000, 16), dtype=np.uint8)
        node.getHyperLogLog(nm).addAll([bytes(x) for x in el])
        r = O.hll_new()
        O.hll_pfadd(r, *O.fixed_arena(el))
        regs.append(r)

    def stored(nm):
        ctx = _ctx(node, node.gpu_of(nm))
        buf = np.zeros(16 + 12288, np.uint8)
        n = C.c_uint64()
        s, keep = L.name_struct(nm)
        assert L.lib().rbx_hll_export_enc_n(ctx, s, 2, buf.ctypes.data_as(L.u8p), buf.size,  # AS_STORED
                                            C.byref(n)) == 0
        return buf[: n.value].tobytes()

    u = O.hll_new()
    for r in regs[:5]:
        O.hll_merge(u, r)
    d1 = fresh + "-d1"
    node.getHyperLogLog(d1).mergeWith(*names[:5])
    s1 = stored(d1)
    assert s1[4] == 1 and np.array_equal(O.hll_sparse_unpack(s1[16:]), u)  # sparse
    d2 = fresh + "-d2"
    node.getHyperLogLog(d2).mergeWith(*names)
    O.hll_merge(u, regs[5])
    s2 = stored(d2)
    assert s2[4] == 0 and np.array_equal(O.hll_dense_unpack(s2[16:]), u)  # dense
    assert node.getHyperLogLog(names[0]).countWith(*names[1:]) == O.hll_count(u)
    assert node.delete(*names, d1, d2) == len(names) + 2


def _exists_anywhere(node, names):
    import ctypes as C

    out = []
    for g in range(N):
        e = C.c_int()
        arr, keep = L.names_array(names)
        assert L.lib().rbx_exists_n(_ctx(node, g), arr, len(names), C.byref(e)) == 0
        out.append(e.value)
    return out


def test_replicated_add_failure_drops_replication(node, fresh):
    """an add of a replicated filter that fails on one replica must not leave the
    copies divergent and still marked replicated.  The node then drops the replication: the copies
    are deleted on every non-home GPU, contains go to the home GPU, and the error is returned.  A
    test hook (rbx_node_test_fail_adds) fails the next add on a chosen GPU before it runs."""
    from redisson_amd.exceptions import DeviceError

    rng = np.random.default_rng(47)
    nm, other = fresh + "-rf", fresh + "-rf-other"
    f = node.getBloomFilter(nm)
    assert f.tryInit(100_000, 0.01)
    ref = O.OracleBloom(f.getSize(), f.getHashIterations())
    nbytes = (f.getSize() + 7) // 8
    home = node.gpu_of(nm)
    k1 = [rng.bytes(20) for _ in range(5000)]
    assert f.add(k1) == ref.add(*O.arena(k1))
    f.replicate()
    # a replica (not the home GPU) fails: home applied the add, the copies are dropped
    victim = (home + 1) % N
    assert L.lib().rbx_node_test_fail_adds(node.node, victim, 1) == 0
    k2 = [rng.bytes(20) for _ in range(5000)]
    with pytest.raises(DeviceError, match="injected"):
        f.add(k2)
    ref.add(*O.arena(k2))
    assert not f.isReplicated()
    assert _export(_ctx(node, home), nm, nbytes) == ref.redis_string()
    ex = _exists_anywhere(node, [nm, "{" + nm + "}:config"])
    assert ex[home] == 2 and all(ex[g] == 0 for g in range(N) if g != home), ex
    probe = k1[:1000] + k2[:1000] + [rng.bytes(20) for _ in range(3000)]
    cp, pres = f.containsEach(probe)
    crp, pr = ref.contains(*O.arena(probe), per_key=True)
    assert cp == crp and np.array_equal(pres, pr)
    # the home GPU fails inside a multi-tenant batch: the replicas applied it, home did not -- the
    # replication is dropped again and home keeps its own (unchanged) filter
    assert node.getBloomFilter(other).tryInit(10_000, 0.01)
    f.replicate()
    assert f.isReplicated()
    assert L.lib().rbx_node_test_fail_adds(node.node, home, 1) == 0
    k3 = [rng.bytes(16) for _ in range(2000)]
    with pytest.raises(DeviceError, match="injected"):
        node.bloom_add_multi([nm, other], [0, 1000, 2000], Arena(k3))
    assert L.lib().rbx_node_test_fail_adds(node.node, home, 0) == 0
    assert not f.isReplicated()
    assert _export(_ctx(node, home), nm, nbytes) == ref.redis_string()
    ex = _exists_anywhere(node, [nm, "{" + nm + "}:config"])
    assert all(ex[g] == 0 for g in range(N) if g != home), ex
    # replicated again, everything agrees
    f.replicate()
    for g in range(N):
        assert _export(_ctx(node, g), nm, nbytes) == ref.redis_string(), g
    # `other` got its bitmap unless its part of the batch ran on the failed (home) GPU
    other_bm = _exists_anywhere(node, [other])[node.gpu_of(other)]
    assert other_bm == (0 if node.gpu_of(other) == home else 1)
    assert node.delete(nm, "{" + nm + "}:config", other, "{" + other + "}:config") == 3 + other_bm


def test_replicate_concurrent_with_adds(node, fresh):
    """replicate(on) concurrent with adds of the same filter.  The copy and the
    routing change are exclusive against batches, so no add reaches only the home GPU: afterwards
    every replica equals the oracle's bitmap, and every added key is present through each replica."""
    import threading

    rng = np.random.default_rng(48)
    nm = fresh + "-rc"
    f = node.getBloomFilter(nm)
    assert f.tryInit(400_000, 0.01)
    ref = O.OracleBloom(f.getSize(), f.getHashIterations())
    nbytes = (f.getSize() + 7) // 8
    batches = [[rng.bytes(24) for _ in range(4000)] for _ in range(40)]
    errors = []

    def adder():
        try:
            for b in batches:
                f.add(b)
        except Exception as e:  # noqa: BLE001 -- reported below
            errors.append(e)

    t = threading.Thread(target=adder)
    t.start()
    f.replicate()
    t.join()
    assert not errors, errors
    for b in batches:
        ref.add(*O.arena(b))
    want = ref.redis_string()
    for g in range(N):
        assert _export(_ctx(node, g), nm, nbytes) == want, g
    allk = [k for b in batches for k in b]
    assert f.contains(allk) == len(allk)  # spread over the replicas
    # and replicate(off) concurrent with contains: the answers never lose a key
    res = []

    def checker():
        for _ in range(10):
            res.append(f.contains(allk[:20_000]))

    t = threading.Thread(target=checker)
    t.start()
    f.replicate(False)
    t.join()
    assert res == [20_000] * 10
    node.delete(nm, "{" + nm + "}:config")


def test_config_only_delete_drops_replica_bitmaps(node, fresh):
    """DEL of only a replicated filter's config ends the replication and deletes the
    copies' bitmaps too (Redis keeps the home bitmap; the copies are the node's own)."""
    nm = fresh + "-cd"
    f = node.getBloomFilter(nm)
    assert f.tryInit(50_000, 0.01)
    f.add([b"a", b"b"])
    f.replicate()
    home = node.gpu_of(nm)
    assert node.delete("{" + nm + "}:config") == 1
    assert not f.isReplicated()
    ex = _exists_anywhere(node, [nm, "{" + nm + "}:config"])
    assert ex[home] == 1 and all(ex[g] == 0 for g in range(N) if g != home), ex
    assert node.delete(nm) == 1
