"""Object lifetimes and stream order of the device-path handles, checked against the oracle.

- A key re-created behind an open handle (DEL, then add_dev / PFADD on a non-default stream)
  starts from zeroed memory although the pool hands back the deleted object's block: the zero
  fill runs on the calling stream, after every earlier call of the context.
- Handles outlive rbx_shutdown safely; every call on them then fails.
- tryInit with a negative expectedInsertions (the reference accepts it,
  M/RedissonBloomFilter.java:270-276): add / contains / count against the oracle, including
  |size| > 2^32, where an index past the Redis offset limit makes the call throw RedisException
  after the batch's other SETBITs ran (rbx.h RBX_E_REDIS).
- Binary (NUL-containing) Bloom names through the *_n entry points.
- Register pack / unpack_max, and an element-partitioned HLL set merged across two processes
  that created their HLLs in different orders (the exchange rbx_hll_allreduce_max performs with
  RCCL, here over gloo on one GPU).
"""
import ctypes as C
import os
import socket

import numpy as np
import pytest

from oracle import oracle as O
from redisson_amd import Arena, BloomHandle, IllegalStateException, RedisException, RedissonClient, device_keys
from redisson_amd import _lib as L
from redisson_amd.client import _check

pytestmark = pytest.mark.gpu


def _del(client, name: str) -> int:
    arr, keep = L.names_array([name])
    n = C.c_int()
    _check(L.lib().rbx_del_n(client.ctx, arr, 1, C.byref(n)))
    return n.value


def test_recreated_bitmap_is_zero_on_caller_stream(client, fresh):
    import torch

    rng = np.random.default_rng(21)
    f = client.getBloomFilter(fresh)
    f.tryInit(200_000, 0.01)
    size, k = f.getSize(), f.getHashIterations()
    h = BloomHandle(client, fresh)
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    first = torch.from_numpy(rng.integers(0, 256, size=(150_000, 32), dtype=np.uint8)).cuda()
    second_np = rng.integers(0, 256, size=(120_000, 32), dtype=np.uint8)
    second = torch.from_numpy(second_np).cuda()
    cnt = torch.zeros(2, dtype=torch.int64, device="cuda")
    flags = torch.zeros(second_np.shape[0], dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()
    for _ in range(3):
        h.add_dev(device_keys(first.data_ptr(), first.shape[0], 32), cnt.data_ptr(), stream=s1.cuda_stream)
        # DEL name (the config stays): the bitmap's block returns to the pool with its bits set
        assert _del(client, fresh) == 1
        # re-created by the next SETBIT, on another stream, from the same pool block
        h.add_dev(device_keys(second.data_ptr(), second.shape[0], 32), cnt.data_ptr() + 8,
                  d_out=flags.data_ptr(), stream=s2.cuda_stream)
        torch.cuda.synchronize()
        ref = O.OracleBloom(size, k)
        c_ref, new_ref = ref.add(*O.fixed_arena(second_np), per_key=True)
        assert np.array_equal(flags.cpu().numpy(), new_ref)
        assert f.exportBitmap() == ref.redis_string()
        assert int(cnt[1].item()) == c_ref
        cnt.zero_()
    h.close()
    f.delete()


def test_recreated_hll_is_zero_on_caller_stream(client, fresh):
    import torch

    rng = np.random.default_rng(22)
    hp = C.c_void_p()
    _check(L.lib().rbx_hll_open(client.ctx, fresh.encode(), 1, C.byref(hp)))
    arr = (C.c_void_p * 1)(hp.value)
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    a = rng.integers(0, 256, size=(200_000, 16), dtype=np.uint8)
    b = rng.integers(0, 256, size=(3_000, 16), dtype=np.uint8)
    da, db = torch.from_numpy(a).cuda(), torch.from_numpy(b).cuda()
    changed = torch.zeros(1, dtype=torch.int32, device="cuda")
    torch.cuda.synchronize()
    for _ in range(3):
        sa = np.array([0, a.shape[0]], np.uint64)
        _check(L.lib().rbx_hll_add_multi_dev(client.ctx, arr, 1, None, sa.ctypes.data_as(L.u64p),
                                             C.byref(device_keys(da.data_ptr(), a.shape[0], 16)),
                                             changed.data_ptr(), s1.cuda_stream))
        assert _del(client, fresh) == 1
        sb = np.array([0, b.shape[0]], np.uint64)
        _check(L.lib().rbx_hll_add_multi_dev(client.ctx, arr, 1, None, sb.ctypes.data_as(L.u64p),
                                             C.byref(device_keys(db.data_ptr(), b.shape[0], 16)),
                                             changed.data_ptr(), s2.cuda_stream))
        torch.cuda.synchronize()
        ref = O.hll_new()
        O.hll_pfadd(ref, *O.fixed_arena(b))
        d = client.getHyperLogLog(fresh).exportDense()
        assert np.array_equal(O.hll_dense_unpack(d[16:]), ref)
    L.lib().rbx_hll_close(hp)


def test_handles_outlive_shutdown():
    c = RedissonClient(0)
    f = c.getBloomFilter("life")
    f.tryInit(1000, 0.01)
    f.add(["a", "b"])
    bh = BloomHandle(c, "life")
    hp = C.c_void_p()
    _check(L.lib().rbx_hll_open(c.ctx, b"life-hll", 1, C.byref(hp)))
    ctx = c.ctx
    c.shutdown()
    import torch

    keys = torch.zeros((4, 16), dtype=torch.uint8, device="cuda")
    cnt = torch.zeros(1, dtype=torch.int64, device="cuda")
    rc = L.lib().rbx_bloom_add_dev(ctx, bh.h, C.byref(device_keys(keys.data_ptr(), 4, 16)), None, cnt.data_ptr(),
                                   None)
    assert rc == L.RBX_E_ILLEGAL_STATE
    with pytest.raises(IllegalStateException):
        _check(rc)
    out = np.zeros(1, np.uint64)
    arr = (C.c_void_p * 1)(hp.value)
    assert L.lib().rbx_hll_count_each_handles(ctx, arr, 1, out.ctypes.data_as(L.u64p)) == L.RBX_E_ILLEGAL_STATE
    # closing after shutdown is safe; the context's memory goes with the last handle
    bh.close()
    assert L.lib().rbx_hll_close(hp) == 0


def test_negative_expected_insertions_filter(client, fresh):
    f = client.getBloomFilter(fresh)
    assert f.tryInit(-20_000, 0.01)
    size, k = f.getSize(), f.getHashIterations()
    assert size < 0 and (size, k) == O.bloom_optimal(-20_000, 0.01)
    ref = O.OracleBloom(size, k)
    rng = np.random.default_rng(23)
    keys = [rng.bytes(int(n)) for n in rng.integers(1, 40, size=15_000)]
    c, new = f.addEach(Arena(keys))
    c_ref, new_ref = ref.add(*O.arena(keys), per_key=True)
    assert c == c_ref and np.array_equal(new, new_ref)
    probe = keys[:5000] + [rng.bytes(20) for _ in range(5000)]
    c, pres = f.containsEach(Arena(probe))
    c_ref, pres_ref = ref.contains(*O.arena(probe), per_key=True)
    assert c == c_ref and np.array_equal(pres, pres_ref)
    assert f.exportBitmap() == ref.redis_string()
    assert f.count() == ref.count()
    f.delete()


def _wide_call(f, ref, keys, is_add):
    """one add / contains on the GPU and the oracle: both fail (-9 / RedisException) or both give
    the same count and per-key flags"""
    c_ref, fl_ref = (ref.add if is_add else ref.contains)(*O.arena(keys), per_key=True)
    if c_ref == -9:
        with pytest.raises(RedisException, match="bit offset is not an integer or out of range"):
            (f.addEach if is_add else f.containsEach)(Arena(keys))
        return False
    c, fl = (f.addEach if is_add else f.containsEach)(Arena(keys))
    assert c == c_ref and np.array_equal(fl, fl_ref)
    return True


def test_filter_past_the_redis_offset_limit(client, fresh):
    """|size| = 4,792,529,188 (tryInit(-5e8, 0.01)): 10% of the indexes pass 2^32 - 1."""
    f = client.getBloomFilter(fresh)
    assert f.tryInit(-500_000_000, 0.01)
    size, k = f.getSize(), f.getHashIterations()
    assert (size, k) == O.bloom_optimal(-500_000_000, 0.01) and -size > (1 << 32)
    ref = O.OracleBloom(size, k)
    rng = np.random.default_rng(31)
    # a batch made only of error replies creates no key: k = 1 over |size| = 1.44e12 bits
    g = client.getBloomFilter(fresh + "-k1")
    assert g.tryInit(-1_000_000_000_000, 0.5)
    gs, gk = g.getSize(), g.getHashIterations()
    assert gk == 1 and -gs > (300 << 32)
    gref = O.OracleBloom(gs, gk)
    lone = next(key for key in (rng.bytes(16) for _ in range(100))
                if O.bloom_indexes(*O.redisson_hash128(key), gk, gs)[0] > 0xFFFFFFFF)
    assert not _wide_call(g, gref, [lone], True)
    assert _del(client, fresh + "-k1") == 0  # no bitmap key (the config stays)
    g.delete()
    ok = [_wide_call(f, ref, [rng.bytes(16)], True) for _ in range(48)]
    assert 5 < sum(ok) < 43  # ~46% of single keys stay below the limit
    assert not _wide_call(f, ref, [rng.bytes(24) for _ in range(3000)], True)  # throws, bits still set
    seen = [rng.bytes(16) for _ in range(8)]
    for key in seen:
        _wide_call(f, ref, [key], True)
    res = [_wide_call(f, ref, [key], False) for key in seen + [rng.bytes(16) for _ in range(24)]]
    assert any(res) and not all(res)
    assert not _wide_call(f, ref, seen * 50, False)
    assert f.exportBitmap() == ref.redis_string()
    assert f.count() == ref.count()
    f.delete()


def test_filter_just_past_2_32_bits(client, fresh):
    """|size| = 2^32 + 7 (tryInit(-448,089,843, 0.01)): indexes mod |size| in 64 bits, and a batch
    of 200K keys (with repeats) almost never reaches an offset past the limit -- per-key in-order
    flags and presence against the oracle."""
    f = client.getBloomFilter(fresh)
    assert f.tryInit(-448_089_843, 0.01)
    size, k = f.getSize(), f.getHashIterations()
    assert -size == (1 << 32) + 7 and k == 7
    ref = O.OracleBloom(size, k)
    rng = np.random.default_rng(32)
    base = [rng.bytes(int(n)) for n in rng.integers(0, 60, size=60_000)]
    for _ in range(2):
        batch = [base[int(j)] for j in rng.integers(0, len(base), size=100_000)]
        assert _wide_call(f, ref, batch, True)
    probe = base[:20_000] + [rng.bytes(33) for _ in range(20_000)]
    assert _wide_call(f, ref, probe, False)
    assert f.exportBitmap() == ref.redis_string()
    f.delete()


def test_wide_filter_short_keys_in_subchunks(client, fresh):
    """a staging chunk of empty / 1-byte keys holds any number of keys, so the wide
    path splits it into sub-chunks (<= 2^29 / k keys: a first-setter table of <= 2^30 entries).
    Here the sub-chunk is capped at 7,001 keys (rbx_tune wide_subchunk) so one 60K-key batch of
    empty, 1- and 2-byte keys (massively repeated: the same bits recur across sub-chunks) runs in
    nine sub-chunks in key order; per-key flags, counts and the bitmap vs the oracle."""
    f = client.getBloomFilter(fresh)
    assert f.tryInit(-448_089_843, 0.01)
    size, k = f.getSize(), f.getHashIterations()
    ref = O.OracleBloom(size, k)
    rng = np.random.default_rng(33)
    pool = [b""] + [bytes([i]) for i in range(256)] + [rng.bytes(2) for _ in range(300)]
    batch = [pool[int(j)] for j in rng.integers(0, len(pool), size=60_000)]
    assert L.lib().rbx_tune(b"wide_subchunk", 7001) == 0
    try:
        assert _wide_call(f, ref, batch, True)
        assert _wide_call(f, ref, batch[:30_000] + [rng.bytes(3) for _ in range(30_000)], False)
    finally:
        L.lib().rbx_tune(b"wide_subchunk", 0)
    assert f.exportBitmap() == ref.redis_string()
    f.delete()


def test_binary_bloom_names(client, fresh):
    rng = np.random.default_rng(24)
    n1, n2 = fresh.encode() + b"\x00x", fresh.encode() + b"\x00y"
    created = C.c_int()
    for nm in (n1, n2):
        s, keep = L.name_struct(nm)
        _check(L.lib().rbx_bloom_try_init_n(client.ctx, s, 5000, 0.01, C.byref(created)))
        assert created.value == 1
    s1, k1 = L.name_struct(n1)
    cfg = L.RbxBloomConfig()
    _check(L.lib().rbx_bloom_read_config_n(client.ctx, s1, C.byref(cfg)))
    keys = [rng.bytes(16) for _ in range(3000)]
    a = Arena(keys)
    cnt = C.c_uint64()
    _check(L.lib().rbx_bloom_add_n(client.ctx, s1, cfg.size, cfg.hash_iterations, a.ptr(), None, C.byref(cnt)))
    ref = O.OracleBloom(cfg.size, cfg.hash_iterations)
    assert cnt.value == ref.add(*O.arena(keys))
    s2, k2 = L.name_struct(n2)
    _check(L.lib().rbx_bloom_contains_n(client.ctx, s2, cfg.size, cfg.hash_iterations, a.ptr(), None,
                                        C.byref(cnt)))
    assert cnt.value == 0  # a different key: nothing added there
    _check(L.lib().rbx_bloom_contains_n(client.ctx, s1, cfg.size, cfg.hash_iterations, a.ptr(), None,
                                        C.byref(cnt)))
    assert cnt.value == 3000
    out = C.c_int64()
    _check(L.lib().rbx_bloom_count_n(client.ctx, s1, C.byref(out)))
    assert out.value == ref.count()
    arr, keep = L.names_array([n1, n2, n1 + b"\x00:missing"])
    ex = C.c_int()
    _check(L.lib().rbx_exists_n(client.ctx, arr, 3, C.byref(ex)))
    assert ex.value == 1  # only n1's bitmap exists (n2 has a config, no bitmap)


def _open_hlls(client, names):
    hs = []
    for nm in names:
        hp = C.c_void_p()
        _check(L.lib().rbx_hll_open(client.ctx, nm.encode(), 1, C.byref(hp)))
        hs.append(hp.value)
    return hs, (C.c_void_p * len(hs))(*hs)


def test_hll_pack_unpack_registers(client, fresh):
    import torch

    rng = np.random.default_rng(25)
    names = [f"{fresh}-{i}" for i in range(3)]
    refs = []
    for nm in names:
        m = rng.integers(0, 256, size=(4000, 16), dtype=np.uint8)
        client.getHyperLogLog(nm).addAll(Arena.fixed(m))
        r = O.hll_new()
        O.hll_pfadd(r, *O.fixed_arena(m))
        refs.append(r)
    hs, arr = _open_hlls(client, names)
    buf = torch.zeros(3 * 16384, dtype=torch.uint8, device="cuda")
    _check(L.lib().rbx_hll_pack_registers(client.ctx, arr, 3, buf.data_ptr(), None))
    L.lib().rbx_synchronize(client.ctx)
    got = buf.cpu().numpy().reshape(3, 16384)
    for i in range(3):
        assert np.array_equal(got[i], refs[i])
    other = rng.integers(0, 20, size=(3, 16384), dtype=np.uint8)
    buf.copy_(torch.from_numpy(other.reshape(-1)).cuda())
    torch.cuda.synchronize()
    _check(L.lib().rbx_hll_unpack_max_registers(client.ctx, arr, 3, buf.data_ptr(), None))
    out = np.zeros(3, np.uint64)
    _check(L.lib().rbx_hll_count_each_handles(client.ctx, arr, 3, out.ctypes.data_as(L.u64p)))
    for i, nm in enumerate(names):
        want = np.maximum(refs[i], other[i])
        assert out[i] == O.hll_count(want)
        d = client.getHyperLogLog(nm).exportDense()
        assert np.array_equal(O.hll_dense_unpack(d[16:]), want)
    for h in hs:
        L.lib().rbx_hll_close(h)


def test_hll_unpack_max_keeps_sparse_strings(client, fresh):
    """The exchange step's register merge into sparse keys follows pfmergeCommand's write-back
    (hllSparseSet per register, ascending), so the stored strings equal the Redis restatement;
    a merge that outgrows hll-sparse-max-bytes promotes."""
    import torch

    rng = np.random.default_rng(26)
    names = [f"{fresh}-{i}" for i in range(3)]
    refs = []
    for nm in names:
        m = rng.integers(0, 256, size=(200, 16), dtype=np.uint8)
        client.getHyperLogLog(nm).addAll(Arena.fixed(m))
        r = O.RedisHll()
        r.pfadd(*O.fixed_arena(m))
        refs.append(r)
    hs, arr = _open_hlls(client, names)
    other = np.zeros((3, 16384), np.uint8)
    for i, n in enumerate((50, 300, 3000)):  # the third grows past the limit
        pos = rng.choice(16384, size=n, replace=False)
        other[i, pos] = rng.integers(1, 6, size=n)
    buf = torch.from_numpy(other.reshape(-1)).cuda()
    torch.cuda.synchronize()
    _check(L.lib().rbx_hll_unpack_max_registers(client.ctx, arr, 3, buf.data_ptr(), None))
    L.lib().rbx_synchronize(client.ctx)
    for i, nm in enumerate(names):
        refs[i].merge_from(np.maximum(refs[i].regs, other[i]), use_dense=False)
        s = client.getHyperLogLog(nm).exportString()
        assert s == refs[i].string(s[8:16]), i
    assert refs[2].dense.value and not refs[0].dense.value
    for h in hs:
        L.lib().rbx_hll_close(h)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


NH, PER = 6, 20_000


def _exchange_rank(rank, world, port, tag, result):
    """One process per 'GPU' (both on cuda:0): PFADD this rank's element slice of every HLL,
    create the HLLs in a rank-dependent order (different register-pool layouts), then the
    all-reduce exchange: pack in name order -> MAX all-reduce -> unpack_max."""
    import torch
    import torch.distributed as dist

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from redisson_amd.sharding import partition_elements

        c = RedissonClient(0)
        names = [f"{tag}-{i}" for i in range(NH)]
        order = list(range(NH)) if rank == 0 else list(reversed(range(NH)))
        # rank 1 also allocates (and frees) extra HLLs first, so its pool offsets differ
        if rank == 1:
            for j in range(3):
                c.getHyperLogLog(f"{tag}-pad{j}").add(b"x")
            c.getHyperLogLog(f"{tag}-pad1").delete()
        rng = np.random.default_rng(99)
        mats = [rng.integers(0, 256, size=(PER, 16), dtype=np.uint8) for _ in range(NH)]
        for i in order:
            lo, hi = partition_elements(PER, world, rank)
            c.getHyperLogLog(names[i]).addAll(Arena.fixed(mats[i][lo:hi]))
        hs, arr = _open_hlls(c, names)
        buf = torch.zeros(NH * 16384, dtype=torch.uint8, device="cuda")
        _check(L.lib().rbx_hll_pack_registers(c.ctx, arr, NH, buf.data_ptr(), None))
        L.lib().rbx_synchronize(c.ctx)
        host = buf.cpu()
        dist.all_reduce(host, op=dist.ReduceOp.MAX)  # what ncclAllReduce(ncclUint8, ncclMax) computes
        buf.copy_(host.cuda())
        torch.cuda.synchronize()
        _check(L.lib().rbx_hll_unpack_max_registers(c.ctx, arr, NH, buf.data_ptr(), None))
        out = np.zeros(NH, np.uint64)
        _check(L.lib().rbx_hll_count_each_handles(c.ctx, arr, NH, out.ctypes.data_as(L.u64p)))
        ok = True
        for i in range(NH):
            ref = O.hll_new()
            O.hll_pfadd(ref, *O.fixed_arena(mats[i]))
            d = c.getHyperLogLog(names[i]).exportDense()
            ok = ok and np.array_equal(O.hll_dense_unpack(d[16:]), ref) and out[i] == O.hll_count(ref)
        result[rank] = 1 if ok else 0
        for h in hs:
            L.lib().rbx_hll_close(h)
        c.shutdown()
    finally:
        dist.destroy_process_group()


def test_element_partitioned_exchange_two_processes(fresh):
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    result = ctx.Array("i", [0, 0])
    port = _free_port()
    procs = [ctx.Process(target=_exchange_rank, args=(r, 2, port, fresh, result)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=240)
        assert p.exitcode == 0, p.exitcode
    assert list(result) == [1, 1]


def test_size_in_memory(client, fresh):
    """sizeInMemory (M/RedissonBloomFilter.java:234-238): the bitmap and the config hash; the
    bitmap's share is its device allocation (bytes rounded to 256, plus the length-word tail)."""
    f = client.getBloomFilter(fresh)
    assert f.sizeInMemory() == 0
    f.tryInit(1000, 0.01)  # 9585 bits -> 1199 bytes -> 1280 allocated
    v0 = f.sizeInMemory()
    assert v0 > 0
    f.add(["a"])
    assert f.sizeInMemory() - v0 == 1280 + 256 + len(fresh)
    f.delete()
    assert f.sizeInMemory() == 0
