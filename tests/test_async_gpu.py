"""RHyperLogLogAsync (M/api/RHyperLogLogAsync.java:37-70) over the *_async entry points: results
equal the synchronous calls and the oracle, calls on one context run in submission order, errors
and callbacks reach the caller."""
import ctypes as C

import numpy as np
import pytest

from oracle import oracle as O
from redisson_amd import Arena, RedisException
from redisson_amd import _lib as L

pytestmark = pytest.mark.gpu


def test_hll_async_methods(client, fresh):
    rng = np.random.default_rng(51)
    a, b = fresh + "a", fresh + "b"
    ea = [rng.bytes(16) for _ in range(20_000)]
    eb = [rng.bytes(16) for _ in range(7_000)]
    ha, hb = client.getHyperLogLog(a), client.getHyperLogLog(b)
    # queued in order: the count sees both adds, the union and the merge see everything before them
    futs = [ha.addAllAsync(ea), hb.addAllAsync(eb), ha.addAsync(ea[0]), ha.countAsync(), ha.countWithAsync(b),
            hb.mergeWithAsync(a), hb.countAsync()]
    res = [f.get(timeout_ms=60_000) for f in futs]
    ra, rb = O.hll_new(), O.hll_new()
    O.hll_pfadd(ra, *O.arena(ea))
    O.hll_pfadd(rb, *O.arena(eb))
    u = ra.copy()
    O.hll_merge(u, rb)
    assert res[:3] == [True, True, False]
    assert res[3] == O.hll_count(ra)
    assert res[4] == O.hll_count(u)
    assert res[5] is None and res[6] == O.hll_count(u)
    assert all(f.isDone() for f in futs)
    assert ha.count() == res[3]


def test_async_error_and_callback(client, fresh):
    f = client.getBloomFilter(fresh)
    f.tryInit(1000, 0.01)
    f.add(["x"])  # `fresh` now holds a bitmap: PFADD on it is WRONGTYPE
    fut = client.getHyperLogLog(fresh).addAllAsync([b"e"])
    with pytest.raises(RedisException, match="WRONGTYPE"):
        fut.get()
    # C callback: rc of each completed call, in submission order
    seen = []
    CB = C.CFUNCTYPE(None, C.c_void_p, C.c_int)
    cb = CB(lambda user, rc: seen.append((user, rc)))
    keys = Arena([b"k1", b"k2"])
    cnt = C.c_uint64()
    fs = []
    for i in range(1, 6):
        fp = C.c_void_p()
        assert L.lib().rbx_bloom_contains_async(client.ctx, fresh.encode(), 0, 0, keys.ptr(), None, C.byref(cnt),
                                                C.cast(cb, C.c_void_p), C.c_void_p(i), C.byref(fp)) == 0
        fs.append(fp)
    for fp in fs:
        rc = C.c_int(-99)
        assert L.lib().rbx_future_wait(fp, -1, C.byref(rc)) == 0 and rc.value == 0
        L.lib().rbx_future_free(fp)
    assert [u for u, _ in seen] == [1, 2, 3, 4, 5] and all(rc == 0 for _, rc in seen)
    assert cnt.value == 0  # neither key was added
    f.delete()


def test_async_bloom_add_then_contains_in_order(client, fresh):
    rng = np.random.default_rng(52)
    f = client.getBloomFilter(fresh)
    f.tryInit(100_000, 0.01)
    f._read_config()
    mat = rng.integers(0, 256, size=(50_000, 32), dtype=np.uint8)
    a = Arena.fixed(mat)
    new = np.zeros(50_000, np.uint8)
    pres = np.zeros(50_000, np.uint8)
    c1, c2 = C.c_uint64(), C.c_uint64()
    f1, f2 = C.c_void_p(), C.c_void_p()
    assert L.lib().rbx_bloom_add_async(client.ctx, fresh.encode(), f._size, f._k, a.ptr(), new.ctypes.data,
                                       C.byref(c1), None, None, C.byref(f1)) == 0
    assert L.lib().rbx_bloom_contains_async(client.ctx, fresh.encode(), f._size, f._k, a.ptr(), pres.ctypes.data,
                                            C.byref(c2), None, None, C.byref(f2)) == 0
    for fp in (f1, f2):
        rc = C.c_int()
        assert L.lib().rbx_future_wait(fp, 60_000, C.byref(rc)) == 0 and rc.value == 0
        L.lib().rbx_future_free(fp)
    ref = O.OracleBloom(f._size, f._k)
    cr, nr = ref.add(*O.fixed_arena(mat), per_key=True)
    assert c1.value == cr and np.array_equal(new, nr)
    assert c2.value == 50_000 and pres.all()
    f.delete()


def _wait_all(futs):
    """(accepted rc list) -- every accepted future completes; none hangs."""
    out = []
    for fp in futs:
        rc = C.c_int(-99)
        assert L.lib().rbx_future_wait(fp, 60_000, C.byref(rc)) == 0, "an accepted call never completed"
        out.append(rc.value)
        L.lib().rbx_future_free(fp)
    return out


def test_async_submit_races_shutdown():
    """*_async submits on several threads while another thread shuts the context down.
    Every submit is either accepted (and its future completes: OK, or ILLEGAL_STATE when it ran after
    the shutdown) or refused with RBX_E_ILLEGAL_STATE; nothing hangs or touches a freed executor."""
    import threading

    from redisson_amd import RedissonClient

    c = RedissonClient(0)
    ctx = c.ctx
    c.getHyperLogLog("race").add(b"x")
    # an open handle keeps the context object alive past rbx_shutdown (calls then fail cleanly)
    hold = C.c_void_p()
    assert L.lib().rbx_hll_open(ctx, b"race", 1, C.byref(hold)) == 0
    accepted, refused, outs, lock = [], [], [], threading.Lock()
    keys = Arena([b"a", b"b", b"c"])

    def submitter():
        for _ in range(300):
            fp = C.c_void_p()
            changed = C.c_int()
            rc = L.lib().rbx_hll_add_async(ctx, b"race", keys.ptr(), C.byref(changed), None, None, C.byref(fp))
            with lock:
                (accepted if rc == 0 else refused).append(fp if rc == 0 else rc)
                outs.append(changed)  # written when the call runs: must outlive it

    th = [threading.Thread(target=submitter) for _ in range(4)]
    for t in th:
        t.start()
    c.shutdown()
    for t in th:
        t.join()
    assert all(r == L.RBX_E_ILLEGAL_STATE for r in refused)
    rcs = _wait_all(accepted)
    assert all(r in (0, L.RBX_E_ILLEGAL_STATE) for r in rcs)
    assert len(accepted) + len(refused) == 1200
    assert L.lib().rbx_hll_close(hold) == 0


def test_shutdown_from_completion_callback():
    """a completion callback (the executor's own thread) calls rbx_shutdown.  The call
    returns, the executor is released from inside instead of joining itself, calls queued behind it
    complete (with RBX_E_ILLEGAL_STATE: the context is shut), and later submits are refused."""
    from redisson_amd import RedissonClient

    c = RedissonClient(0)
    ctx = c.ctx
    hold = C.c_void_p()
    assert L.lib().rbx_hll_open(ctx, b"cbshut", 1, C.byref(hold)) == 0  # keeps the context object alive
    state = {}
    CB = C.CFUNCTYPE(None, C.c_void_p, C.c_int)

    def on_done(user, rc):
        if user == 1:
            state["shutdown_rc"] = L.lib().rbx_shutdown(ctx)

    cb = CB(on_done)
    keys = Arena([b"k"])
    futs, outs = [], []
    for i in range(1, 6):
        fp = C.c_void_p()
        changed = C.c_int()
        assert L.lib().rbx_hll_add_async(ctx, b"cbshut", keys.ptr(), C.byref(changed), C.cast(cb, C.c_void_p),
                                         C.c_void_p(i), C.byref(fp)) in (0, L.RBX_E_ILLEGAL_STATE)
        outs.append(changed)  # written when the call runs: must outlive it
        if fp.value:
            futs.append(fp)
    rcs = _wait_all(futs)
    assert rcs[0] == 0 and state["shutdown_rc"] == 0
    assert all(r in (0, L.RBX_E_ILLEGAL_STATE) for r in rcs[1:])
    fp = C.c_void_p()
    changed = C.c_int()
    assert L.lib().rbx_hll_add_async(ctx, b"cbshut", keys.ptr(), C.byref(changed), None, None,
                                     C.byref(fp)) == L.RBX_E_ILLEGAL_STATE
    assert L.lib().rbx_hll_close(hold) == 0
    c._ctx = C.c_void_p()  # already shut from the callback
