"""Key timeouts (RExpirable, M/RedissonExpirable.java:53-251) on the engine's keyspace.

RBloomFilter applies a timeout to the bitmap and its config hash together
(M/RedissonBloomFilter.java:303-314); RHyperLogLog to its one key.  Per key the rules are Redis
7.2's PEXPIRE / PEXPIREAT / PERSIST / PTTL: NX / XX / GT / LT conditions (no timeout counts as
infinite), a time not in the future deletes the key, keys disappear lazily once expired, and
RENAME keeps the timeout.  T/ = redisson/src/test/java/org/redisson/ (T/RedissonBloomFilterTest.java
:99-110 exercises expire on a filter).
"""
import time

import numpy as np
import pytest

from redisson_amd import Arena, BloomHandle, IllegalStateException, RedisException

pytestmark = pytest.mark.gpu


def _filter(client, name, n=1000):
    f = client.getBloomFilter(name)
    assert f.tryInit(100_000, 0.01)
    rng = np.random.default_rng(len(name))
    keys = [rng.bytes(16) for _ in range(n)]
    if n:
        assert f.add(Arena(keys)) == n
    return f, keys


def test_bloom_expire_removes_both_keys(client, fresh):
    f, keys = _filter(client, fresh)
    assert f.remainTimeToLive() == -1
    assert f.expire(300)
    ttl = f.remainTimeToLive()
    assert 0 < ttl <= 300
    from redisson_amd import _lib as L
    import ctypes as C

    out = C.c_int64()
    assert L.lib().rbx_pttl(client.ctx, ("{%s}:config" % fresh).encode(), C.byref(out)) == 0
    assert 0 < out.value <= 300  # the config hash carries the same timeout
    assert abs(f.getExpireTime() - (int(time.time() * 1000) + ttl)) < 1000
    assert f.contains(Arena(keys)) == len(keys)
    time.sleep(0.45)
    assert not f.isExists()
    assert f.remainTimeToLive() == -2
    # the cached (size, k) no longer match a config: addConfigCheck fails (:207-213)
    with pytest.raises(RedisException):
        f.contains(Arena(keys))
    # a fresh object has no cached config: readConfig finds none (:240-255)
    with pytest.raises(IllegalStateException):
        client.getBloomFilter(fresh).contains(Arena(keys))
    # and the name can be initialized again
    g = client.getBloomFilter(fresh)
    assert g.tryInit(1000, 0.01)
    assert g.contains(Arena(keys)) == 0
    g.delete()


def test_bloom_clear_expire_and_conditions(client, fresh):
    f, _ = _filter(client, fresh)
    assert not f.expireIfSet(10_000)      # XX: no timeout yet
    assert f.expireIfNotSet(10_000)       # NX
    assert not f.expireIfNotSet(20_000)   # NX: already has one
    assert f.expireIfSet(20_000)          # XX
    assert f.expireIfGreater(30_000)      # GT: later
    assert not f.expireIfGreater(5_000)   # GT: earlier
    assert f.expireIfLess(5_000)          # LT: earlier
    assert not f.expireIfLess(60_000)     # LT: later
    assert 0 < f.remainTimeToLive() <= 5_000
    assert f.clearExpire()
    assert f.remainTimeToLive() == -1
    assert not f.clearExpire()            # PERSIST on a key without timeout
    assert not f.expireIfGreater(10_000)  # GT: no timeout = infinite
    assert f.expireIfLess(10_000)         # LT: anything is less than infinite
    f.delete()


def test_expire_in_the_past_deletes(client, fresh):
    f, _ = _filter(client, fresh)
    assert f.expire(0)
    assert not f.isExists()
    f2, _ = _filter(client, fresh + "b")
    assert f2.expireAt(int(time.time() * 1000) - 1000)
    assert not f2.isExists()
    # missing keys: nothing to set
    assert not client.getBloomFilter(fresh + "none").expire(1000)
    assert client.getBloomFilter(fresh + "none").remainTimeToLive() == -2


def test_rename_keeps_timeout(client, fresh):
    f, keys = _filter(client, fresh)
    assert f.expire(50_000)
    f.rename(fresh + "r")
    assert 0 < f.remainTimeToLive() <= 50_000
    assert f.contains(Arena(keys)) == len(keys)
    f.delete()


def test_handles_follow_their_name(client, fresh):
    """A device-path handle re-resolves its name when the keyspace changes: after the filter
    expires the cached config check fails, as Redisson's addConfigCheck does."""
    import torch

    from redisson_amd import device_keys

    f, keys = _filter(client, fresh, n=0)
    h = BloomHandle(client, fresh)
    mat = np.frombuffer(b"".join(np.random.default_rng(3).bytes(32) for _ in range(4096)), np.uint8).reshape(-1, 32)
    d = torch.from_numpy(mat.copy()).cuda()
    cnt = torch.zeros(2, dtype=torch.int64, device="cuda")
    torch.cuda.synchronize()
    h.add_dev(device_keys(d.data_ptr(), len(mat), 32), cnt.data_ptr())
    h.contains_dev(device_keys(d.data_ptr(), len(mat), 32), cnt.data_ptr() + 8)
    torch.cuda.synchronize()
    assert cnt.tolist()[1] == len(mat)
    assert f.expire(150)
    time.sleep(0.3)
    with pytest.raises(RedisException):
        h.contains_dev(device_keys(d.data_ptr(), len(mat), 32), cnt.data_ptr() + 8)
    h.close()


def test_hll_expire(client, fresh):
    h = client.getHyperLogLog(fresh)
    assert h.addAll([b"a", b"b", b"c"])
    assert h.count() == 3
    assert h.expire(200)
    assert 0 < h.remainTimeToLive() <= 200
    time.sleep(0.35)
    assert not h.isExists()
    assert h.count() == 0
    assert h.add(b"x")  # PFADD creates the key again, without a timeout
    assert h.count() == 1 and h.remainTimeToLive() == -1
    h.delete()
