"""Host mirror of the reference's object API for this path, over librbx.so.

Names, argument meaning and error behaviour follow the Java API so code (and tests)
read like the reference's own:

  RedissonClient.getBloomFilter / getHyperLogLog   M/api/RedissonClient.java:272,283,1038,1049
  RBloomFilter   M/api/RBloomFilter.java:27-113     (impl M/RedissonBloomFilter.java)
  RHyperLogLog   M/api/RHyperLogLog.java:27-68      (impl M/RedissonHyperLogLog.java)

M/ = /root/reference/redisson/src/main/java/org/redisson/
"""
from __future__ import annotations

import ctypes as C
import threading
from collections.abc import Collection

import numpy as np

from . import _lib as L
from .codec import DEFAULT_CODEC, Codec
from .exceptions import IllegalArgumentException, raise_for
from .keys import Arena, _OneKey


def _check(rc: int) -> None:
    if rc != L.RBX_OK:
        raise_for(rc, L.last_error())


def _is_collection(x) -> bool:
    return isinstance(x, (list, tuple)) or (isinstance(x, Collection) and not isinstance(x, (str, bytes, bytearray)))


class RedissonClient:
    """Redisson.create(...) for one GPU (M/Redisson.java).  One engine context per device."""

    def __init__(self, device: int = 0):
        self._ctx = C.c_void_p()
        _check(L.lib().rbx_init(device, C.byref(self._ctx)))
        self.device = device
        self._lock = threading.Lock()

    @classmethod
    def create(cls, device: int = 0) -> "RedissonClient":
        return cls(device)

    @property
    def ctx(self):
        if not self._ctx:
            raise RuntimeError("client has been shut down")
        return self._ctx

    def getBloomFilter(self, name: str, codec: Codec | None = None) -> "RBloomFilter":
        return RBloomFilter(self, name, codec or DEFAULT_CODEC)

    def getHyperLogLog(self, name: str, codec: Codec | None = None) -> "RHyperLogLog":
        return RHyperLogLog(self, name, codec or DEFAULT_CODEC)

    def shutdown(self) -> None:
        if self._ctx:
            _check(L.lib().rbx_shutdown(self._ctx))
            self._ctx = C.c_void_p()

    def synchronize(self) -> None:
        _check(L.lib().rbx_synchronize(self.ctx))

    def stream(self) -> int:
        return L.lib().rbx_stream(self.ctx) or 0

    get_bloom_filter = getBloomFilter
    get_hyper_log_log = getHyperLogLog

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.shutdown()


def _config_name(name: str) -> str:
    """suffixName(name, "config") (M/RedissonObject.java): the config hash shares the name's slot."""
    return name + ":config" if "{" in name else "{" + name + "}:config"


class _Expirable:
    """RExpirable (M/RedissonExpirable.java:53-251) over rbx_pexpire / rbx_persist / rbx_pttl.
    Times are milliseconds; `_expire_keys()` lists the keys a timeout applies to."""

    _COND = {None: 0, "NX": 1, "XX": 2, "GT": 3, "LT": 4}

    def _pexpire(self, when_ms: int, absolute: bool, cond=None) -> bool:
        keys = [k.encode() for k in self._expire_keys()]
        arr = (C.c_char_p * len(keys))(*keys)
        r = C.c_int()
        _check(L.lib().rbx_pexpire(self._client.ctx, arr, len(keys), int(when_ms), int(absolute), self._COND[cond],
                                   C.byref(r)))
        return bool(r.value)

    def expire(self, ttl_ms: int) -> bool:
        """expire(Duration) :118-125 -- PEXPIRE on every key"""
        return self._pexpire(ttl_ms, False)

    def expireAt(self, unix_ms: int) -> bool:
        """expireAt(long) :58-65 -- PEXPIREAT"""
        return self._pexpire(unix_ms, True)

    def expireIfSet(self, ttl_ms: int) -> bool:
        """:138-145 -- PEXPIRE .. XX"""
        return self._pexpire(ttl_ms, False, "XX")

    def expireIfNotSet(self, ttl_ms: int) -> bool:
        """:148-155 -- PEXPIRE .. NX"""
        return self._pexpire(ttl_ms, False, "NX")

    def expireIfGreater(self, ttl_ms: int) -> bool:
        """PEXPIRE .. GT"""
        return self._pexpire(ttl_ms, False, "GT")

    def expireIfLess(self, ttl_ms: int) -> bool:
        """PEXPIRE .. LT"""
        return self._pexpire(ttl_ms, False, "LT")

    def clearExpire(self) -> bool:
        """clearExpireAsync :183-185 / :241-251 -- PERSIST"""
        keys = [k.encode() for k in self._expire_keys()]
        arr = (C.c_char_p * len(keys))(*keys)
        r = C.c_int()
        _check(L.lib().rbx_persist(self._client.ctx, arr, len(keys), C.byref(r)))
        return bool(r.value)

    def remainTimeToLive(self) -> int:
        """:188-195 -- PTTL name (-2 missing, -1 no timeout)"""
        out = C.c_int64()
        _check(L.lib().rbx_pttl(self._client.ctx, self._expire_keys()[0].encode(), C.byref(out)))
        return int(out.value)

    def getExpireTime(self) -> int:
        """:198-205 -- PEXPIRETIME name"""
        out = C.c_int64()
        _check(L.lib().rbx_pexpiretime(self._client.ctx, self._expire_keys()[0].encode(), C.byref(out)))
        return int(out.value)


class RBloomFilter(_Expirable):
    """M/RedissonBloomFilter.java.  size/hashIterations are cached like the reference's
    volatile fields (:61-62) and re-validated on every batch (addConfigCheck :207-213)."""

    def __init__(self, client: RedissonClient, name: str, codec: Codec):
        self._client = client
        self._name = name
        self._codec = codec
        self._size = 0
        self._k = 0

    # ---- naming --------------------------------------------------------------------
    def getName(self) -> str:
        return self._name

    def _bname(self) -> bytes:
        return self._name.encode("utf-8")

    # ---- init / config -----------------------------------------------------------------
    def tryInit(self, expectedInsertions: int, falseProbability: float) -> bool:
        """:262-300 -- False (and the existing config cached) when already initialized."""
        created = C.c_int()
        _check(L.lib().rbx_bloom_try_init(self._client.ctx, self._bname(), int(expectedInsertions),
                                          float(falseProbability), C.byref(created)))
        self._read_config()
        return bool(created.value)

    def tryInitRaw(self, size: int, hashIterations: int) -> bool:
        """Engine-level init with an explicit (size, k); reaches size = 2^32."""
        created = C.c_int()
        _check(L.lib().rbx_bloom_init_raw(self._client.ctx, self._bname(), int(size), int(hashIterations),
                                          C.byref(created)))
        self._read_config()
        return bool(created.value)

    def _config(self) -> L.RbxBloomConfig:
        cfg = L.RbxBloomConfig()
        _check(L.lib().rbx_bloom_read_config(self._client.ctx, self._bname(), C.byref(cfg)))
        return cfg

    def _read_config(self) -> None:  # readConfig() :240-255
        cfg = self._config()
        self._size = cfg.size
        self._k = cfg.hash_iterations

    def getSize(self) -> int:
        return int(self._config().size)

    def getHashIterations(self) -> int:
        return int(self._config().hash_iterations)

    def getExpectedInsertions(self) -> int:
        return int(self._config().expected_insertions)

    def getFalseProbability(self) -> float:
        return float(self._config().false_probability_str.decode())

    # ---- hot path ------------------------------------------------------------------
    def _encode_all(self, objects) -> Arena:
        return Arena([self._codec.encode(o) for o in objects])

    def _one(self, obj) -> "_OneKey":
        return _OneKey(self._codec.encode(obj))

    def _batch(self, fn, objects, flags: bool):
        if self._size == 0:  # :106-108
            self._read_config()
        a = objects if isinstance(objects, (Arena, _OneKey)) else self._encode_all(objects)
        out = np.zeros(max(a.n, 1), np.uint8) if flags else None
        cnt = C.c_uint64()
        _check(fn(self._client.ctx, self._bname(), self._size, self._k, a.ptr(),
                  out.ctypes.data_as(L.u8p) if flags else None, C.byref(cnt)))
        return (int(cnt.value), out[: a.n]) if flags else int(cnt.value)

    def add(self, objects):
        """add(T) -> bool  |  add(Collection<T>) -> long  (:99-137)"""
        if isinstance(objects, Arena) or _is_collection(objects):
            return self._batch(L.lib().rbx_bloom_add, objects, False)
        return self._batch(L.lib().rbx_bloom_add, self._one(objects), False) > 0

    def contains(self, objects):
        """contains(T) -> bool  |  contains(Collection<T>) -> long  (:153-201)"""
        if isinstance(objects, Arena) or _is_collection(objects):
            return self._batch(L.lib().rbx_bloom_contains, objects, False)
        return self._batch(L.lib().rbx_bloom_contains, self._one(objects), False) > 0

    def addEach(self, objects):
        """(count, per-key 'newly added' flags) -- engine extension of add(Collection)."""
        return self._batch(L.lib().rbx_bloom_add, objects, True)

    def containsEach(self, objects):
        """(count, per-key presence flags) -- engine extension of contains(Collection)."""
        return self._batch(L.lib().rbx_bloom_contains, objects, True)

    def count(self) -> int:
        """:215-227"""
        out = C.c_int64()
        _check(L.lib().rbx_bloom_count(self._client.ctx, self._bname(), C.byref(out)))
        self._read_config()
        return int(out.value)

    # ---- RObject / RExpirable --------------------------------------------------------
    def delete(self) -> bool:
        n = C.c_int()
        _check(L.lib().rbx_bloom_delete(self._client.ctx, self._bname(), C.byref(n)))
        return n.value > 0

    def isExists(self) -> bool:
        e = C.c_int()
        _check(L.lib().rbx_bloom_is_exists(self._client.ctx, self._bname(), C.byref(e)))
        return bool(e.value)

    def sizeInMemory(self) -> int:
        """:234-238 -- the bitmap and the config hash (engine bytes)"""
        out = C.c_uint64()
        _check(L.lib().rbx_bloom_size_in_memory(self._client.ctx, self._bname(), C.byref(out)))
        return int(out.value)

    def _expire_keys(self):
        # M/RedissonBloomFilter.java:303-314: the bitmap and its config hash
        return [self._name, _config_name(self._name)]

    def rename(self, newName: str) -> None:
        _check(L.lib().rbx_bloom_rename(self._client.ctx, self._bname(), newName.encode()))
        self._name = newName

    def renamenx(self, newName: str) -> bool:
        r = C.c_int()
        _check(L.lib().rbx_bloom_renamenx(self._client.ctx, self._bname(), newName.encode(), C.byref(r)))
        if r.value:
            self._name = newName
        return bool(r.value)

    # ---- persistence (Redis string format) ----------------------------------------------
    def exportBitmap(self) -> bytes:
        n = C.c_uint64()
        _check(L.lib().rbx_bloom_export(self._client.ctx, self._bname(), None, 0, C.byref(n)))
        buf = np.zeros(max(n.value, 1), np.uint8)
        _check(L.lib().rbx_bloom_export(self._client.ctx, self._bname(), buf.ctypes.data_as(L.u8p), n.value,
                                        C.byref(n)))
        return buf[: n.value].tobytes()

    def importBitmap(self, data: bytes) -> None:
        buf = np.frombuffer(data, np.uint8) if data else np.zeros(1, np.uint8)
        _check(L.lib().rbx_bloom_import(self._client.ctx, self._bname(), buf.ctypes.data_as(L.u8p), len(data)))

    def digest(self) -> int:
        """Order-independent 64-bit digest of `GET name` (0 = no bitmap): replica comparison."""
        out = C.c_uint64()
        _check(L.lib().rbx_bloom_digest(self._client.ctx, self._bname(), C.byref(out)))
        return int(out.value)

    def bitcount(self) -> int:
        out = C.c_uint64()
        _check(L.lib().rbx_bloom_bitcount(self._client.ctx, self._bname(), C.byref(out)))
        return int(out.value)

    # snake_case aliases
    try_init = tryInit
    get_size = getSize
    get_hash_iterations = getHashIterations
    is_exists = isExists


class BloomHandle:
    """Open handle for the device-resident batch path (rbx_bloom_*_dev)."""

    def __init__(self, client: RedissonClient, name: str):
        self._client = client
        self.h = C.c_void_p()
        _check(L.lib().rbx_bloom_open(client.ctx, name.encode(), C.byref(self.h)))
        s, k = C.c_uint64(), C.c_uint32()
        _check(L.lib().rbx_bloom_handle_config(self.h, C.byref(s), C.byref(k)))
        self.size, self.k = int(s.value), int(k.value)

    def contains_dev(self, keys: L.RbxKeys, d_count: int, d_out: int | None = None, stream: int | None = None):
        _check(L.lib().rbx_bloom_contains_dev(self._client.ctx, self.h, C.byref(keys), d_out, d_count, stream))

    def add_dev(self, keys: L.RbxKeys, d_count: int, d_out: int | None = None, stream: int | None = None):
        _check(L.lib().rbx_bloom_add_dev(self._client.ctx, self.h, C.byref(keys), d_out, d_count, stream))

    def close(self):
        if self.h:
            _check(L.lib().rbx_bloom_close(self.h))
            self.h = C.c_void_p()


def _handles(hs):
    arr = (C.c_void_p * len(hs))(*[h.h.value for h in hs])
    return arr


def bloom_contains_multi(client: RedissonClient, handles: list[BloomHandle], seg_offsets: np.ndarray,
                         arena: Arena, per_key: bool = False):
    """One contains(Collection) per segment (multi-tenant host path)."""
    nseg = len(handles)
    seg = np.ascontiguousarray(seg_offsets, dtype=np.uint64)
    counts = np.zeros(nseg, np.uint64)
    out = np.zeros(max(arena.n, 1), np.uint8) if per_key else None
    _check(L.lib().rbx_bloom_contains_multi(client.ctx, _handles(handles), nseg, seg.ctypes.data_as(L.u64p),
                                            arena.ptr(), out.ctypes.data_as(L.u8p) if per_key else None,
                                            counts.ctypes.data_as(L.u64p)))
    return (counts, out[: arena.n]) if per_key else counts


def bloom_add_multi(client: RedissonClient, handles: list[BloomHandle], seg_offsets: np.ndarray,
                    arena: Arena, per_key: bool = False):
    """One add(Collection) per segment, applied in segment order (multi-tenant host path)."""
    nseg = len(handles)
    seg = np.ascontiguousarray(seg_offsets, dtype=np.uint64)
    counts = np.zeros(nseg, np.uint64)
    out = np.zeros(max(arena.n, 1), np.uint8) if per_key else None
    _check(L.lib().rbx_bloom_add_multi(client.ctx, _handles(handles), nseg, seg.ctypes.data_as(L.u64p),
                                       arena.ptr(), out.ctypes.data_as(L.u8p) if per_key else None,
                                       counts.ctypes.data_as(L.u64p)))
    return (counts, out[: arena.n]) if per_key else counts


def bloom_stream(client: RedissonClient, handles: list[BloomHandle], key_filter, key_op, arena: Arena):
    """Ordered mixed stream of single-key contains (op 0) / add (op 1) commands on
    handles[key_filter[i]]; returns (per-key results, [present contains, newly added])."""
    kf = np.ascontiguousarray(key_filter, dtype=np.uint32)
    op = np.ascontiguousarray(key_op, dtype=np.uint8)
    out = np.zeros(max(arena.n, 1), np.uint8)
    counts = np.zeros(2, np.uint64)
    _check(L.lib().rbx_bloom_stream(client.ctx, _handles(handles), len(handles), kf.ctypes.data_as(L.u32p),
                                    op.ctypes.data_as(L.u8p), arena.ptr(), out.ctypes.data_as(L.u8p),
                                    counts.ctypes.data_as(L.u64p)))
    return out[: arena.n], counts


class RFuture:
    """org.redisson.api.RFuture over an rbx_future: the asynchronous call runs on the context's
    serial executor; get() waits and returns the converted result (or raises the call's error)."""

    def __init__(self, fut: C.c_void_p, convert, keep):
        self._f = fut
        self._convert = convert
        self._keep = keep  # buffers the call reads / writes until it completes
        self._done = False

    def isDone(self) -> bool:
        d = C.c_int()
        _check(L.lib().rbx_future_done(self._f, C.byref(d)))
        return bool(d.value)

    def get(self, timeout_ms: int = -1):
        """Result of the call; TimeoutError if it has not completed within timeout_ms."""
        rc = C.c_int()
        r = L.lib().rbx_future_wait(self._f, int(timeout_ms), C.byref(rc))
        if r == L.RBX_E_TIMEOUT:
            raise TimeoutError("the call has not completed")
        _check(r)
        _check(rc.value)
        return self._convert()

    def __del__(self):
        f = getattr(self, "_f", None)
        if f:
            try:
                L.lib().rbx_future_wait(f, -1, None)  # the buffers in _keep must outlive the call
                L.lib().rbx_future_free(f)
            except Exception:  # interpreter shutdown
                pass

    is_done = isDone


class RHyperLogLog(_Expirable):
    """M/RedissonHyperLogLog.java (PFADD / PFCOUNT / PFMERGE) and RHyperLogLogAsync
    (M/api/RHyperLogLogAsync.java:37-70: the *Async methods return an RFuture)."""

    def __init__(self, client: RedissonClient, name: str, codec: Codec):
        self._client = client
        self._name = name
        self._codec = codec

    def getName(self) -> str:
        return self._name

    def add(self, obj) -> bool:
        """:71-73 PFADD name e"""
        return self.addAll(_OneKey(self._codec.encode(obj)))

    def addAll(self, objects) -> bool:
        """:76-81 PFADD name e1..en"""
        a = objects if isinstance(objects, (Arena, _OneKey)) else Arena([self._codec.encode(o) for o in objects])
        ch = C.c_int()
        _check(L.lib().rbx_hll_add(self._client.ctx, self._name.encode(), a.ptr(), C.byref(ch)))
        return bool(ch.value)

    def count(self) -> int:
        """:84-86 PFCOUNT name"""
        return self.countWith()

    def countWith(self, *otherLogNames: str) -> int:
        """:89-94 PFCOUNT name o1..on"""
        names = [self._name, *otherLogNames]
        arr = (C.c_char_p * len(names))(*[n.encode() for n in names])
        out = C.c_uint64()
        _check(L.lib().rbx_hll_count(self._client.ctx, arr, len(names), C.byref(out)))
        return int(out.value)

    def mergeWith(self, *otherLogNames: str) -> None:
        """:97-102 PFMERGE name o1..on"""
        arr = (C.c_char_p * max(len(otherLogNames), 1))(*[n.encode() for n in otherLogNames])
        _check(L.lib().rbx_hll_merge(self._client.ctx, self._name.encode(), arr, len(otherLogNames)))

    # ---- RHyperLogLogAsync ------------------------------------------------------------------
    def addAsync(self, obj) -> RFuture:
        return self.addAllAsync([obj])

    def addAllAsync(self, objects) -> RFuture:
        a = objects if isinstance(objects, Arena) else Arena([self._codec.encode(o) for o in objects])
        ch = C.c_int()
        f = C.c_void_p()
        _check(L.lib().rbx_hll_add_async(self._client.ctx, self._name.encode(), a.ptr(), C.byref(ch), None, None,
                                         C.byref(f)))
        return RFuture(f, lambda: bool(ch.value), (a, ch))

    def countAsync(self) -> RFuture:
        return self.countWithAsync()

    def countWithAsync(self, *otherLogNames: str) -> RFuture:
        names = [self._name, *otherLogNames]
        arr = (C.c_char_p * len(names))(*[n.encode() for n in names])
        out = C.c_uint64()
        f = C.c_void_p()
        _check(L.lib().rbx_hll_count_async(self._client.ctx, arr, len(names), C.byref(out), None, None, C.byref(f)))
        return RFuture(f, lambda: int(out.value), (arr, out))

    def mergeWithAsync(self, *otherLogNames: str) -> RFuture:
        arr = (C.c_char_p * max(len(otherLogNames), 1))(*[n.encode() for n in otherLogNames])
        f = C.c_void_p()
        _check(L.lib().rbx_hll_merge_async(self._client.ctx, self._name.encode(), arr, len(otherLogNames), None,
                                           None, C.byref(f)))
        return RFuture(f, lambda: None, (arr,))

    def delete(self) -> bool:
        n = C.c_int()
        _check(L.lib().rbx_hll_delete(self._client.ctx, self._name.encode(), C.byref(n)))
        return n.value > 0

    def isExists(self) -> bool:
        e = C.c_int()
        _check(L.lib().rbx_hll_exists(self._client.ctx, self._name.encode(), C.byref(e)))
        return bool(e.value)

    def _expire_keys(self):
        return [self._name]

    def exportDense(self) -> bytes:
        """GET name, as the Redis dense HLL string."""
        n = C.c_uint64()
        buf = np.zeros(16 + 12288, np.uint8)
        _check(L.lib().rbx_hll_export(self._client.ctx, self._name.encode(), buf.ctypes.data_as(L.u8p),
                                      buf.size, C.byref(n)))
        return buf[: n.value].tobytes()

    _ENCODINGS = {"dense": 0, "sparse": 1, "stored": 2}

    def exportString(self, encoding: str = "stored") -> bytes:
        """GET name as a Redis HLL string: "stored" = the encoding Redis would hold (sparse until
        promoted), "dense", or "sparse" (IllegalArgumentException if a register exceeds 32).
        Empty bytes if the key does not exist."""
        if encoding not in self._ENCODINGS:
            raise IllegalArgumentException("encoding must be one of %s" % sorted(self._ENCODINGS))
        n = C.c_uint64()
        buf = np.zeros(16 + 12288, np.uint8)
        _check(L.lib().rbx_hll_export_enc(self._client.ctx, self._name.encode(), self._ENCODINGS[encoding],
                                          buf.ctypes.data_as(L.u8p), buf.size, C.byref(n)))
        return buf[: n.value].tobytes()

    def importString(self, data: bytes) -> None:
        """SET name <Redis HLL string> (dense or sparse)."""
        buf = np.frombuffer(data, np.uint8)
        _check(L.lib().rbx_hll_import(self._client.ctx, self._name.encode(), buf.ctypes.data_as(L.u8p), len(data)))

    add_all = addAll
    count_with = countWith
    merge_with = mergeWith
    add_all_async = addAllAsync
    count_async = countAsync
    merge_with_async = mergeWithAsync


def hll_add_multi(client: RedissonClient, names: list[str], seg_offsets, arena: Arena) -> np.ndarray:
    """A pipeline of PFADD commands (segment s -> names[s]); returns each reply."""
    nseg = len(names)
    arr = (C.c_char_p * nseg)(*[n.encode() for n in names])
    seg = np.ascontiguousarray(seg_offsets, dtype=np.uint64)
    out = np.zeros(max(nseg, 1), np.uint8)
    _check(L.lib().rbx_hll_add_multi(client.ctx, arr, nseg, seg.ctypes.data_as(L.u64p), arena.ptr(),
                                     out.ctypes.data_as(L.u8p)))
    return out[:nseg]


def hll_count_each(client: RedissonClient, names: list[str]) -> np.ndarray:
    n = len(names)
    arr = (C.c_char_p * max(n, 1))(*[x.encode() for x in names])
    out = np.zeros(max(n, 1), np.uint64)
    _check(L.lib().rbx_hll_count_each(client.ctx, arr, n, out.ctypes.data_as(L.u64p)))
    return out[:n]


def crc16(data: bytes) -> int:
    b = (C.c_uint8 * max(1, len(data))).from_buffer_copy(data or b"\0")
    return int(L.lib().rbx_crc16(b, len(data)))


def calc_slot(key: bytes | str) -> int:
    """ClusterConnectionManager.calcSlot (M/cluster/ClusterConnectionManager.java:777-830)."""
    if isinstance(key, str):
        key = key.encode("utf-8")
    b = (C.c_uint8 * max(1, len(key))).from_buffer_copy(key or b"\0")
    return int(L.lib().rbx_calc_slot(b, len(key)))


def slot_to_gpu(slot: int, n_gpus: int) -> int:
    return int(L.lib().rbx_slot_to_gpu(slot, n_gpus))
