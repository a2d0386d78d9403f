"""ctypes/numpy front end of the CPU oracle (oracle/rbx_oracle.c).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg -- never by the product package redisson_amd/.

Every function restates a reference item; see the citations in rbx_oracle.c
(M/ = /root/reference/redisson/src/main/java/org/redisson/).
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_SO = os.path.join(_HERE, "_build", "liborc.so")

u8p = C.POINTER(C.c_uint8)
u64p = C.POINTER(C.c_uint64)
i64p = C.POINTER(C.c_int64)

REDISSON_MAX_SIZE = 2147483647 * 2  # RedissonBloomFilter.getMaxSize(), :257-259
HLL_REGISTERS = 16384


def build() -> None:
    """Compile liborc.so (gcc only; cheap, idempotent)."""
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


def _load():
    if not os.path.exists(_SO):
        build()
    lib = C.CDLL(_SO)
    sig = {
        "orc_highway_hash64": (C.c_uint64, [u8p, C.c_size_t, u64p]),
        "orc_highway_hash128": (None, [u8p, C.c_size_t, u64p, u64p]),
        "orc_redisson_hash128": (None, [u8p, C.c_size_t, u64p]),
        "orc_java_math_round": (C.c_int64, [C.c_double]),
        "orc_bloom_optimal": (C.c_int, [C.c_int64, C.c_double, C.c_int64, i64p, C.POINTER(C.c_int32)]),
        "orc_bloom_indexes": (None, [C.c_uint64, C.c_uint64, C.c_int, C.c_int64, i64p]),
        "orc_bloom_hash_batch": (None, [u8p, u64p, C.c_uint64, C.c_int, C.c_int64, i64p]),
        "orc_bloom_add": (C.c_int64, [u8p, u64p, u8p, u64p, C.c_uint64, C.c_int, C.c_int64, u8p]),
        "orc_bloom_contains": (C.c_int64, [u8p, C.c_uint64, u8p, u64p, C.c_uint64, C.c_int, C.c_int64, u8p]),
        "orc_bitcount": (C.c_uint64, [u8p, C.c_uint64]),
        "orc_bloom_count_estimate": (C.c_int64, [C.c_uint64, C.c_int64, C.c_int]),
        "orc_crc16": (C.c_uint16, [u8p, C.c_size_t]),
        "orc_calc_slot": (C.c_int, [u8p, C.c_size_t]),
        "orc_murmur64a": (C.c_uint64, [u8p, C.c_int, C.c_uint64]),
        "orc_hll_patlen": (C.c_int, [u8p, C.c_size_t, C.POINTER(C.c_long)]),
        "orc_hll_pfadd": (C.c_int, [u8p, u8p, u64p, C.c_uint64]),
        "orc_hll_dense_pack": (None, [u8p, u8p]),
        "orc_hll_dense_unpack": (None, [u8p, u8p]),
        "orc_hll_count_histo": (C.c_uint64, [C.POINTER(C.c_int)]),
        "orc_hll_histogram": (None, [u8p, C.POINTER(C.c_int)]),
        "orc_hll_count": (C.c_uint64, [u8p]),
        "orc_hll_merge": (None, [u8p, u8p]),
        "orc_hll_sparse_set": (C.c_int, [u8p, C.POINTER(C.c_size_t), C.c_size_t, C.c_long, C.c_int, C.c_size_t]),
        "orc_hll_sparse_new": (C.c_size_t, [u8p]),
        "orc_hll_sparse_pfadd": (C.c_int, [u8p, C.POINTER(C.c_size_t), C.c_size_t, C.POINTER(C.c_int), u8p, u8p,
                                           u64p, C.c_uint64, C.c_size_t]),
        "orc_hll_sparse_merge": (C.c_int, [u8p, C.POINTER(C.c_size_t), C.c_size_t, C.POINTER(C.c_int), u8p,
                                           C.c_size_t]),
        "orc_murmur_batch": (None, [u8p, u64p, C.c_uint64, u64p]),
        "orc_bloom_contains_mt": (C.c_int64, [u8p, C.c_uint64, u8p, u64p, C.c_uint64, C.c_int, C.c_int64, u8p,
                                              C.c_int]),
        "orc_bloom_add_mt": (C.c_int64, [u8p, u64p, u8p, u64p, C.c_uint64, C.c_int, C.c_int64, u8p, C.c_int]),
        "orc_hash128_batch": (None, [u8p, u64p, C.c_uint64, u64p]),
        "orc_bloom_stream": (None, [C.POINTER(u8p), u64p, i64p, C.POINTER(C.c_int32), C.POINTER(C.c_uint32), u8p,
                                    u8p, u64p, C.c_uint64, C.c_uint64, u8p, u64p]),
    }
    for name, (res, args) in sig.items():
        f = getattr(lib, name)
        f.restype = res
        f.argtypes = args
    return lib


_lib = None


def lib():
    global _lib
    if _lib is None:
        _lib = _load()
    return _lib


def _p(a: np.ndarray, t=u8p):
    return a.ctypes.data_as(t)


def arena(keys) -> tuple[np.ndarray, np.ndarray]:
    """list[bytes] -> (bytes u8[], offsets u64[n+1]) -- the engine's key-arena layout."""
    offs = np.zeros(len(keys) + 1, dtype=np.uint64)
    if keys:
        offs[1:] = np.cumsum([len(k) for k in keys], dtype=np.uint64)
    buf = np.frombuffer(b"".join(keys), dtype=np.uint8).copy() if keys else np.zeros(1, np.uint8)
    if buf.size == 0:
        buf = np.zeros(1, np.uint8)
    return buf, offs


def fixed_arena(mat: np.ndarray) -> tuple[np.ndarray, np.ndarray]:
    """uint8[n, L] -> arena (contiguous bytes, offsets i*L)."""
    n, L = mat.shape
    return np.ascontiguousarray(mat).reshape(-1), (np.arange(n + 1, dtype=np.uint64) * np.uint64(L))


# ---- HighwayHash -------------------------------------------------------------------

def highway_hash64(data: bytes, key) -> int:
    k = (C.c_uint64 * 4)(*key)
    b = (C.c_uint8 * max(1, len(data))).from_buffer_copy(data or b"\0")
    return lib().orc_highway_hash64(b, len(data), k)


def highway_hash128(data: bytes, key) -> tuple[int, int]:
    k = (C.c_uint64 * 4)(*key)
    o = (C.c_uint64 * 2)()
    b = (C.c_uint8 * max(1, len(data))).from_buffer_copy(data or b"\0")
    lib().orc_highway_hash128(b, len(data), k, o)
    return o[0], o[1]


def redisson_hash128(data: bytes) -> tuple[int, int]:
    """Hash.hash128 (M/misc/Hash.java:53-74)."""
    o = (C.c_uint64 * 2)()
    b = (C.c_uint8 * max(1, len(data))).from_buffer_copy(data or b"\0")
    lib().orc_redisson_hash128(b, len(data), o)
    return o[0], o[1]


def hash128_batch(buf: np.ndarray, offs: np.ndarray) -> np.ndarray:
    n = offs.size - 1
    out = np.zeros(2 * max(n, 1), dtype=np.uint64)
    lib().orc_hash128_batch(_p(buf), _p(offs, u64p), n, _p(out, u64p))
    return out[: 2 * n].reshape(n, 2)


# ---- Bloom -------------------------------------------------------------------------

class OracleError(Exception):
    pass


def bloom_optimal(n: int, p: float, max_size: int = REDISSON_MAX_SIZE) -> tuple[int, int]:
    """tryInit sizing (RedissonBloomFilter.java:79-88, :262-277).  Raises on IAE."""
    s = C.c_int64()
    k = C.c_int32()
    rc = lib().orc_bloom_optimal(n, p, max_size, C.byref(s), C.byref(k))
    if rc != 0:
        raise OracleError("IllegalArgumentException")
    return s.value, k.value


def bloom_indexes(h1: int, h2: int, k: int, size: int) -> list[int]:
    out = (C.c_int64 * k)()
    lib().orc_bloom_indexes(h1, h2, k, size, out)
    return list(out)


def bloom_hash_batch(buf, offs, k, size) -> np.ndarray:
    n = offs.size - 1
    out = np.zeros(max(n, 1) * k, dtype=np.int64)
    lib().orc_bloom_hash_batch(_p(buf), _p(offs, u64p), n, k, size, _p(out, i64p))
    return out[: n * k].reshape(n, k)


class OracleBloom:
    """A Redis bitmap string + Redisson's add/contains/count semantics."""

    def __init__(self, size: int, k: int):
        self.size, self.k = int(size), int(k)  # size: the Java long (negative sizes index [0, |size|))
        # a Redis string holds at most 2^32 bits (offsets past it are errors: orc_bloom_add)
        self.bitmap = np.zeros((min(abs(self.size), 1 << 32) + 7) // 8 + 1, dtype=np.uint8)
        self.redis_len = 0

    def add(self, buf, offs, per_key: bool = False):
        n = offs.size - 1
        out = np.zeros(max(n, 1), np.uint8)
        rl = C.c_uint64(self.redis_len)
        c = lib().orc_bloom_add(_p(self.bitmap), C.byref(rl), _p(buf), _p(offs, u64p), n, self.k,
                                self.size, _p(out))
        self.redis_len = rl.value
        return (c, out[:n]) if per_key else c

    def contains(self, buf, offs, per_key: bool = False):
        n = offs.size - 1
        out = np.zeros(max(n, 1), np.uint8)
        c = lib().orc_bloom_contains(_p(self.bitmap), self.redis_len, _p(buf), _p(offs, u64p), n,
                                     self.k, self.size, _p(out))
        return (c, out[:n]) if per_key else c

    def add_mt(self, buf, offs, nthreads: int, per_key: bool = False):
        """add() on nthreads threads (rbx_oracle_mt.c): the same flags, count and bitmap."""
        n = offs.size - 1
        out = np.zeros(max(n, 1), np.uint8)
        rl = C.c_uint64(self.redis_len)
        c = lib().orc_bloom_add_mt(_p(self.bitmap), C.byref(rl), _p(buf), _p(offs, u64p), n, self.k, self.size,
                                   _p(out), int(nthreads))
        self.redis_len = rl.value
        return (c, out[:n]) if per_key else c

    def contains_mt(self, buf, offs, nthreads: int, per_key: bool = False):
        n = offs.size - 1
        out = np.zeros(max(n, 1), np.uint8)
        c = lib().orc_bloom_contains_mt(_p(self.bitmap), self.redis_len, _p(buf), _p(offs, u64p), n, self.k,
                                        self.size, _p(out) if per_key else None, int(nthreads))
        return (c, out[:n]) if per_key else c

    def bitcount(self) -> int:
        return lib().orc_bitcount(_p(self.bitmap), self.redis_len)

    def count(self) -> int:
        return lib().orc_bloom_count_estimate(self.bitcount(), self.size, self.k)

    def redis_string(self) -> bytes:
        """What `GET name` returns."""
        return self.bitmap[: self.redis_len].tobytes()


def bloom_stream(filters: list, kf: np.ndarray, op: np.ndarray, buf: np.ndarray, offs: np.ndarray | None = None,
                 stride: int = 0):
    """An ordered stream of single-key add(T)/contains(T) commands (orc_bloom_stream): command i
    runs on filters[kf[i]] (OracleBloom objects, updated in place) in index order.  Keys: an arena
    (buf, offs) or fixed-stride bytes (offs None).  Returns (replies u8[n], [present, added])."""
    n = int(kf.size)
    kf = np.ascontiguousarray(kf, dtype=np.uint32)
    op = np.ascontiguousarray(op, dtype=np.uint8)
    buf = np.ascontiguousarray(buf, dtype=np.uint8).reshape(-1)
    bms = (u8p * len(filters))(*[_p(f.bitmap) for f in filters])
    lens = np.array([f.redis_len for f in filters], dtype=np.uint64)
    sizes = np.array([f.size for f in filters], dtype=np.int64)
    ks = np.array([f.k for f in filters], dtype=np.int32)
    assert int(ks.max()) <= 64 and (n == 0 or int(kf.max()) < len(filters))
    out = np.zeros(max(n, 1), np.uint8)
    cnt = np.zeros(2, np.uint64)
    lib().orc_bloom_stream(bms, _p(lens, u64p), _p(sizes, i64p), ks.ctypes.data_as(C.POINTER(C.c_int32)),
                           kf.ctypes.data_as(C.POINTER(C.c_uint32)), _p(op), _p(buf),
                           _p(offs, u64p) if offs is not None else None, int(stride), n, _p(out), _p(cnt, u64p))
    for f, ln in zip(filters, lens):
        f.redis_len = int(ln)
    return out[:n], [int(cnt[0]), int(cnt[1])]


def java_math_round(x: float) -> int:
    return lib().orc_java_math_round(x)


# ---- CRC16 / slots -----------------------------------------------------------------

def crc16(data: bytes) -> int:
    b = (C.c_uint8 * max(1, len(data))).from_buffer_copy(data or b"\0")
    return lib().orc_crc16(b, len(data))


def calc_slot(key: bytes) -> int:
    b = (C.c_uint8 * max(1, len(key))).from_buffer_copy(key or b"\0")
    return lib().orc_calc_slot(b, len(key))


# ---- HyperLogLog -------------------------------------------------------------------

def murmur64a(data: bytes, seed: int = 0xADC83B19) -> int:
    b = (C.c_uint8 * max(1, len(data))).from_buffer_copy(data or b"\0")
    return lib().orc_murmur64a(b, len(data), seed)


def murmur_batch(buf, offs) -> np.ndarray:
    n = offs.size - 1
    out = np.zeros(max(n, 1), np.uint64)
    lib().orc_murmur_batch(_p(buf), _p(offs, u64p), n, _p(out, u64p))
    return out[:n]


def hll_patlen(data: bytes) -> tuple[int, int]:
    """(register index, count)."""
    b = (C.c_uint8 * max(1, len(data))).from_buffer_copy(data or b"\0")
    r = C.c_long()
    c = lib().orc_hll_patlen(b, len(data), C.byref(r))
    return r.value, c


def hll_new() -> np.ndarray:
    return np.zeros(HLL_REGISTERS, dtype=np.uint8)


def hll_pfadd(regs: np.ndarray, buf, offs) -> int:
    n = offs.size - 1
    return lib().orc_hll_pfadd(_p(regs), _p(buf), _p(offs, u64p), n)


def hll_count(regs: np.ndarray) -> int:
    return lib().orc_hll_count(_p(np.ascontiguousarray(regs, dtype=np.uint8)))


def hll_count_histo(h) -> int:
    a = (C.c_int * 64)(*[int(x) for x in h])
    return lib().orc_hll_count_histo(a)


def hll_histogram(regs: np.ndarray) -> np.ndarray:
    a = (C.c_int * 64)()
    lib().orc_hll_histogram(_p(np.ascontiguousarray(regs, dtype=np.uint8)), a)
    return np.array(list(a), dtype=np.int64)


def hll_merge(dst: np.ndarray, src: np.ndarray) -> None:
    lib().orc_hll_merge(_p(dst), _p(np.ascontiguousarray(src, dtype=np.uint8)))


def hll_dense_pack(regs: np.ndarray) -> bytes:
    out = np.zeros(12289, np.uint8)
    lib().orc_hll_dense_pack(_p(np.ascontiguousarray(regs, dtype=np.uint8)), _p(out))
    return out[:12288].tobytes()


# Redis sparse HLL opcodes [redis-7.2 hyperloglog.c, "sparse representation" comment block]:
#   ZERO  00xxxxxx           run of 1..64 zero registers
#   XZERO 01xxxxxx yyyyyyyy  run of 1..16384 zero registers (14-bit length - 1)
#   VAL   1vvvvvxx           run of 1..4 registers holding value 1..32
def hll_sparse_pack(regs: np.ndarray) -> bytes | None:
    """Fewest-bytes sparse opcode string of the registers (no header); None if a register > 32."""
    out = bytearray()
    r = np.asarray(regs, dtype=np.uint8)
    i = 0
    while i < 16384:
        v = int(r[i])
        j = i + 1
        while j < 16384 and r[j] == v:
            j += 1
        run = j - i
        if v == 0:
            if run > 64:
                out += bytes([0x40 | ((run - 1) >> 8), (run - 1) & 0xFF])
            else:
                out.append(run - 1)
        else:
            if v > 32:
                return None
            while run:
                n = min(run, 4)
                out.append(0x80 | ((v - 1) << 2) | (n - 1))
                run -= n
        i = j
    return bytes(out)


def hll_sparse_unpack(ops: bytes) -> np.ndarray:
    """Registers of a sparse opcode string (no header); ValueError unless it covers 16384."""
    out = hll_new()
    i = p = 0
    while p < len(ops):
        b = ops[p]
        if b & 0xC0 == 0:
            i, p = i + (b & 0x3F) + 1, p + 1
        elif b & 0xC0 == 0x40:
            i, p = i + (((b & 0x3F) << 8) | ops[p + 1]) + 1, p + 2
        else:
            n = (b & 3) + 1
            out[i:i + n] = ((b >> 2) & 0x1F) + 1
            i, p = i + n, p + 1
        if i > 16384:
            raise ValueError("sparse string overruns 16384 registers")
    if i != 16384:
        raise ValueError("sparse string covers %d registers" % i)
    return out


def hll_dense_unpack(data: bytes) -> np.ndarray:
    src = np.zeros(12289, np.uint8)
    src[:12288] = np.frombuffer(data[:12288], np.uint8)
    out = hll_new()
    lib().orc_hll_dense_unpack(_p(src), _p(out))
    return out


HLL_SPARSE_MAX_BYTES = 3000  # redis.conf hll-sparse-max-bytes (default)


class RedisHll:
    """One Redis HLL key as redis-server holds it [redis-7.2 hyperloglog.c, external; restated in
    rbx_oracle.c orc_hll_sparse_*]: created sparse (createHLLObject), every PFADD element applied
    in order through hllSparseSet until the first promotion, dense afterwards.  `regs` tracks the
    registers in both encodings; `string(card)` is the GET value."""

    CAP = 16384 + 8  # an opcode covers >= 1 register

    def __init__(self, max_bytes: int = HLL_SPARSE_MAX_BYTES):
        self.ops = np.zeros(self.CAP, np.uint8)
        self.len = C.c_size_t(lib().orc_hll_sparse_new(_p(self.ops)))
        self.dense = C.c_int(0)
        self.regs = hll_new()
        self.max_bytes = max_bytes

    @classmethod
    def from_string(cls, s: bytes, max_bytes: int = HLL_SPARSE_MAX_BYTES):
        h = cls(max_bytes)
        if s[4] == 0:
            h.dense.value = 1
            h.regs = hll_dense_unpack(s[16:])
        else:
            h.regs = hll_sparse_unpack(s[16:])
            h.ops[:len(s) - 16] = np.frombuffer(s[16:], np.uint8)
            h.len.value = len(s) - 16
        return h

    def pfadd(self, buf, offs) -> int:
        r = lib().orc_hll_sparse_pfadd(_p(self.ops), C.byref(self.len), self.CAP, C.byref(self.dense), _p(self.regs),
                                       _p(buf), _p(offs, u64p), offs.size - 1, self.max_bytes)
        assert r >= 0, "invalid sparse string"
        return r

    def merge_from(self, maxregs: np.ndarray, use_dense: bool) -> None:
        """pfmergeCommand's write-back: maxregs = max over the sources and this key."""
        if use_dense:
            self.dense.value = 1
        if not self.dense.value:
            assert lib().orc_hll_sparse_merge(_p(self.ops), C.byref(self.len), self.CAP, C.byref(self.dense),
                                              _p(np.ascontiguousarray(maxregs, dtype=np.uint8)), self.max_bytes) == 0
        self.regs = np.maximum(self.regs, maxregs).astype(np.uint8)

    @property
    def sparse_ops(self) -> bytes:
        return self.ops[:self.len.value].tobytes()

    def string(self, card: bytes) -> bytes:
        """GET: header (card = the 8 cached-cardinality bytes) + opcodes or dense registers."""
        if self.dense.value:
            return b"HYLL" + bytes([0, 0, 0, 0]) + card + hll_dense_pack(self.regs)
        return b"HYLL" + bytes([1, 0, 0, 0]) + card + self.sparse_ops
