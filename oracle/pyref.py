"""Pure-Python restatement of the hash functions (TEST INFRASTRUCTURE, small inputs only).

A second, independent transcription used to cross-check oracle/rbx_oracle.c:
  HighwayHash   M/misc/HighwayHash.java:93-285, Hash.java:30,53-74
  Bloom index   M/RedissonBloomFilter.java:139-151
  CRC16/slot    M/connection/CRC16.java:51-57, M/cluster/ClusterConnectionManager.java:777-792
  MurmurHash64A / hllPatLen  [redis-7.2 hyperloglog.c, external]
(M/ = /root/reference/redisson/src/main/java/org/redisson/)
"""
from __future__ import annotations

M64 = (1 << 64) - 1
REDISSON_KEY = (0x9E3779B97F4A7C15, 0xF39CC0605CEDC834, 0x1082276BF3A27251, 0xF86C6A11D0C18E95)


def _rot32(x: int) -> int:
    return ((x >> 32) | (x << 32)) & M64


class _HH:
    def __init__(self, key):
        self.mul0 = [0xDBE6D5D5FE4CCE2F, 0xA4093822299F31D0, 0x13198A2E03707344, 0x243F6A8885A308D3]
        self.mul1 = [0x3BD39E10CB0EF593, 0xC0ACF169B5F18A8C, 0xBE5466CF34E90C6C, 0x452821E638D01377]
        self.v0 = [self.mul0[i] ^ key[i] for i in range(4)]
        self.v1 = [self.mul1[i] ^ _rot32(key[i]) for i in range(4)]

    @staticmethod
    def _zm(v1: int, v0: int):
        """returns (zipperMerge0(v1, v0), zipperMerge1(v1, v0)) by byte positions."""
        a = v0.to_bytes(8, "little")
        b = v1.to_bytes(8, "little")
        z0 = bytes([a[3], b[4], a[2], a[5], b[6], a[1], b[7], a[0]])
        z1 = bytes([b[3], a[4], b[2], b[5], b[1], a[6], b[0], a[7]])
        return int.from_bytes(z0, "little"), int.from_bytes(z1, "little")

    def update(self, a):
        v0, v1, m0, m1 = self.v0, self.v1, self.mul0, self.mul1
        for i in range(4):
            v1[i] = (v1[i] + m0[i] + a[i]) & M64
        for i in range(4):
            m0[i] ^= ((v1[i] & 0xFFFFFFFF) * (v0[i] >> 32)) & M64
            v0[i] = (v0[i] + m1[i]) & M64
            m1[i] ^= ((v0[i] & 0xFFFFFFFF) * (v1[i] >> 32)) & M64
        z = self._zm(v1[1], v1[0])
        w = self._zm(v1[3], v1[2])
        v0[0] = (v0[0] + z[0]) & M64
        v0[1] = (v0[1] + z[1]) & M64
        v0[2] = (v0[2] + w[0]) & M64
        v0[3] = (v0[3] + w[1]) & M64
        z = self._zm(v0[1], v0[0])
        w = self._zm(v0[3], v0[2])
        v1[0] = (v1[0] + z[0]) & M64
        v1[1] = (v1[1] + z[1]) & M64
        v1[2] = (v1[2] + w[0]) & M64
        v1[3] = (v1[3] + w[1]) & M64

    def packet(self, p: bytes):
        self.update([int.from_bytes(p[8 * j:8 * j + 8], "little") for j in range(4)])

    def remainder(self, t: bytes):
        r = len(t)
        sm4, rem = r & 3, r & ~3
        for i in range(4):
            self.v0[i] = (self.v0[i] + (r << 32) + r) & M64
            lo, hi = self.v1[i] & 0xFFFFFFFF, self.v1[i] >> 32
            lo = ((lo << r) | (lo >> (32 - r))) & 0xFFFFFFFF
            hi = ((hi << r) | (hi >> (32 - r))) & 0xFFFFFFFF
            self.v1[i] = (hi << 32) | lo
        pk = bytearray(32)
        pk[:rem] = t[:rem]
        if r & 16:
            pk[28:32] = t[rem + sm4 - 4:rem + sm4]
        elif sm4:
            pk[16] = t[rem]
            pk[17] = t[rem + (sm4 >> 1)]
            pk[18] = t[rem + sm4 - 1]
        self.packet(bytes(pk))

    def process(self, data: bytes):
        n = len(data)
        i = 0
        while i + 32 <= n:
            self.packet(data[i:i + 32])
            i += 32
        if n & 31:
            self.remainder(data[i:])

    def permute(self):
        v0 = self.v0
        self.update([_rot32(v0[2]), _rot32(v0[3]), _rot32(v0[0]), _rot32(v0[1])])


def highway_hash64(data: bytes, key) -> int:
    s = _HH(key)
    s.process(data)
    for _ in range(4):
        s.permute()
    return (s.v0[0] + s.v1[0] + s.mul0[0] + s.mul1[0]) & M64


def highway_hash128(data: bytes, key=REDISSON_KEY) -> tuple[int, int]:
    s = _HH(key)
    s.process(data)
    for _ in range(6):
        s.permute()
    return ((s.v0[0] + s.mul0[0] + s.v1[2] + s.mul1[2]) & M64,
            (s.v0[1] + s.mul0[1] + s.v1[3] + s.mul1[3]) & M64)


def bloom_indexes(h1: int, h2: int, k: int, size: int) -> list[int]:
    # Java's `x % size` takes the dividend's sign: for x >= 0 it is x % |size| (negative sizes too)
    out, h = [], h1
    for i in range(k):
        out.append((h & 0x7FFFFFFFFFFFFFFF) % abs(size))
        h = (h + (h2 if i % 2 == 0 else h1)) & M64
    return out


def crc16(data: bytes) -> int:
    crc = 0
    for b in data:
        crc ^= b << 8
        for _ in range(8):
            crc = ((crc << 1) ^ 0x1021) if crc & 0x8000 else (crc << 1)
            crc &= 0xFFFF
    return crc


def calc_slot(key: bytes) -> int:
    s = key.find(b"{")
    if s != -1:
        e = key.find(b"}")
        if e != -1 and s + 1 < e:
            key = key[s + 1:e]
    return crc16(key) % 16384


def murmur64a(data: bytes, seed: int = 0xADC83B19) -> int:
    m, r = 0xC6A4A7935BD1E995, 47
    n = len(data)
    h = (seed ^ ((n * m) & M64)) & M64
    nb = n - (n & 7)
    for i in range(0, nb, 8):
        k = int.from_bytes(data[i:i + 8], "little")
        k = (k * m) & M64
        k ^= k >> r
        k = (k * m) & M64
        h ^= k
        h = (h * m) & M64
    t = n & 7
    if t:
        h ^= int.from_bytes(data[nb:], "little")
        h = (h * m) & M64
    h ^= h >> r
    h = (h * m) & M64
    h ^= h >> r
    return h


def hll_patlen(data: bytes) -> tuple[int, int]:
    h = murmur64a(data)
    idx = h & 16383
    x = (h >> 14) | (1 << 50)
    return idx, ((x & -x).bit_length())
