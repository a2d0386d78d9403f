"""Spring Data Redis connection surface for HyperLogLog (second caller of the HLL path).

Mirrors redisson-spring-data's RedissonConnection.pfAdd / pfCount / pfMerge
(redisson-spring-data/redisson-spring-data-32/src/main/java/org/redisson/spring/data/connection/
RedissonConnection.java:2200-2226): raw byte[] keys and members, no codec (ByteArrayCodec /
StringCodec pass the bytes through), PFADD's integer reply as a Long.

Keys are binary-safe: they travel as (bytes, length) pairs through the *_n entry points
(rbx_hll_add_multi_n / rbx_hll_count_n / rbx_hll_merge_n), so a key may hold any byte, zero
bytes included, exactly as a Redis key can.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _lib as L
from .client import RedissonClient, _check
from .exceptions import IllegalArgumentException
from .keys import Arena


def _key(k) -> bytes:
    if k is None:
        raise IllegalArgumentException("Keys must not contain 'null'.")
    return bytes(k)


class RedissonConnection:
    def __init__(self, client: RedissonClient):
        self._client = client

    def pfAdd(self, key: bytes, *values: bytes) -> int:
        """PFADD key v1..vn -> 1 if the HLL was created or a register changed, else 0."""
        a = Arena([bytes(v) for v in values])
        names, keep = L.names_array([_key(key)])
        seg = np.array([0, a.n], dtype=np.uint64)
        ch = np.zeros(1, np.uint8)
        _check(L.lib().rbx_hll_add_multi_n(self._client.ctx, names, 1, seg.ctypes.data_as(L.u64p), a.ptr(),
                                           ch.ctypes.data_as(L.u8p)))
        return int(ch[0])

    def pfCount(self, *keys: bytes) -> int:
        """PFCOUNT k1..kn (union when n > 1)."""
        if not keys:
            raise IllegalArgumentException("PFCOUNT requires at least one non 'null' key.")
        if any(k is None for k in keys):
            raise IllegalArgumentException("Keys for PFOUNT must not contain 'null'.")
        names, keep = L.names_array([_key(k) for k in keys])
        out = C.c_uint64()
        _check(L.lib().rbx_hll_count_n(self._client.ctx, names, len(keys), C.byref(out)))
        return int(out.value)

    def pfMerge(self, destinationKey: bytes, *sourceKeys: bytes) -> None:
        """PFMERGE dest s1..sn (dest's own registers included)."""
        srcs, keep = L.names_array([_key(k) for k in sourceKeys])
        dest, keep_d = L.name_struct(_key(destinationKey))
        _check(L.lib().rbx_hll_merge_n(self._client.ctx, dest, srcs, len(sourceKeys)))
