"""Spring Data Redis connection surface for HyperLogLog (second caller of the HLL path).

Mirrors redisson-spring-data's RedissonConnection.pfAdd / pfCount / pfMerge
(redisson-spring-data/redisson-spring-data-32/src/main/java/org/redisson/spring/data/connection/
RedissonConnection.java:2200-2226): raw byte[] keys and members, no codec (ByteArrayCodec /
StringCodec pass the bytes through), PFADD's integer reply as a Long.

Key names travel through the C ABI as NUL-terminated strings, so a key containing a zero
byte is rejected (IllegalArgumentException) rather than silently truncated.
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
    b = bytes(k)
    if b"\0" in b:
        raise IllegalArgumentException("key names with a zero byte are not supported by the C ABI")
    return b


class RedissonConnection:
    def __init__(self, client: RedissonClient):
        self._client = client

    def pfAdd(self, key: bytes, *values: bytes) -> int:
        """PFADD key v1..vn -> 1 if the HLL was created or a register changed, else 0."""
        a = Arena([bytes(v) for v in values])
        ch = C.c_int()
        _check(L.lib().rbx_hll_add(self._client.ctx, _key(key), a.ptr(), C.byref(ch)))
        return int(ch.value)

    def pfCount(self, *keys: bytes) -> int:
        """PFCOUNT k1..kn (union when n > 1)."""
        if not keys:
            raise IllegalArgumentException("PFCOUNT requires at least one non 'null' key.")
        if any(k is None for k in keys):
            raise IllegalArgumentException("Keys for PFOUNT must not contain 'null'.")
        arr = (C.c_char_p * len(keys))(*[_key(k) for k in keys])
        out = C.c_uint64()
        _check(L.lib().rbx_hll_count(self._client.ctx, arr, len(keys), C.byref(out)))
        return int(out.value)

    def pfMerge(self, destinationKey: bytes, *sourceKeys: bytes) -> None:
        """PFMERGE dest s1..sn (dest's own registers included)."""
        arr = (C.c_char_p * max(len(sourceKeys), 1))(*[_key(k) for k in sourceKeys])
        _check(L.lib().rbx_hll_merge(self._client.ctx, _key(destinationKey), arr, len(sourceKeys)))
