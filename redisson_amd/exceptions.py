"""Exceptions mirroring what the reference path throws (M/ = redisson/src/main/java/org/redisson/)."""


class RedissonAmdError(Exception):
    """Base class."""


class IllegalArgumentException(RedissonAmdError, ValueError):
    """java.lang.IllegalArgumentException (RedissonBloomFilter.tryInit, M/RedissonBloomFilter.java:263-276)."""


class IllegalStateException(RedissonAmdError):
    """java.lang.IllegalStateException "Bloom filter is not initialized!" (:251, :386)."""


class RedisException(RedissonAmdError):
    """org.redisson.client.RedisException (Lua assert, WRONGTYPE, ERR no such key)."""


class ArithmeticException(RedissonAmdError, ZeroDivisionError):
    """java.lang.ArithmeticException "/ by zero": add/contains of an empty collection (:121, :170)."""


class DeviceError(RedissonAmdError):
    """HIP / RCCL failure inside librbx.so."""


def raise_for(code: int, msg: str) -> None:
    from . import _lib as L

    if code == L.RBX_OK:
        return
    cls = {
        L.RBX_E_ILLEGAL_ARGUMENT: IllegalArgumentException,
        L.RBX_E_ILLEGAL_STATE: IllegalStateException,
        L.RBX_E_CONFIG_CHANGED: RedisException,
        L.RBX_E_ARITHMETIC: ArithmeticException,
        L.RBX_E_WRONGTYPE: RedisException,
        L.RBX_E_NO_SUCH_KEY: RedisException,
        L.RBX_E_REDIS: RedisException,
        L.RBX_E_OOM: DeviceError,
        L.RBX_E_DEVICE: DeviceError,
    }.get(code, RedissonAmdError)
    raise cls(msg)
