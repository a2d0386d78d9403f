"""Value codecs: object -> encoded bytes (RedissonObject.encode, M/RedissonObject.java:319-321).

The engine hashes codec OUTPUT, exactly like the reference.  Kryo5Codec (the
reference default, M/config/Config.java:110) is a JVM library and is not restated;
StringCodec (M/client/codec/StringCodec.java:36-44: UTF-8 of toString()) and
ByteArrayCodec (identity, M/client/codec/ByteArrayCodec.java:35-40) are.
"""
from __future__ import annotations


class Codec:
    def encode(self, value) -> bytes:  # pragma: no cover - interface
        raise NotImplementedError


class ByteArrayCodec(Codec):
    def encode(self, value) -> bytes:
        if isinstance(value, (bytes, bytearray, memoryview)):
            return bytes(value)
        raise TypeError("ByteArrayCodec encodes byte arrays only")


def _java_to_string(value) -> str:
    if isinstance(value, bool):
        return "true" if value else "false"
    if isinstance(value, float):
        raise TypeError("Double.toString formatting is not mirrored; pass str/bytes")
    return str(value)


class StringCodec(Codec):
    """UTF-8 of value.toString(); bytes pass through unchanged."""

    def encode(self, value) -> bytes:
        if isinstance(value, (bytes, bytearray, memoryview)):
            return bytes(value)
        return _java_to_string(value).encode("utf-8")


DEFAULT_CODEC = StringCodec()
