"""redisson_amd -- MI355X-native batched sketch engine for Redisson's probabilistic
structures (RBloomFilter / RHyperLogLog), behind a C ABI (include/rbx.h, librbx.so).

Host mirror of the reference API: RedissonClient.getBloomFilter / getHyperLogLog.
"""
from .client import (BloomHandle, RBloomFilter, RedissonClient, RHyperLogLog, bloom_add_multi, bloom_stream,
                     bloom_contains_multi, calc_slot, crc16, hll_add_multi, hll_count_each, slot_to_gpu)
from .codec import ByteArrayCodec, StringCodec
from .exceptions import (ArithmeticException, DeviceError, IllegalArgumentException, IllegalStateException,
                         RedisException)
from .keys import Arena, device_keys

Redisson = RedissonClient

__all__ = [
    "Arena", "ArithmeticException", "BloomHandle", "bloom_stream", "ByteArrayCodec", "DeviceError", "IllegalArgumentException",
    "IllegalStateException", "RBloomFilter", "RHyperLogLog", "RedisException", "Redisson", "RedissonClient",
    "StringCodec", "bloom_add_multi", "bloom_contains_multi", "calc_slot", "crc16", "device_keys",
    "hll_add_multi", "hll_count_each", "slot_to_gpu",
]
