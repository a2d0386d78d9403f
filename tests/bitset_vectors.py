"""Reference-held bitmap vectors (test data; see test_oracle.py / test_bloom_gpu.py)."""
from oracle import oracle as O

# ---- T/RedissonBitSetTest.java vectors: the Redis bitmap's MSB-first bits and lazy length ------
# RBitSet.size() = STRLEN * 8 and cardinality() = BITCOUNT (M/RedissonBitSet.java:302-305,482-484);
# a Bloom filter writes its bitmap through the same SETBIT.  A raw (size 64, k = 1) filter sets
# exactly one chosen bit per key, so each test's SETBIT sequence is replayed as an add() of keys.
BITSET_VECTORS = [
    # (bits set in order, expected size() in bits, expected cardinality)   T/RedissonBitSetTest.java
    ([10, 31], 32, 2),                    # testSetGet :140-152
    (list(range(3, 10)), 16, 7),          # testSetRange :154-160  set(3, 10) = bits 3..9
    ([3, 41], 48, 2),                     # testAsBitSet :162-176
    ([3, 4], 8, 2),                       # testAnd :178-186  bs1.set(3, 5) = bits 3, 4
]


def key_for_bit(bit: int, size: int = 64) -> bytes:
    """A key whose single Bloom index (k = 1) under a raw `size`-bit filter is `bit`."""
    i = 0
    while True:
        k = b"bit-%d-%d" % (bit, i)
        if O.bloom_indexes(*O.redisson_hash128(k), 1, size)[0] == bit:
            return k
        i += 1
