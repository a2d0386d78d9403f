/*
 * rbx_oracle.c -- CPU restatement of Redisson's probabilistic-structure hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in the product (redisson_amd/, include/) links,
 * loads or calls this file.  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg use it, and only as the checker / the timed CPU baseline.
 *
 * Reference: Redisson 3.25.2-SNAPSHOT at /root/reference (read-only).  Abbreviations:
 *   M/ = /root/reference/redisson/src/main/java/org/redisson/
 *
 * Parity status (see DESIGN.md "Oracle"):
 *   - HighwayHash / Hash.hash128 / Bloom index math: restated line by line from the
 *     Java sources cited below, pinned by the upstream HighwayHash known-answer
 *     vectors and the Redisson 729/5 config KAT (tests/test_oracle.py).
 *   - Redis bitmap (SETBIT/GETBIT/BITCOUNT) semantics and HyperLogLog register math
 *     (MurmurHash64A, patLen, dense layout, estimator) live in redis-server 7.2,
 *     which is NOT in /root/reference.  They are restated from the published
 *     redis 7.2 src/bitops.c and src/hyperloglog.c algorithms; MurmurHash64A is
 *     pinned by the SMHasher verification value 0x1F0D3804, CRC16 by the Redis
 *     Cluster spec KAT CRC16("123456789") = 0x31C3, and HLL counts only by the
 *     small-cardinality results of the Redisson/Redis tests ("weakly pinned").
 *
 * Build: oracle/Makefile (gcc -O2 -ffp-contract=off -fPIC -shared).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

/* ------------------------------------------------------------------------- */
/* HighwayHash (portable), M/misc/HighwayHash.java                            */
/* ------------------------------------------------------------------------- */

typedef struct {
    uint64_t v0[4], v1[4], mul0[4], mul1[4];
} orc_hh;

/* HighwayHash.java:229-246 */
static void hh_reset(orc_hh *s, const uint64_t key[4]) {
    s->mul0[0] = 0xdbe6d5d5fe4cce2fULL;
    s->mul0[1] = 0xa4093822299f31d0ULL;
    s->mul0[2] = 0x13198a2e03707344ULL;
    s->mul0[3] = 0x243f6a8885a308d3ULL;
    s->mul1[0] = 0x3bd39e10cb0ef593ULL;
    s->mul1[1] = 0xc0acf169b5f18a8cULL;
    s->mul1[2] = 0xbe5466cf34e90c6cULL;
    s->mul1[3] = 0x452821e638d01377ULL;
    for (int i = 0; i < 4; i++) {
        s->v0[i] = s->mul0[i] ^ key[i];
        s->v1[i] = s->mul1[i] ^ ((key[i] >> 32) | (key[i] << 32));
    }
}

/* HighwayHash.java:248-253 (argument order as in Java: (v1, v0)) */
static uint64_t zipper_merge0(uint64_t v1, uint64_t v0) {
    return (((v0 & 0xff000000ULL) | (v1 & 0xff00000000ULL)) >> 24) |
           (((v0 & 0xff0000000000ULL) | (v1 & 0xff000000000000ULL)) >> 16) |
           (v0 & 0xff0000ULL) | ((v0 & 0xff00ULL) << 32) |
           ((v1 & 0xff00000000000000ULL) >> 8) | (v0 << 56);
}

/* HighwayHash.java:255-260 */
static uint64_t zipper_merge1(uint64_t v1, uint64_t v0) {
    return (((v1 & 0xff000000ULL) | (v0 & 0xff00000000ULL)) >> 24) |
           (v1 & 0xff0000ULL) | ((v1 & 0xff0000000000ULL) >> 16) |
           ((v1 & 0xff00ULL) << 24) | ((v0 & 0xff000000000000ULL) >> 8) |
           ((v1 & 0xffULL) << 48) | (v0 & 0xff00000000000000ULL);
}

/* HighwayHash.java:93-114 */
static void hh_update(orc_hh *s, uint64_t a0, uint64_t a1, uint64_t a2, uint64_t a3) {
    s->v1[0] += s->mul0[0] + a0;
    s->v1[1] += s->mul0[1] + a1;
    s->v1[2] += s->mul0[2] + a2;
    s->v1[3] += s->mul0[3] + a3;
    for (int i = 0; i < 4; ++i) {
        s->mul0[i] ^= (s->v1[i] & 0xffffffffULL) * (s->v0[i] >> 32);
        s->v0[i] += s->mul1[i];
        s->mul1[i] ^= (s->v0[i] & 0xffffffffULL) * (s->v1[i] >> 32);
    }
    s->v0[0] += zipper_merge0(s->v1[1], s->v1[0]);
    s->v0[1] += zipper_merge1(s->v1[1], s->v1[0]);
    s->v0[2] += zipper_merge0(s->v1[3], s->v1[2]);
    s->v0[3] += zipper_merge1(s->v1[3], s->v1[2]);
    s->v1[0] += zipper_merge0(s->v0[1], s->v0[0]);
    s->v1[1] += zipper_merge1(s->v0[1], s->v0[0]);
    s->v1[2] += zipper_merge0(s->v0[3], s->v0[2]);
    s->v1[3] += zipper_merge1(s->v0[3], s->v0[2]);
}

/* HighwayHash.java:262-268 (little-endian) */
static uint64_t read64(const uint8_t *p) {
    uint64_t r = 0;
    for (int i = 7; i >= 0; i--) r = (r << 8) | p[i];
    return r;
}

/* HighwayHash.java:71-83 */
static void hh_update_packet(orc_hh *s, const uint8_t *packet) {
    hh_update(s, read64(packet), read64(packet + 8), read64(packet + 16), read64(packet + 24));
}

/* HighwayHash.java:270-278 */
static void rotate32_by(uint64_t count, uint64_t lanes[4]) {
    for (int i = 0; i < 4; ++i) {
        uint64_t half0 = lanes[i] & 0xffffffffULL;
        uint64_t half1 = (lanes[i] >> 32) & 0xffffffffULL;
        lanes[i] = ((half0 << count) & 0xffffffffULL) | (half0 >> (32 - count));
        lanes[i] |= (uint64_t)(((half1 << count) & 0xffffffffULL) | (half1 >> (32 - count))) << 32;
    }
}

/* HighwayHash.java:126-159 */
static void hh_update_remainder(orc_hh *s, const uint8_t *bytes, int size_mod32) {
    int size_mod4 = size_mod32 & 3;
    int remainder = size_mod32 & ~3;
    uint8_t packet[32];
    memset(packet, 0, sizeof packet);
    for (int i = 0; i < 4; ++i) s->v0[i] += ((uint64_t)size_mod32 << 32) + (uint64_t)size_mod32;
    rotate32_by((uint64_t)size_mod32, s->v1);
    for (int i = 0; i < remainder; i++) packet[i] = bytes[i];
    if ((size_mod32 & 16) != 0) {
        for (int i = 0; i < 4; i++) packet[28 + i] = bytes[remainder + i + size_mod4 - 4];
    } else if (size_mod4 != 0) {
        packet[16 + 0] = bytes[remainder + 0];
        packet[16 + 1] = bytes[remainder + (size_mod4 >> 1)];
        packet[16 + 2] = bytes[remainder + (size_mod4 - 1)];
    }
    hh_update_packet(s, packet);
}

/* HighwayHash.java:280-285 */
static void hh_permute_and_update(orc_hh *s) {
    hh_update(s, (s->v0[2] >> 32) | (s->v0[2] << 32), (s->v0[3] >> 32) | (s->v0[3] << 32),
              (s->v0[0] >> 32) | (s->v0[0] << 32), (s->v0[1] >> 32) | (s->v0[1] << 32));
}

/* HighwayHash.java:343-351 processAll */
static void hh_process_all(orc_hh *s, const uint8_t *data, size_t length) {
    size_t i;
    for (i = 0; i + 32 <= length; i += 32) hh_update_packet(s, data + i);
    if ((length & 31) != 0) hh_update_remainder(s, data + i, (int)(length & 31));
}

/* HighwayHash.java:169-176 */
uint64_t orc_highway_hash64(const uint8_t *data, size_t len, const uint64_t key[4]) {
    orc_hh s;
    hh_reset(&s, key);
    hh_process_all(&s, data, len);
    for (int i = 0; i < 4; i++) hh_permute_and_update(&s);
    return s.v0[0] + s.v1[0] + s.mul0[0] + s.mul1[0];
}

/* HighwayHash.java:186-198 (Redisson's 128-bit finalizer) */
void orc_highway_hash128(const uint8_t *data, size_t len, const uint64_t key[4], uint64_t out[2]) {
    orc_hh s;
    hh_reset(&s, key);
    hh_process_all(&s, data, len);
    for (int i = 0; i < 6; i++) hh_permute_and_update(&s);
    out[0] = s.v0[0] + s.mul0[0] + s.v1[2] + s.mul1[2];
    out[1] = s.v0[1] + s.mul0[1] + s.v1[3] + s.mul1[3];
}

/* M/misc/Hash.java:30 KEY and :53-74 hash128/calcHash (32-byte packets, then the
 * remainder; identical to processAll on a contiguous buffer). */
static const uint64_t REDISSON_KEY[4] = {0x9e3779b97f4a7c15ULL, 0xf39cc0605cedc834ULL,
                                         0x1082276bf3a27251ULL, 0xf86c6a11d0c18e95ULL};

void orc_redisson_hash128(const uint8_t *data, size_t len, uint64_t out[2]) {
    orc_hh s;
    hh_reset(&s, REDISSON_KEY);
    size_t i;
    for (i = 0; i + 32 <= len; i += 32) hh_update_packet(&s, data + i);      /* Hash.java:64-67 */
    if ((len & 31) != 0) hh_update_remainder(&s, data + i, (int)(len & 31)); /* Hash.java:68-72 */
    for (int r = 0; r < 6; r++) hh_permute_and_update(&s);
    out[0] = s.v0[0] + s.mul0[0] + s.v1[2] + s.mul1[2];
    out[1] = s.v0[1] + s.mul0[1] + s.v1[3] + s.mul1[3];
}

/* ------------------------------------------------------------------------- */
/* Java numeric helpers                                                       */
/* ------------------------------------------------------------------------- */

/* (long) cast of a double in Java: NaN -> 0, saturating. */
static int64_t java_d2l(double d) {
    if (d != d) return 0;
    if (d >= 9223372036854775807.0) return INT64_MAX;
    if (d <= -9223372036854775808.0) return INT64_MIN;
    return (int64_t)d;
}

/* java.lang.Math.round(double) (JDK 8+): round half up, exact, saturating. */
int64_t orc_java_math_round(double a) {
    uint64_t bits;
    memcpy(&bits, &a, 8);
    int64_t biased_exp = (int64_t)((bits & 0x7ff0000000000000ULL) >> 52);
    int64_t shift = (52 - 1 + 1023) - biased_exp; /* SIGNIFICAND_WIDTH-2+EXP_BIAS */
    if ((shift & -64) == 0) {
        int64_t r = (int64_t)((bits & 0x000fffffffffffffULL) | 0x0010000000000000ULL);
        if ((int64_t)bits < 0) r = -r;
        return ((r >> shift) + 1) >> 1;
    }
    return java_d2l(a);
}

/* ------------------------------------------------------------------------- */
/* Bloom filter, M/RedissonBloomFilter.java                                   */
/* ------------------------------------------------------------------------- */

/* Status codes mirror include/rbx.h. */
#define ORC_OK 0
#define ORC_E_ILLEGAL_ARGUMENT (-1)

/* RedissonBloomFilter.java:79-88 and tryInit validation :262-277.  max_size is
 * getMaxSize() = Integer.MAX_VALUE*2L (:257-259). */
int orc_bloom_optimal(int64_t n, double p, int64_t max_size, int64_t *size_out, int32_t *k_out) {
    if (p > 1) return ORC_E_ILLEGAL_ARGUMENT;
    if (p < 0) return ORC_E_ILLEGAL_ARGUMENT;
    double pp = p;
    if (pp == 0) pp = 4.9e-324; /* Double.MIN_VALUE */
    /* (double)(-n): Java's wrapping negation of a long */
    int64_t size = java_d2l((double)(int64_t)(0 - (uint64_t)n) * log(pp) / (log(2.0) * log(2.0)));
    if (size == 0) return ORC_E_ILLEGAL_ARGUMENT;
    if (size > max_size) return ORC_E_ILLEGAL_ARGUMENT;
    /* optimalNumOfHashFunctions: Math.max(1, (int) Math.round((double) m / n * Math.log(2))) */
    int64_t r = orc_java_math_round((double)size / (double)n * log(2.0));
    int32_t k = (int32_t)(uint32_t)(uint64_t)r; /* (int) cast of long: low 32 bits */
    if (k < 1) k = 1;
    *size_out = size;
    *k_out = k;
    return ORC_OK;
}

/* RedissonBloomFilter.java:139-151.  Java's `x % size` for x >= 0 takes the divisor's magnitude:
 * a negative size (tryInit with a negative expectedInsertions) indexes [0, |size|). */
void orc_bloom_indexes(uint64_t hash1, uint64_t hash2, int iterations, int64_t size, int64_t *out) {
    uint64_t hash = hash1;
    const uint64_t m = size < 0 ? 0 - (uint64_t)size : (uint64_t)size;
    for (int i = 0; i < iterations; i++) {
        out[i] = (int64_t)((hash & 0x7fffffffffffffffULL) % m);
        if (i % 2 == 0) hash += hash2;
        else hash += hash1;
    }
}

/* index() :188-196 over an arena of encoded keys (offsets has n+1 entries). */
void orc_bloom_hash_batch(const uint8_t *bytes, const uint64_t *offsets, uint64_t n, int k,
                          int64_t size, int64_t *out_idx) {
    for (uint64_t i = 0; i < n; i++) {
        uint64_t h[2];
        orc_redisson_hash128(bytes + offsets[i], (size_t)(offsets[i + 1] - offsets[i]), h);
        orc_bloom_indexes(h[0], h[1], k, size, out_idx + i * (uint64_t)k);
    }
}

/* Redis bitmap semantics [redis-7.2 bitops.c, external; Redisson's MSB-first view
 * M/RedissonBitSet.java:396-407]: bit i is byte i>>3, mask 0x80 >> (i & 7).
 * SETBIT returns the old bit and grows the string to (i>>3)+1 bytes; GETBIT past
 * the string end returns 0.  `bitmap` must hold (size+7)/8 bytes, zero past
 * *redis_len. */
static int getbit(const uint8_t *bm, uint64_t redis_len, uint64_t i) {
    uint64_t byte = i >> 3;
    if (byte >= redis_len) return 0;
    return (bm[byte] >> (7 - (i & 7))) & 1;
}

static int setbit(uint8_t *bm, uint64_t *redis_len, uint64_t i) {
    uint64_t byte = i >> 3;
    if (byte + 1 > *redis_len) *redis_len = byte + 1;
    int old = (bm[byte] >> (7 - (i & 7))) & 1;
    bm[byte] |= (uint8_t)(0x80 >> (i & 7));
    return old;
}

/* Redis bit offsets end at 2^32 - 1 [redis-7.2 bitops.c getBitOffsetFromArgument: 512 MiB strings]:
 * SETBIT / GETBIT past it reply "ERR bit offset is not an integer or out of range" without touching
 * the key.  Only a filter whose |size| exceeds 2^32 (tryInit with a negative expectedInsertions,
 * M/RedissonBloomFilter.java:262-277) produces such indexes.  In a pipelined batch every other
 * command still runs, and the batch then fails (CommandBatchService: the first error reply
 * completes execute() exceptionally) -- so add() has set every in-range bit and throws. */
#define ORC_MAX_OFFSET 0xFFFFFFFFULL
#define ORC_E_REDIS (-9)

/* add(Collection) :104-137: n*k SETBITs executed in submission order
 * (CommandBatchService ordering), then the fold over windows of s = k replies.
 * Returns the count, -4 (ArithmeticException "/ by zero") for n == 0, or -9 (RedisException: an
 * index past the Redis offset limit; every in-range bit is set). */
int64_t orc_bloom_add(uint8_t *bitmap, uint64_t *redis_len, const uint8_t *bytes,
                      const uint64_t *offsets, uint64_t n, int k, int64_t size, uint8_t *out_new) {
    if (n == 0) return -4;
    int64_t *idx = (int64_t *)malloc(sizeof(int64_t) * (size_t)k);
    int64_t c = 0;
    int err = 0;
    for (uint64_t i = 0; i < n; i++) {
        uint64_t h[2];
        orc_redisson_hash128(bytes + offsets[i], (size_t)(offsets[i + 1] - offsets[i]), h);
        orc_bloom_indexes(h[0], h[1], k, size, idx);
        int zeros = 0;
        for (int j = 0; j < k; j++) {
            if ((uint64_t)idx[j] > ORC_MAX_OFFSET) {
                err = 1;
                continue;
            }
            if (!setbit(bitmap, redis_len, (uint64_t)idx[j])) zeros++;
        }
        if (out_new) out_new[i] = zeros > 0;
        if (zeros > 0) c++;
    }
    free(idx);
    if (err) return ORC_E_REDIS;
    return (int64_t)(int32_t)c; /* `int c` accumulator in Java */
}

/* contains(Collection) :153-186: objects.size() - missed.  -4 for n == 0, -9 (RedisException) when
 * an index is past the Redis offset limit (GETBIT replies an error; nothing is changed). */
int64_t orc_bloom_contains(const uint8_t *bitmap, uint64_t redis_len, const uint8_t *bytes,
                           const uint64_t *offsets, uint64_t n, int k, int64_t size,
                           uint8_t *out_present) {
    if (n == 0) return -4;
    int64_t *idx = (int64_t *)malloc(sizeof(int64_t) * (size_t)k);
    int64_t missed = 0;
    int err = 0;
    for (uint64_t i = 0; i < n; i++) {
        uint64_t h[2];
        orc_redisson_hash128(bytes + offsets[i], (size_t)(offsets[i + 1] - offsets[i]), h);
        orc_bloom_indexes(h[0], h[1], k, size, idx);
        int zeros = 0;
        for (int j = 0; j < k; j++) {
            if ((uint64_t)idx[j] > ORC_MAX_OFFSET) {
                err = 1;
                continue;
            }
            if (!getbit(bitmap, redis_len, (uint64_t)idx[j])) zeros++;
        }
        if (out_present) out_present[i] = zeros == 0;
        if (zeros > 0) missed++;
    }
    free(idx);
    if (err) return ORC_E_REDIS;
    return (int64_t)n - missed;
}

/* An ordered stream of single-key commands (BASELINE config 5): command i is add(T) (op[i] != 0)
 * or contains(T) (op[i] == 0) on filter kf[i], executed one after another.  add(T) is
 * add(Arrays.asList(T)) > 0 (M/RedissonBloomFilter.java:99-102) and contains(T) is
 * contains(Arrays.asList(T)) > 0 (:198-201), i.e. one k-command batch per key.  Filter f is
 * bitmaps[f] / redis_lens[f] with sizes[f] bits and ks[f] hash iterations (k <= 64).  Keys: an
 * arena (offsets, n+1 entries) or, when offsets is NULL, fixed stride bytes.  out[i] = the
 * boolean reply; out_counts = {present contains, new adds}. */
void orc_bloom_stream(uint8_t *const *bitmaps, uint64_t *redis_lens, const int64_t *sizes, const int32_t *ks,
                      const uint32_t *kf, const uint8_t *op, const uint8_t *bytes, const uint64_t *offsets,
                      uint64_t stride, uint64_t n, uint8_t *out, uint64_t *out_counts) {
    int64_t idx[64];
    uint64_t present = 0, added = 0;
    for (uint64_t i = 0; i < n; i++) {
        const uint32_t f = kf[i];
        const uint64_t a = offsets ? offsets[i] : i * stride;
        const uint64_t len = offsets ? offsets[i + 1] - offsets[i] : stride;
        uint64_t h[2];
        orc_redisson_hash128(bytes + a, (size_t)len, h);
        const int k = ks[f];
        orc_bloom_indexes(h[0], h[1], k, sizes[f], idx);
        int zeros = 0;
        if (op[i]) {
            for (int j = 0; j < k; j++)
                if (!setbit(bitmaps[f], &redis_lens[f], (uint64_t)idx[j])) zeros++;
            out[i] = zeros > 0;
            added += zeros > 0;
        } else {
            for (int j = 0; j < k; j++)
                if (!getbit(bitmaps[f], redis_lens[f], (uint64_t)idx[j])) zeros++;
            out[i] = zeros == 0;
            present += zeros == 0;
        }
    }
    if (out_counts) {
        out_counts[0] = present;
        out_counts[1] = added;
    }
}

/* BITCOUNT over the whole string [redis-7.2 bitops.c]. */
uint64_t orc_bitcount(const uint8_t *bitmap, uint64_t redis_len) {
    uint64_t c = 0;
    for (uint64_t i = 0; i < redis_len; i++) c += (uint64_t)__builtin_popcount(bitmap[i]);
    return c;
}

/* count() :215-227: Math.round(-size / (double) k * Math.log(1 - bitcount / (double) size)) */
int64_t orc_bloom_count_estimate(uint64_t bitcount, int64_t size, int k) {
    double v = (double)(-size) / ((double)k) * log(1 - (double)bitcount / ((double)size));
    return orc_java_math_round(v);
}

/* ------------------------------------------------------------------------- */
/* CRC16 / slot: M/connection/CRC16.java:25-57, M/cluster/ClusterConnectionManager.java:777-792 */
/* ------------------------------------------------------------------------- */

uint16_t orc_crc16(const uint8_t *bytes, size_t len) {
    /* XMODEM CRC16, poly 0x1021, init 0 -- computed bitwise here (the reference uses
     * the equivalent 256-entry LOOKUP_TABLE, CRC16.java:25-46). */
    uint32_t crc = 0;
    for (size_t i = 0; i < len; i++) {
        crc ^= (uint32_t)bytes[i] << 8;
        for (int b = 0; b < 8; b++) crc = (crc & 0x8000) ? ((crc << 1) ^ 0x1021) : (crc << 1);
        crc &= 0xffff;
    }
    return (uint16_t)crc;
}

/* calcSlot(byte[]) ClusterConnectionManager.java:777-792 */
int orc_calc_slot(const uint8_t *key, size_t len) {
    if (key == NULL) return 0;
    long start = -1, end = -1;
    for (size_t i = 0; i < len; i++)
        if (key[i] == '{') { start = (long)i; break; }
    if (start != -1) {
        for (size_t i = 0; i < len; i++)
            if (key[i] == '}') { end = (long)i; break; }
        if (end != -1 && start + 1 < end) return orc_crc16(key + start + 1, (size_t)(end - start - 1)) % 16384;
    }
    return orc_crc16(key, len) % 16384;
}

/* ------------------------------------------------------------------------- */
/* HyperLogLog [redis-7.2 src/hyperloglog.c, external -- restated]            */
/* ------------------------------------------------------------------------- */

#define HLL_P 14
#define HLL_Q (64 - HLL_P)
#define HLL_REGISTERS (1 << HLL_P)
#define HLL_P_MASK (HLL_REGISTERS - 1)
#define HLL_BITS 6
#define HLL_REGISTER_MAX ((1 << HLL_BITS) - 1)
#define HLL_ALPHA_INF 0.721347520444481703680

/* MurmurHash64A as used by hyperloglog.c (x86-64, little-endian, unaligned reads). */
uint64_t orc_murmur64a(const uint8_t *key, int len, uint64_t seed) {
    const uint64_t m = 0xc6a4a7935bd1e995ULL;
    const int r = 47;
    uint64_t h = seed ^ ((uint64_t)(int64_t)len * m);
    const uint8_t *data = key;
    const uint8_t *end = data + (len - (len & 7));
    while (data != end) {
        uint64_t k = read64(data);
        k *= m;
        k ^= k >> r;
        k *= m;
        h ^= k;
        h *= m;
        data += 8;
    }
    switch (len & 7) {
    case 7: h ^= (uint64_t)data[6] << 48; /* fall-thru */
    case 6: h ^= (uint64_t)data[5] << 40; /* fall-thru */
    case 5: h ^= (uint64_t)data[4] << 32; /* fall-thru */
    case 4: h ^= (uint64_t)data[3] << 24; /* fall-thru */
    case 3: h ^= (uint64_t)data[2] << 16; /* fall-thru */
    case 2: h ^= (uint64_t)data[1] << 8;  /* fall-thru */
    case 1: h ^= (uint64_t)data[0]; h *= m;
    }
    h ^= h >> r;
    h *= m;
    h ^= h >> r;
    return h;
}

/* hllPatLen: register index and run length ("000..1" pattern, 1..51). */
int orc_hll_patlen(const uint8_t *ele, size_t elesize, long *regp) {
    uint64_t hash = orc_murmur64a(ele, (int)elesize, 0xadc83b19ULL);
    uint64_t index = hash & HLL_P_MASK;
    hash >>= HLL_P;
    hash |= ((uint64_t)1 << HLL_Q);
    uint64_t bit = 1;
    int count = 1;
    while ((hash & bit) == 0) {
        count++;
        bit <<= 1;
    }
    *regp = (long)index;
    return count;
}

/* PFADD over raw (unpacked u8) registers: returns 1 iff any register grew
 * (hllAdd == 1 for some element).  Key creation (which also returns 1) is the
 * caller's business. */
int orc_hll_pfadd(uint8_t *regs, const uint8_t *bytes, const uint64_t *offsets, uint64_t n) {
    int updated = 0;
    for (uint64_t i = 0; i < n; i++) {
        long index;
        uint8_t count = (uint8_t)orc_hll_patlen(bytes + offsets[i], (size_t)(offsets[i + 1] - offsets[i]), &index);
        if (count > regs[index]) {
            regs[index] = count;
            updated = 1;
        }
    }
    return updated;
}

/* HLL_DENSE_GET_REGISTER / HLL_DENSE_SET_REGISTER over a 12288-byte array
 * (the macros may touch p[12288], the sds terminator; we allow a 12289-byte buffer). */
void orc_hll_dense_pack(const uint8_t *regs, uint8_t *p /* >= 12289 bytes */) {
    memset(p, 0, 12289);
    for (unsigned long regnum = 0; regnum < HLL_REGISTERS; regnum++) {
        unsigned long byte = regnum * HLL_BITS / 8;
        unsigned long fb = regnum * HLL_BITS & 7;
        unsigned long fb8 = 8 - fb;
        unsigned long v = regs[regnum];
        p[byte] &= (uint8_t)~(HLL_REGISTER_MAX << fb);
        p[byte] |= (uint8_t)(v << fb);
        p[byte + 1] &= (uint8_t)~(HLL_REGISTER_MAX >> fb8);
        p[byte + 1] |= (uint8_t)(v >> fb8);
    }
}

void orc_hll_dense_unpack(const uint8_t *p /* >= 12289 bytes */, uint8_t *regs) {
    for (unsigned long regnum = 0; regnum < HLL_REGISTERS; regnum++) {
        unsigned long byte = regnum * HLL_BITS / 8;
        unsigned long fb = regnum * HLL_BITS & 7;
        unsigned long fb8 = 8 - fb;
        unsigned long b0 = p[byte];
        unsigned long b1 = p[byte + 1];
        regs[regnum] = (uint8_t)(((b0 >> fb) | (b1 << fb8)) & HLL_REGISTER_MAX);
    }
}

/* hllSigma / hllTau (Ertl, arXiv:1702.01284), exactly as hyperloglog.c. */
static double hll_sigma(double x) {
    if (x == 1.) return INFINITY;
    double zPrime;
    double y = 1;
    double z = x;
    do {
        x *= x;
        zPrime = z;
        z += x * y;
        y += y;
    } while (zPrime != z);
    return z;
}

static double hll_tau(double x) {
    if (x == 0. || x == 1.) return 0.;
    double zPrime;
    double y = 1.0;
    double z = 1 - x;
    do {
        x = sqrt(x);
        zPrime = z;
        y *= 0.5;
        z -= pow(1 - x, 2) * y;
    } while (zPrime != z);
    return z / 3;
}

/* hllCount from a register histogram reghisto[64]. */
uint64_t orc_hll_count_histo(const int *reghisto) {
    double m = HLL_REGISTERS;
    double E;
    int j;
    double z = m * hll_tau((m - reghisto[HLL_Q + 1]) / (double)m);
    for (j = HLL_Q; j >= 1; --j) {
        z += reghisto[j];
        z *= 0.5;
    }
    z += m * hll_sigma(reghisto[0] / (double)m);
    E = (double)llroundl(HLL_ALPHA_INF * m * m / z);
    return (uint64_t)E;
}

void orc_hll_histogram(const uint8_t *regs, int *reghisto /* 64 */) {
    memset(reghisto, 0, sizeof(int) * 64);
    for (int i = 0; i < HLL_REGISTERS; i++) reghisto[regs[i] & 63]++;
}

uint64_t orc_hll_count(const uint8_t *regs) {
    int h[64];
    orc_hll_histogram(regs, h);
    return orc_hll_count_histo(h);
}

/* PFMERGE / multi-key PFCOUNT register union: dst[i] = max(dst[i], src[i]). */
void orc_hll_merge(uint8_t *dst, const uint8_t *src) {
    for (int i = 0; i < HLL_REGISTERS; i++)
        if (src[i] > dst[i]) dst[i] = src[i];
}

/* Batched helpers for tests / the CPU baseline. */
void orc_murmur_batch(const uint8_t *bytes, const uint64_t *offsets, uint64_t n, uint64_t *out) {
    for (uint64_t i = 0; i < n; i++)
        out[i] = orc_murmur64a(bytes + offsets[i], (int)(offsets[i + 1] - offsets[i]), 0xadc83b19ULL);
}

void orc_hash128_batch(const uint8_t *bytes, const uint64_t *offsets, uint64_t n, uint64_t *out /* 2n */) {
    for (uint64_t i = 0; i < n; i++)
        orc_redisson_hash128(bytes + offsets[i], (size_t)(offsets[i + 1] - offsets[i]), out + 2 * i);
}

/* ------------------------------------------------------------------------- */
/* Sparse HLL strings [redis-7.2 src/hyperloglog.c hllSparseSet / hllSparseAdd /  */
/* pfaddCommand / pfmergeCommand, external -- restated byte for byte].  The caller */
/* is M/RedissonHyperLogLog.java:71-102 (PFADD / PFMERGE); Redis keeps the sparse   */
/* string it built incrementally, so GET bytes depend on the order of the updates. */
/* `ops` is the opcode string without the 16-byte header, *len its length, cap its */
/* capacity (>= *len + 3).  max_bytes = hll-sparse-max-bytes, compared with the    */
/* whole string (header included), as sdslen(o->ptr) is.                          */
/* Returns 0 = no change, 1 = updated, 2 = promote (string untouched), -1 invalid.  */
/* ------------------------------------------------------------------------- */
#define SP_IS_ZERO(p) (((*(p)) & 0xc0) == 0)
#define SP_IS_XZERO(p) (((*(p)) & 0xc0) == 0x40)
#define SP_IS_VAL(p) ((*(p)) & 0x80)
#define SP_ZERO_LEN(p) (((*(p)) & 0x3f) + 1)
#define SP_XZERO_LEN(p) (((((*(p)) & 0x3f) << 8) | (*((p) + 1))) + 1)
#define SP_VAL_VALUE(p) ((((*(p)) >> 2) & 0x1f) + 1)
#define SP_VAL_LEN(p) (((*(p)) & 0x3) + 1)
#define SP_ZERO_SET(p, len) (*(p) = (uint8_t)((len) - 1))
#define SP_XZERO_SET(p, len)                          \
    do {                                              \
        int _l = (len) - 1;                           \
        *(p) = (uint8_t)((_l >> 8) | 0x40);           \
        *((p) + 1) = (uint8_t)(_l & 0xff);            \
    } while (0)
#define SP_VAL_SET(p, val, len) (*(p) = (uint8_t)((((val) - 1) << 2 | ((len) - 1)) | 0x80))

int orc_hll_sparse_set(uint8_t *ops, size_t *len, size_t cap, long index, int count, size_t max_bytes) {
    if (count > 32) return 2; /* HLL_SPARSE_VAL_MAX_VALUE */
    if (cap < *len + 3) return -1;
    uint8_t *sparse = ops, *p = ops, *end = ops + *len, *prev = NULL, *next;
    long first = 0, span = 0;
    /* step 1: the opcode covering `index` */
    while (p < end) {
        long oplen = 1;
        if (SP_IS_ZERO(p)) {
            span = SP_ZERO_LEN(p);
        } else if (SP_IS_VAL(p)) {
            span = SP_VAL_LEN(p);
        } else {
            span = SP_XZERO_LEN(p);
            oplen = 2;
        }
        if (index <= first + span - 1) break;
        prev = p;
        p += oplen;
        first += span;
    }
    if (span == 0 || p >= end) return -1;
    next = SP_IS_XZERO(p) ? p + 2 : p + 1;
    if (next >= end) next = NULL;
    int is_zero = 0, is_xzero = 0, is_val = 0;
    long runlen;
    if (SP_IS_ZERO(p)) {
        is_zero = 1;
        runlen = SP_ZERO_LEN(p);
    } else if (SP_IS_XZERO(p)) {
        is_xzero = 1;
        runlen = SP_XZERO_LEN(p);
    } else {
        is_val = 1;
        runlen = SP_VAL_LEN(p);
    }
    /* step 2: cases A-C */
    if (is_val) {
        if (SP_VAL_VALUE(p) >= count) return 0;
        if (runlen == 1) {
            SP_VAL_SET(p, count, 1);
            goto updated;
        }
    }
    if (is_zero && runlen == 1) {
        SP_VAL_SET(p, count, 1);
        goto updated;
    }
    /* case D: split into at most three opcodes (<= 5 bytes) */
    {
        uint8_t seq[5], *n = seq;
        long last = first + span - 1, l;
        if (is_zero || is_xzero) {
            if (index != first) {
                l = index - first;
                if (l > 64) {
                    SP_XZERO_SET(n, l);
                    n += 2;
                } else {
                    SP_ZERO_SET(n, l);
                    n++;
                }
            }
            SP_VAL_SET(n, count, 1);
            n++;
            if (index != last) {
                l = last - index;
                if (l > 64) {
                    SP_XZERO_SET(n, l);
                    n += 2;
                } else {
                    SP_ZERO_SET(n, l);
                    n++;
                }
            }
        } else {
            int curval = SP_VAL_VALUE(p);
            if (index != first) {
                l = index - first;
                SP_VAL_SET(n, curval, l);
                n++;
            }
            SP_VAL_SET(n, count, 1);
            n++;
            if (index != last) {
                l = last - index;
                SP_VAL_SET(n, curval, l);
                n++;
            }
        }
        /* step 3: substitute */
        long seqlen = n - seq, oldlen = is_xzero ? 2 : 1, deltalen = seqlen - oldlen;
        if (deltalen > 0 && 16 + *len + deltalen > max_bytes) return 2;
        if (deltalen && next) memmove(next + deltalen, next, (size_t)(end - next));
        *len += deltalen;
        memcpy(p, seq, (size_t)seqlen);
        end += deltalen;
    }
updated:
    /* step 4: merge adjacent VAL opcodes of one value, up to 5 opcodes from prev */
    p = prev ? prev : sparse;
    int scanlen = 5;
    while (p < end && scanlen--) {
        if (SP_IS_XZERO(p)) {
            p += 2;
            continue;
        } else if (SP_IS_ZERO(p)) {
            p++;
            continue;
        }
        if (p + 1 < end && SP_IS_VAL(p + 1)) {
            int v1 = SP_VAL_VALUE(p), v2 = SP_VAL_VALUE(p + 1);
            if (v1 == v2) {
                int l = SP_VAL_LEN(p) + SP_VAL_LEN(p + 1);
                if (l <= 4) {
                    SP_VAL_SET(p + 1, v1, l);
                    memmove(p, p + 1, (size_t)(end - p));
                    *len -= 1;
                    end--;
                    continue; /* retry at p: the merged opcode may merge again */
                }
            }
        }
        p++;
    }
    return 1;
}

/* createHLLObject: one XZERO covering the 16384 registers (2 bytes). */
size_t orc_hll_sparse_new(uint8_t *ops) {
    SP_XZERO_SET(ops, HLL_REGISTERS);
    return 2;
}

/* PFADD on an HLL held as (regs, sparse string, *dense): elements in order; while sparse each
 * goes through hllSparseSet, the first promotion converts to dense (the registers are kept in
 * `regs` throughout).  Returns 1 iff a register changed. */
int orc_hll_sparse_pfadd(uint8_t *ops, size_t *len, size_t cap, int *dense, uint8_t *regs, const uint8_t *bytes,
                         const uint64_t *offsets, uint64_t n, size_t max_bytes) {
    int updated = 0;
    for (uint64_t i = 0; i < n; i++) {
        long index;
        int count = orc_hll_patlen(bytes + offsets[i], (size_t)(offsets[i + 1] - offsets[i]), &index);
        if (!*dense) {
            int r = orc_hll_sparse_set(ops, len, cap, index, count, max_bytes);
            if (r < 0) return -1;
            if (r == 2) *dense = 1;
        }
        if (count > regs[index]) {
            regs[index] = (uint8_t)count;
            updated = 1;
        }
    }
    return updated;
}

/* pfmergeCommand's write-back into a sparse destination: hllSparseSet(j, max[j]) for every
 * nonzero max[j], ascending j (a promotion converts the rest to dense).  `maxregs` already
 * includes the destination's own registers. */
int orc_hll_sparse_merge(uint8_t *ops, size_t *len, size_t cap, int *dense, const uint8_t *maxregs, size_t max_bytes) {
    for (long j = 0; j < HLL_REGISTERS && !*dense; j++) {
        if (!maxregs[j]) continue;
        int r = orc_hll_sparse_set(ops, len, cap, j, maxregs[j], max_bytes);
        if (r < 0) return -1;
        if (r == 2) *dense = 1;
    }
    return 0;
}
