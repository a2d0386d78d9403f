// rbx_device.h -- device primitives of the sketch engine (gfx950).
//
// HighwayHash128 over codec bytes (M/misc/HighwayHash.java, M/misc/Hash.java:53-74),
// the Bloom double-hash index `(h & Long.MAX_VALUE) % size` (M/RedissonBloomFilter.java:139-151)
// with an exact divide-free 63-bit modulo, MurmurHash64A + patLen for HyperLogLog
// [redis-7.2 hyperloglog.c], and coalesced key loads from a byte arena.
// M/ = /root/reference/redisson/src/main/java/org/redisson/
//
// Everything here is __host__ __device__ where it can be, so the same code is
// exercised on the CPU by tests/test_fastmod.py (via rbx_selftest in librbx.so).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#define RBX_HD __host__ __device__ __forceinline__

namespace rbx {

// ---------------------------------------------------------------------------------
// Exact (h mod d) for h < 2^63 and 1 <= d <= 2^32 without a hardware divide.
// d = 2^j uses a mask.  Otherwise d is normalized (dn = d << s, bit 31 set) and the
// 95-bit value h << s is reduced by two Moller-Granlund 2-by-1 word divisions
// ("Improved division by invariant integers", IEEE TC 2011, Alg. 4) with the
// precomputed reciprocal v = floor((2^64-1)/dn) - 2^32.
// ---------------------------------------------------------------------------------
struct ModParams {
    uint64_t size;  // the Bloom "size" (bits), 1..2^32
    uint32_t mask;  // size-1 when size is a power of two
    uint32_t pow2;  // 1 when size is a power of two
    uint32_t dn;    // size << s (normalized divisor)
    uint32_t v;     // reciprocal
    uint32_t s;     // normalization shift
    uint32_t pad;
};

inline ModParams make_mod_params(uint64_t size) {
    ModParams p{};
    p.size = size;
    if ((size & (size - 1)) == 0) {
        p.pow2 = 1;
        p.mask = (uint32_t)(size - 1);
        return p;
    }
    uint32_t d = (uint32_t)size;
    uint32_t s = (uint32_t)__builtin_clz(d);
    p.s = s;
    p.dn = d << s;
    p.v = (uint32_t)((~0ULL) / p.dn - (1ULL << 32));
    return p;
}

// remainder of (u1*2^32 + u0) / d for normalized d and u1 < d
RBX_HD uint32_t div21_rem(uint32_t u1, uint32_t u0, uint32_t d, uint32_t v) {
    uint64_t q = (uint64_t)v * u1;
    q += ((uint64_t)u1 << 32) | u0;
    uint32_t q1 = (uint32_t)(q >> 32) + 1u;
    uint32_t q0 = (uint32_t)q;
    uint32_t r = u0 - q1 * d;
    if (r > q0) r += d;
    if (r >= d) r -= d;
    return r;
}

RBX_HD uint32_t mod63(uint64_t h, const ModParams &p) {
    if (p.pow2) return (uint32_t)h & p.mask;
    const uint32_t s = p.s;
    const uint64_t mid = h << s;                        // low 64 bits of h << s
    const uint32_t n2 = s ? (uint32_t)(h >> (64 - s)) : 0u;  // bits 64..94
    uint32_t r = div21_rem(n2, (uint32_t)(mid >> 32), p.dn, p.v);
    r = div21_rem(r, (uint32_t)mid, p.dn, p.v);
    return r >> s;
}

// The fields mod63 reads, in 4 dwords (per-lane copies in register-heavy kernels).
struct ModC {
    uint32_t mask, sp, dn, v;  // sp = s | pow2 << 8
};
RBX_HD ModC mod_compact(const ModParams &p) { return ModC{p.mask, p.s | (p.pow2 << 8), p.dn, p.v}; }
RBX_HD uint32_t mod63c(uint64_t h, const ModC &p) {
    if (p.sp >> 8) return (uint32_t)h & p.mask;
    const uint32_t s = p.sp & 0xff;
    const uint64_t mid = h << s;
    const uint32_t n2 = s ? (uint32_t)(h >> (64 - s)) : 0u;
    uint32_t r = div21_rem(n2, (uint32_t)(mid >> 32), p.dn, p.v);
    r = div21_rem(r, (uint32_t)mid, p.dn, p.v);
    return r >> s;
}

// ---------------------------------------------------------------------------------
// HighwayHash (portable form), Redisson flavour.  State lives in 32 VGPRs.
// ---------------------------------------------------------------------------------
struct HH {
    uint64_t v0[4], v1[4], mul0[4], mul1[4];
};

// Hash.java:30 KEY
constexpr uint64_t kKey0 = 0x9e3779b97f4a7c15ULL, kKey1 = 0xf39cc0605cedc834ULL,
                   kKey2 = 0x1082276bf3a27251ULL, kKey3 = 0xf86c6a11d0c18e95ULL;
constexpr uint64_t kMul0[4] = {0xdbe6d5d5fe4cce2fULL, 0xa4093822299f31d0ULL, 0x13198a2e03707344ULL,
                               0x243f6a8885a308d3ULL};
constexpr uint64_t kMul1[4] = {0x3bd39e10cb0ef593ULL, 0xc0acf169b5f18a8cULL, 0xbe5466cf34e90c6cULL,
                               0x452821e638d01377ULL};
constexpr uint64_t swap32c(uint64_t x) { return (x >> 32) | (x << 32); }

// HighwayHash.java:229-246 reset(), evaluated at compile time for the Redisson KEY.
RBX_HD void hh_reset(HH &s) {
    s.mul0[0] = kMul0[0]; s.mul0[1] = kMul0[1]; s.mul0[2] = kMul0[2]; s.mul0[3] = kMul0[3];
    s.mul1[0] = kMul1[0]; s.mul1[1] = kMul1[1]; s.mul1[2] = kMul1[2]; s.mul1[3] = kMul1[3];
    s.v0[0] = kMul0[0] ^ kKey0; s.v0[1] = kMul0[1] ^ kKey1;
    s.v0[2] = kMul0[2] ^ kKey2; s.v0[3] = kMul0[3] ^ kKey3;
    s.v1[0] = kMul1[0] ^ swap32c(kKey0); s.v1[1] = kMul1[1] ^ swap32c(kKey1);
    s.v1[2] = kMul1[2] ^ swap32c(kKey2); s.v1[3] = kMul1[3] ^ swap32c(kKey3);
}

// v_perm_b32: byte i of the result = byte sel[i] of the 8-byte value {hi:x, lo:y}
// (selectors 0-3 pick y, 4-7 pick x, 0x0c gives 0).  The host build emulates it so the
// CPU self-test exercises the same byte plans.
RBX_HD uint32_t perm_b32(uint32_t x, uint32_t y, uint32_t sel) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __builtin_amdgcn_perm(x, y, sel);
#else
    const uint64_t v = ((uint64_t)x << 32) | y;
    uint32_t r = 0;
    for (int i = 0; i < 4; ++i) {
        const uint32_t s = (sel >> (8 * i)) & 0xffu;
        const uint32_t b = s < 8 ? (uint32_t)(v >> (8 * s)) & 0xffu : 0u;
        r |= b << (8 * i);
    }
    return r;
#endif
}

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));

// Two 32-bit halves as one 64-bit value.  On the device this is a bit cast (a register
// pair): written as `hi << 32 | lo` the compiler turned `x += w2(lo, hi)` into two 64-bit
// adds plus register copies (tools/hashbench.hip: 645 -> 495 VALU instructions per hash).
RBX_HD uint64_t w2(uint32_t lo, uint32_t hi) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __builtin_bit_cast(uint64_t, u32x2{lo, hi});
#else
    return ((uint64_t)hi << 32) | lo;
#endif
}

// 64-bit add of an operand given as halves, as an add-with-carry pair (finalize's swapped
// operands: no register copies to form a pair)
RBX_HD uint64_t add_halves(uint64_t x, uint32_t lo, uint32_t hi) {
#if defined(__HIP_DEVICE_COMPILE__)
    unsigned int c;
    const uint32_t l = __builtin_addc((uint32_t)x, lo, 0u, &c);
    return w2(l, (uint32_t)(x >> 32) + hi + c);
#else
    return x + w2(lo, hi);
#endif
}

// zipperMerge0/1 (HighwayHash.java:248-260).  With a = lower-lane operand (Java's "v0"
// parameter) and b = upper (Java's "v1"), byte j of the result:
//   zm0 = [a3 b4 a2 a5 | b6 a1 b7 a0]      zm1 = [b3 a4 b2 b5 | b1 a6 b0 a7]
// Each high word is one byte permute (v_perm_b32) of two source words; each low word needs three
// source words, but both low words take their two bytes from {a4 a5 b4 b5}, gathered once as
// X = [b4 a5 b5 a4]: the pair costs five permutes instead of six.
RBX_HD void zipper_pair(uint64_t b, uint64_t a, uint64_t &z0, uint64_t &z1) {
    const uint32_t al = (uint32_t)a, ah = (uint32_t)(a >> 32), bl = (uint32_t)b, bh = (uint32_t)(b >> 32);
    const uint32_t x = perm_b32(ah, bh, 0x04010500u);                                // [b4 a5 b5 a4]
    z0 = w2(perm_b32(x, al, 0x05020403u), perm_b32(bh, al, 0x00070106u));  // [a3 b4 a2 a5 | b6 a1 b7 a0]
    z1 = w2(perm_b32(x, bl, 0x06020703u), perm_b32(ah, bl, 0x07000601u));  // [b3 a4 b2 b5 | b1 a6 b0 a7]
}

RBX_HD uint64_t mul32x32(uint64_t x, uint64_t y) {  // (x & 0xffffffff) * (y >> 32)
    return (uint64_t)(uint32_t)x * (uint64_t)(uint32_t)(y >> 32);
}

// HighwayHash.java:93-114 update(), after its first step (v1 += mul0 + a)
RBX_HD void hh_update_tail(HH &s) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        s.mul0[i] ^= mul32x32(s.v1[i], s.v0[i]);
        s.v0[i] += s.mul1[i];
        s.mul1[i] ^= mul32x32(s.v0[i], s.v1[i]);
    }
    uint64_t z0, z1, z2, z3;
    zipper_pair(s.v1[1], s.v1[0], z0, z1);
    zipper_pair(s.v1[3], s.v1[2], z2, z3);
    s.v0[0] += z0;
    s.v0[1] += z1;
    s.v0[2] += z2;
    s.v0[3] += z3;
    zipper_pair(s.v0[1], s.v0[0], z0, z1);
    zipper_pair(s.v0[3], s.v0[2], z2, z3);
    s.v1[0] += z0;
    s.v1[1] += z1;
    s.v1[2] += z2;
    s.v1[3] += z3;
}

// HighwayHash.java:93-114 update()
RBX_HD void hh_update(HH &s, uint64_t a0, uint64_t a1, uint64_t a2, uint64_t a3) {
    s.v1[0] += s.mul0[0] + a0;
    s.v1[1] += s.mul0[1] + a1;
    s.v1[2] += s.mul0[2] + a2;
    s.v1[3] += s.mul0[3] + a3;
    hh_update_tail(s);
}

// streaming (read-once) vector loads of key bytes
__device__ __forceinline__ uint4 ld_nt16(const void *p) {
    const u32x4 v = __builtin_nontemporal_load((const u32x4 *)p);
    return make_uint4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ uint2 ld_nt8(const void *p) {
    const u32x2 v = __builtin_nontemporal_load((const u32x2 *)p);
    return make_uint2(v.x, v.y);
}

// A 32-byte packet given as 8 little-endian words (updatePacket, :71-83).
RBX_HD void hh_packet(HH &s, const uint32_t w[8]) {
    hh_update(s, w2(w[0], w[1]), w2(w[2], w[3]), w2(w[4], w[5]), w2(w[6], w[7]));
}

RBX_HD uint32_t rotl32(uint32_t x, uint32_t c) { return (x << c) | (x >> ((32u - c) & 31u)); }

// updateRemainder (:126-159) prologue: v0 += (r<<32)+r ; rotate32By(r, v1)   (1 <= r <= 31)
RBX_HD void hh_remainder_prologue(HH &s, uint32_t r) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        s.v0[i] += ((uint64_t)r << 32) + r;
        const uint32_t lo = (uint32_t)s.v1[i], hi = (uint32_t)(s.v1[i] >> 32);
        s.v1[i] = w2(rotl32(lo, r), rotl32(hi, r));
    }
}

// permuteAndUpdate (:280-285) x6 and finalize128 (:186-198).  permute() swaps the halves of
// v0[2], v0[3], v0[0], v0[1]; the swapped words are added as halves with a carry.
RBX_HD void hh_finalize128(HH &s, uint64_t &h1, uint64_t &h2) {
#pragma unroll
    for (int r = 0; r < 6; ++r) {
        const uint64_t p0 = s.v0[2], p1 = s.v0[3], p2 = s.v0[0], p3 = s.v0[1];
        s.v1[0] = add_halves(s.v1[0] + s.mul0[0], (uint32_t)(p0 >> 32), (uint32_t)p0);
        s.v1[1] = add_halves(s.v1[1] + s.mul0[1], (uint32_t)(p1 >> 32), (uint32_t)p1);
        s.v1[2] = add_halves(s.v1[2] + s.mul0[2], (uint32_t)(p2 >> 32), (uint32_t)p2);
        s.v1[3] = add_halves(s.v1[3] + s.mul0[3], (uint32_t)(p3 >> 32), (uint32_t)p3);
        hh_update_tail(s);
    }
    h1 = s.v0[0] + s.mul0[0] + s.v1[2] + s.mul1[2];
    h2 = s.v0[1] + s.mul0[1] + s.v1[3] + s.mul1[3];
}

// Builds updateRemainder's 32-byte packet from the tail bytes t[0..r) given as
// 8 little-endian words (bytes past r may hold garbage; they are masked here).
RBX_HD void hh_tail_packet(const uint32_t t[8], uint32_t r, uint32_t p[8]) {
    const uint32_t rem4 = r >> 2;  // number of whole words
    const uint32_t sm4 = r & 3u;
#pragma unroll
    for (int j = 0; j < 8; ++j) p[j] = (uint32_t)j < rem4 ? t[j] : 0u;
    if (r & 16u) {
        // packet[28..31] = bytes[r-4 .. r-1]
        uint32_t lo = 0, hi = 0;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            if ((uint32_t)j == rem4 - 1u) lo = t[j];
            if ((uint32_t)j == rem4) hi = t[j];
        }
        // bytes [4*(rem4-1) + sm4, +4): funnel of (hi:lo) >> 8*sm4
        p[7] = sm4 ? (uint32_t)((((uint64_t)hi << 32) | lo) >> (8 * sm4)) : lo;
    } else if (sm4) {
        uint32_t w = 0;
#pragma unroll
        for (int j = 0; j < 4; ++j)
            if ((uint32_t)j == rem4) w = t[j];
        const uint32_t b0 = w & 0xffu;
        const uint32_t b1 = (w >> (8 * (sm4 >> 1))) & 0xffu;
        const uint32_t b2 = (w >> (8 * (sm4 - 1))) & 0xffu;
        p[4] = b0 | (b1 << 8) | (b2 << 16);
    }
}

// ---------------------------------------------------------------------------------
// Key loads.  A key of `len` bytes at byte address p (any alignment) is read with
// naturally aligned dword loads only (never touching a dword with no key byte in it),
// funnel-shifted into place with v_alignbyte_b32.
// ---------------------------------------------------------------------------------
__device__ __forceinline__ void load_words_unaligned(const uint8_t *p, uint32_t len, uint32_t out[8]) {
    // loads up to 32 bytes [p, p+min(len,32)) into out[0..7]; bytes past len undefined.
    const uintptr_t a = (uintptr_t)p;
    const uint32_t *q = (const uint32_t *)(a & ~(uintptr_t)3);
    const uint32_t sh = (uint32_t)(a & 3u);
    const uint32_t nb = len < 32u ? len : 32u;
    const uint32_t ndw = (sh + nb + 3u) >> 2;  // dwords touched
    uint32_t r[9];
#pragma unroll
    for (int i = 0; i < 9; ++i) r[i] = (uint32_t)i < ndw ? __builtin_nontemporal_load(q + i) : 0u;
#pragma unroll
    for (int i = 0; i < 8; ++i) out[i] = __builtin_amdgcn_alignbyte(r[i + 1], r[i], sh);
}

// HighwayHash128 of an arbitrary-length key (generic path).
__device__ __forceinline__ void hh128_bytes(const uint8_t *p, uint64_t len, uint64_t &h1, uint64_t &h2) {
    HH s;
    hh_reset(s);
    uint64_t i = 0;
    uint32_t w[8];
    for (; i + 32 <= len; i += 32) {
        load_words_unaligned(p + i, 32u, w);
        hh_packet(s, w);
    }
    const uint32_t r = (uint32_t)(len & 31u);
    if (r) {
        uint32_t pk[8];
        load_words_unaligned(p + i, r, w);
        hh_tail_packet(w, r, pk);
        hh_remainder_prologue(s, r);
        hh_packet(s, pk);
    }
    hh_finalize128(s, h1, h2);
}

// HighwayHash128 of a fixed-length key already in registers (L/16 little-endian 16-byte words).
template <int L>
__device__ __forceinline__ void hh128_regs(const uint4 (&x)[L / 16], uint64_t &h1, uint64_t &h2) {
    static_assert(L % 16 == 0 && L > 0, "fast path needs 16-byte multiples");
    HH s;
    hh_reset(s);
    constexpr int NV = L / 16;
#pragma unroll
    for (int pk = 0; pk + 1 < NV; pk += 2) {
        const uint32_t w[8] = {x[pk].x, x[pk].y, x[pk].z, x[pk].w,
                               x[pk + 1].x, x[pk + 1].y, x[pk + 1].z, x[pk + 1].w};
        hh_packet(s, w);
    }
    if (NV & 1) {  // 16 trailing bytes: r = 16 -> words 0..3 + packet[28..31] = bytes 12..15
        const uint4 t = x[NV - 1];
        const uint32_t w[8] = {t.x, t.y, t.z, t.w, 0u, 0u, 0u, t.w};
        hh_remainder_prologue(s, 16u);
        hh_packet(s, w);
    }
    hh_finalize128(s, h1, h2);
}

// HighwayHash128 of a fixed-length key at a 16-byte aligned address (fast path).
template <int L>
__device__ __forceinline__ void hh128_fixed(const uint8_t *p, uint64_t &h1, uint64_t &h2) {
    static_assert(L % 16 == 0 && L > 0, "fast path needs 16-byte multiples");
    const uint4 *v = (const uint4 *)p;
    uint4 x[L / 16];
#pragma unroll
    for (int j = 0; j < L / 16; ++j) x[j] = ld_nt16(v + j);
    hh128_regs<L>(x, h1, h2);
}

// ---------------------------------------------------------------------------------
// Bitmap addressing: device bitmap = the Redis string bytes (MSB-first, bit i in
// byte i>>3 under mask 0x80 >> (i&7), M/RedissonBitSet.java:396-407) read as
// little-endian u32 words: word i>>5, bit ((i ^ 7) & 31).
// ---------------------------------------------------------------------------------
RBX_HD uint32_t bit_in_word(uint32_t idx) { return 1u << ((idx ^ 7u) & 31u); }

// ---------------------------------------------------------------------------------
// MurmurHash64A (seed 0xadc83b19) and hllPatLen [redis-7.2 hyperloglog.c].
// ---------------------------------------------------------------------------------
constexpr uint64_t kMurM = 0xc6a4a7935bd1e995ULL;
constexpr uint64_t kHllSeed = 0xadc83b19ULL;

RBX_HD uint64_t murmur_block(uint64_t h, uint64_t k) {
    k *= kMurM;
    k ^= k >> 47;
    k *= kMurM;
    h ^= k;
    h *= kMurM;
    return h;
}

RBX_HD uint64_t murmur_final(uint64_t h) {
    h ^= h >> 47;
    h *= kMurM;
    h ^= h >> 47;
    return h;
}

// Fixed-length 16-byte-aligned elements (L multiple of 8).
template <int L>
__device__ __forceinline__ uint64_t murmur_fixed(const uint8_t *p) {
    static_assert(L % 8 == 0 && L > 0, "fast path needs 8-byte multiples");
    uint64_t h = kHllSeed ^ ((uint64_t)L * kMurM);
    if constexpr (L % 16 == 0) {
        const uint4 *v = (const uint4 *)p;
#pragma unroll
        for (int j = 0; j < L / 16; ++j) {
            const uint4 x = ld_nt16(v + j);
            h = murmur_block(h, w2(x.x, x.y));
            h = murmur_block(h, w2(x.z, x.w));
        }
    } else {
        const uint2 *v = (const uint2 *)p;
#pragma unroll
        for (int j = 0; j < L / 8; ++j) {
            const uint2 x = ld_nt8(v + j);
            h = murmur_block(h, w2(x.x, x.y));
        }
    }
    return murmur_final(h);
}

// Generic path (any length, any alignment).
__device__ __forceinline__ uint64_t murmur_bytes(const uint8_t *p, uint64_t len) {
    uint64_t h = kHllSeed ^ ((uint64_t)(int64_t)(int32_t)len * kMurM);
    uint64_t i = 0;
    uint32_t w[8];
    for (; i + 32 <= len; i += 32) {
        load_words_unaligned(p + i, 32u, w);
#pragma unroll
        for (int j = 0; j < 4; ++j) h = murmur_block(h, w2(w[2 * j], w[2 * j + 1]));
    }
    const uint32_t r = (uint32_t)(len - i);
    if (r) {
        load_words_unaligned(p + i, r, w);
        const uint32_t nblk = r >> 3;
#pragma unroll
        for (int j = 0; j < 4; ++j)
            if ((uint32_t)j < nblk) h = murmur_block(h, w2(w[2 * j], w[2 * j + 1]));
        const uint32_t t = r & 7u;
        if (t) {
            // tail bytes live in words 2*nblk (and 2*nblk+1)
            uint32_t lo = 0, hi = 0;
#pragma unroll
            for (int j = 0; j < 4; ++j)
                if ((uint32_t)j == nblk) { lo = w[2 * j]; hi = w[2 * j + 1]; }
            uint64_t tail = w2(lo, hi);
            tail &= (t == 8u) ? ~0ULL : ((1ULL << (8 * t)) - 1ULL);
            h ^= tail;
            h *= kMurM;
        }
    }
    return murmur_final(h);
}

// (register index, count) from the 64-bit hash: count = 1 + ctz((h >> 14) | 1<<50).
RBX_HD uint32_t hll_count_of(uint64_t h) {
    const uint64_t x = (h >> 14) | (1ULL << 50);
    return (uint32_t)__builtin_ctzll(x) + 1u;
}

}  // namespace rbx
