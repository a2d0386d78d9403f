// hll_kernels.hip -- RHyperLogLog hot path on gfx950.
//
// Replaces redis-server's PFADD / PFCOUNT / PFMERGE arithmetic [redis-7.2
// src/hyperloglog.c: MurmurHash64A seed 0xadc83b19, hllPatLen, hllDenseSet, hllCount
// with the Ertl estimator] that Redisson reaches through RedissonHyperLogLog.addAllAsync /
// countAsync / mergeWithAsync (M/RedissonHyperLogLog.java:71-102).
//
// Device layout: one byte per register (16384 B per HLL); the Redis dense 6-bit
// string is produced only at export.  PFADD: one workgroup per (command, element tile)
// keeps the 16384 registers as u32 in LDS (64 KiB), folds every element with
// ds_max_u32, then merges into HBM with a bytewise-max CAS per 4-register word; the
// command's reply ("any register changed") is the OR over its tiles.
// M/ = /root/reference/redisson/src/main/java/org/redisson/
#include "rbx_kernels.h"

namespace rbx {

constexpr int kHllRegs = 16384;
constexpr int kPfaddThreads = 1024;

__device__ __forceinline__ uint32_t bytemax4(uint32_t a, uint32_t b) {
    uint32_t r = 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const uint32_t x = (a >> (8 * i)) & 0xffu, y = (b >> (8 * i)) & 0xffu;
        r |= (x > y ? x : y) << (8 * i);
    }
    return r;
}

template <int ELEN>
__device__ __forceinline__ uint64_t elem_hash(const KeysDev &e, uint64_t i) {
    if constexpr (ELEN > 0) {
        return murmur_fixed<ELEN>(e.bytes + i * (uint64_t)ELEN);
    } else {
        uint64_t a, len;
        if (e.offsets) {
            a = e.offsets[i];
            len = e.offsets[i + 1] - a;
            a -= e.off_base;
        } else {
            a = i * e.stride;
            len = e.stride;
        }
        return murmur_bytes(e.bytes + a, len);
    }
}

template <int ELEN>
__global__ __launch_bounds__(kPfaddThreads) void k_hll_pfadd(KeysDev elems, const HllSeg *__restrict__ tiles,
                                                             uint32_t *__restrict__ changed) {
    extern __shared__ __attribute__((aligned(16))) uint32_t lds_regs[];  // 16384 u32
    const HllSeg tile = tiles[blockIdx.x];
    uint4 *l4 = (uint4 *)lds_regs;
    for (int i = threadIdx.x; i < kHllRegs / 4; i += blockDim.x) l4[i] = make_uint4(0, 0, 0, 0);
    __syncthreads();

    uint64_t e = tile.begin + threadIdx.x;
    // 4 elements per lane per round: loads and hashes overlap before the LDS atomics
    for (; e + 3ull * blockDim.x < tile.end; e += 4ull * blockDim.x) {
        uint64_t h[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) h[u] = elem_hash<ELEN>(elems, e + (uint64_t)u * blockDim.x);
#pragma unroll
        for (int u = 0; u < 4; ++u) atomicMax(&lds_regs[h[u] & (kHllRegs - 1)], hll_count_of(h[u]));
    }
    for (; e < tile.end; e += blockDim.x) {
        const uint64_t h = elem_hash<ELEN>(elems, e);
        atomicMax(&lds_regs[h & (kHllRegs - 1)], hll_count_of(h));
    }
    __syncthreads();

    // merge into the HBM registers (4 registers per u32 word)
    uint32_t *g = (uint32_t *)tile.regs;
    int any = 0;
    for (int w = threadIdx.x; w < kHllRegs / 4; w += blockDim.x) {
        const uint4 r = l4[w];
        const uint32_t cand = r.x | (r.y << 8) | (r.z << 16) | (r.w << 24);
        if (!cand) continue;
        uint32_t old = g[w];
        for (;;) {
            const uint32_t nw = bytemax4(old, cand);
            if (nw == old) break;
            const uint32_t prev = atomicCAS(&g[w], old, nw);
            if (prev == old) {
                any = 1;
                break;
            }
            old = prev;
        }
    }
    any = __syncthreads_or(any);
    // every writer stores 1 into a zeroed word: a plain (atomic) store, not an RMW -- the word may sit in
    // coherent host memory (bloom_host_tiny), where a device RMW would be a host-link atomic
    if (threadIdx.x == 0 && any) __hip_atomic_store(&changed[tile.seg], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

void launch_hll_pfadd(const KeysDev &elems, int elen_fast, const HllSeg *d_tiles, uint32_t ntiles,
                      uint32_t *d_changed, hipStream_t st) {
    if (!ntiles) return;
    const size_t lds = kHllRegs * sizeof(uint32_t);
    switch (elen_fast) {
    case 16: hipLaunchKernelGGL(k_hll_pfadd<16>, dim3(ntiles), dim3(kPfaddThreads), lds, st, elems, d_tiles, d_changed); break;
    case 32: hipLaunchKernelGGL(k_hll_pfadd<32>, dim3(ntiles), dim3(kPfaddThreads), lds, st, elems, d_tiles, d_changed); break;
    case 64: hipLaunchKernelGGL(k_hll_pfadd<64>, dim3(ntiles), dim3(kPfaddThreads), lds, st, elems, d_tiles, d_changed); break;
    case 8: hipLaunchKernelGGL(k_hll_pfadd<8>, dim3(ntiles), dim3(kPfaddThreads), lds, st, elems, d_tiles, d_changed); break;
    default: hipLaunchKernelGGL(k_hll_pfadd<0>, dim3(ntiles), dim3(kPfaddThreads), lds, st, elems, d_tiles, d_changed); break;
    }
}

// ---------------------------------------------------------------------------------
// PFCOUNT: register histogram + estimator (hllCount), one 256-thread block per HLL.
// ---------------------------------------------------------------------------------
__device__ double hll_sigma(double x) {
    if (x == 1.) return __builtin_inf();
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

__global__ __launch_bounds__(256) void k_hll_count(uint8_t *const *__restrict__ regs, int *__restrict__ histo,
                                                   unsigned long long *__restrict__ out) {
    __shared__ int h[4][64];
    const uint8_t *r = regs[blockIdx.x];
    const int wid = threadIdx.x >> 6;
    for (int i = threadIdx.x; i < 256; i += blockDim.x) (&h[0][0])[i] = 0;
    __syncthreads();
    const uint4 *r4 = (const uint4 *)r;
    for (int i = threadIdx.x; i < kHllRegs / 16; i += blockDim.x) {
        const uint4 x = r4[i];
        const uint32_t w[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
            for (int b = 0; b < 4; ++b) atomicAdd(&h[wid][(w[j] >> (8 * b)) & 63u], 1);
    }
    __syncthreads();
    if (threadIdx.x < 64) {
        const int t = threadIdx.x;
        const int s = h[0][t] + h[1][t] + h[2][t] + h[3][t];
        h[0][t] = s;
        histo[(size_t)blockIdx.x * 64 + t] = s;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        const int *rh = h[0];
        if (rh[51] != 0) {  // hllTau path: host evaluates it with glibc pow (redis semantics)
            out[blockIdx.x] = ~0ULL;
            return;
        }
        const double m = kHllRegs;
        double z = 0.0;  // m * hllTau(1.0) == 0
        for (int j = 50; j >= 1; --j) {
            z += rh[j];
            z *= 0.5;
        }
        z += m * hll_sigma(rh[0] / (double)m);
        const double E = (double)llround(0.721347520444481703680 * m * m / z);
        out[blockIdx.x] = (unsigned long long)E;
    }
}

void launch_hll_count(uint8_t *const *d_regs, uint32_t n, int *d_histo, unsigned long long *d_out,
                      hipStream_t st) {
    if (!n) return;
    hipLaunchKernelGGL(k_hll_count, dim3(n), dim3(256), 0, st, d_regs, d_histo, d_out);
}

// ---------------------------------------------------------------------------------
// PFMERGE / union: bytewise max over 16384 registers
// ---------------------------------------------------------------------------------
typedef unsigned char u8x16 __attribute__((ext_vector_type(16)));

__global__ __launch_bounds__(256) void k_hll_merge(uint8_t *__restrict__ dst, uint8_t *const *__restrict__ srcs,
                                                   uint32_t nsrc, int init_zero) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;  // one 16-byte vector
    if (i >= kHllRegs / 16) return;
    u8x16 acc = init_zero ? (u8x16)(0) : ((const u8x16 *)dst)[i];
    for (uint32_t s = 0; s < nsrc; ++s) acc = __builtin_elementwise_max(acc, ((const u8x16 *)srcs[s])[i]);
    ((u8x16 *)dst)[i] = acc;
}

void launch_hll_merge(uint8_t *dst, uint8_t *const *d_srcs, uint32_t nsrc, hipStream_t st) {
    hipLaunchKernelGGL(k_hll_merge, dim3(kHllRegs / 16 / 256), dim3(256), 0, st, dst, d_srcs, nsrc, 0);
}

void launch_hll_union(uint8_t *const *d_srcs, uint32_t nsrc, uint8_t *out, hipStream_t st) {
    hipLaunchKernelGGL(k_hll_merge, dim3(kHllRegs / 16 / 256), dim3(256), 0, st, out, d_srcs, nsrc, 1);
}

// ---------------------------------------------------------------------------------
// Sparse strings, replayed ([redis-7.2] hyperloglog.c hllSparseSet, restated in
// oracle/rbx_oracle.c orc_hll_sparse_set).  Redis updates a sparse HLL element by element: the
// opcode covering the register is split into at most three (case D), the string may not grow
// past hll-sparse-max-bytes (else the key is promoted to dense for good), and up to five opcodes
// from the previous one are scanned to merge adjacent VALs of one value (runs of <= 4).  The
// bytes it ends with depend on the order of the updates, so they are replayed here, in command
// order, one block per sparse HLL: the block holds the string as run starts in LDS -- a bitmap
// of the registers that start an opcode (+ a summary of its nonzero words) and the opcode at
// each start -- so finding the opcode that covers a register is two or three LDS reads instead
// of a walk over the string.  The lanes hash 256 elements at a time and mark those that raise
// their register (count > the value the string holds); lane 0 applies them in element order
// (the rest cannot change anything: registers only grow).  The registers themselves are
// updated by k_hll_pfadd / k_hll_merge as for dense keys; this kernel owns only the string
// and the promotion word.
// ---------------------------------------------------------------------------------
namespace sp {
__device__ __forceinline__ bool is_val(uint32_t op) { return op >= 0x80u && op < 0x100u; }
__device__ __forceinline__ bool is_xzero(uint32_t op) { return op >= 0x100u; }
__device__ __forceinline__ uint32_t len(uint32_t op) {
    return op < 0x80u ? op + 1u : (op < 0x100u ? (op & 3u) + 1u : (op & 0x3fffu) + 1u);
}
__device__ __forceinline__ uint32_t bytes(uint32_t op) { return op >= 0x100u ? 2u : 1u; }
__device__ __forceinline__ uint32_t value(uint32_t op) { return ((op >> 2) & 31u) + 1u; }
__device__ __forceinline__ uint32_t mkval(uint32_t v, uint32_t l) { return 0x80u | ((v - 1u) << 2) | (l - 1u); }
__device__ __forceinline__ uint32_t mkzero(uint32_t l) { return l > 64u ? (0x4000u | (l - 1u)) : l - 1u; }

// meta[r] for an opcode starting at register r is its Redis byte for ZERO and VAL, and 0x40 for
// an XZERO, whose length is the distance to the next start (16 KiB of LDS, not 32: 21 KiB per
// block, seven blocks per CU instead of four)
struct Lds {
    unsigned long long bits[256];  // bit r: register r starts an opcode
    unsigned long long sum[4];     // bit w: bits[w] != 0
    uint8_t meta[kHllRegs];
    uint32_t idx[256];
    uint32_t cnt[256];
    unsigned long long mask[4];    // per wave: elements that raise their register
    uint32_t part[256];
    uint32_t nbytes, state, changed;
};

// The bitmap summary as lane 0 holds it while it applies a batch (registers, not LDS: the
// replay is a chain of dependent single-lane accesses), with its running string length.
struct Hot {
    unsigned long long s0, s1, s2, s3;
    uint32_t nbytes;
    __device__ __forceinline__ unsigned long long operator[](uint32_t i) const {
        return i == 0u ? s0 : (i == 1u ? s1 : (i == 2u ? s2 : s3));
    }
    __device__ __forceinline__ void set(uint32_t i, unsigned long long v) {
        if (i == 0u) s0 = v;
        else if (i == 1u) s1 = v;
        else if (i == 2u) s2 = v;
        else s3 = v;
    }
};
struct LdsSum {
    const unsigned long long *p;
    __device__ __forceinline__ unsigned long long operator[](uint32_t i) const { return p[i]; }
};

template <class S>
__device__ __forceinline__ uint32_t pred(const Lds &L, const S &sum, uint32_t r) {  // the start covering r
    const uint32_t w = r >> 6;
    const unsigned long long m = L.bits[w] & (~0ULL >> (63u - (r & 63u)));
    if (m) return (w << 6) + 63u - (uint32_t)__builtin_clzll(m);
    int sw = (int)(w >> 6);
    unsigned long long mm = sum[(uint32_t)sw] & ((1ULL << (w & 63u)) - 1ULL);
    while (!mm) mm = sum[(uint32_t)(--sw)];  // register 0 always starts an opcode
    const uint32_t w2 = ((uint32_t)sw << 6) + 63u - (uint32_t)__builtin_clzll(mm);
    return (w2 << 6) + 63u - (uint32_t)__builtin_clzll(L.bits[w2]);
}

template <class S>
__device__ __forceinline__ uint32_t succ(const Lds &L, const S &sum, uint32_t r) {  // next start after r, or 16384
    const uint32_t w = r >> 6, b = r & 63u;
    const unsigned long long m = b == 63u ? 0ULL : L.bits[w] & (~0ULL << (b + 1u));
    if (m) return (w << 6) + (uint32_t)__builtin_ctzll(m);
    uint32_t sw = w >> 6;
    unsigned long long mm = (w & 63u) == 63u ? 0ULL : sum[sw] & (~0ULL << ((w & 63u) + 1u));
    while (!mm) {
        if (++sw == 4u) return (uint32_t)kHllRegs;
        mm = sum[sw];
    }
    const uint32_t w2 = (sw << 6) + (uint32_t)__builtin_ctzll(mm);
    return (w2 << 6) + (uint32_t)__builtin_ctzll(L.bits[w2]);
}

template <class S>
__device__ __forceinline__ uint32_t opat(const Lds &L, const S &sum, uint32_t r) {  // the u16 opcode at r
    const uint32_t b = L.meta[r];
    return b == 0x40u ? 0x4000u | (succ(L, sum, r) - r - 1u) : b;
}

__device__ __forceinline__ void put(Lds &L, uint32_t r, uint32_t op) { L.meta[r] = (uint8_t)(op >= 0x100u ? 0x40u : op); }

__device__ __forceinline__ void set_start(Lds &L, Hot &H, uint32_t r, uint32_t op) {
    L.bits[r >> 6] |= 1ULL << (r & 63u);
    H.set(r >> 12, H[r >> 12] | (1ULL << ((r >> 6) & 63u)));
    put(L, r, op);
}

__device__ __forceinline__ void clear_start(Lds &L, Hot &H, uint32_t r) {
    const unsigned long long b = L.bits[r >> 6] & ~(1ULL << (r & 63u));
    L.bits[r >> 6] = b;
    if (!b) H.set(r >> 12, H[r >> 12] & ~(1ULL << ((r >> 6) & 63u)));
}

__device__ __forceinline__ uint32_t value_at(const Lds &L, uint32_t r) {
    const uint32_t op = L.meta[pred(L, LdsSum{L.sum}, r)];  // (an XZERO's marker byte is not a VAL either)
    return is_val(op) ? value(op) : 0u;
}

// hllSparseSet on the LDS image (lane 0 only): 0 = no change, 1 = updated, 2 = promote
__device__ uint32_t set(Lds &L, Hot &H, uint32_t index, uint32_t count, uint64_t max_bytes) {
    if (count > 32u) return 2u;  // HLL_SPARSE_VAL_MAX_VALUE
    const uint32_t first = pred(L, H, index), op = opat(L, H, first), span = len(op), last = first + span - 1u;
    if (is_val(op)) {
        if (value(op) >= count) return 0u;  // case A
        if (span == 1u) {                   // case B
            put(L, first, mkval(count, 1u));
            goto updated;
        }
    } else if (!is_xzero(op) && span == 1u) {  // case C
        put(L, first, mkval(count, 1u));
        goto updated;
    }
    {  // case D: split into <= 3 opcodes: [head at first] VAL(count, 1) at index [tail at index + 1]
        const bool zero = !is_val(op), head = index != first, tail = index != last;
        const uint32_t cur = zero ? 0u : value(op);
        const uint32_t qa = head ? (zero ? mkzero(index - first) : mkval(cur, index - first)) : 0u;
        const uint32_t qc = tail ? (zero ? mkzero(last - index) : mkval(cur, last - index)) : 0u;
        const uint32_t seq = 1u + (head ? bytes(qa) : 0u) + (tail ? bytes(qc) : 0u);
        const int delta = (int)seq - (int)bytes(op);
        if (delta > 0 && 16u + (uint64_t)H.nbytes + (uint64_t)delta > max_bytes) return 2u;
        if (head) set_start(L, H, first, qa);
        set_start(L, H, index, mkval(count, 1u));
        if (tail) set_start(L, H, index + 1u, qc);
        H.nbytes = (uint32_t)((int)H.nbytes + delta);
    }
updated:
    {  // merge adjacent VALs of one value, scanning up to 5 opcodes from the previous one
        uint32_t p = first ? pred(L, H, first - 1u) : 0u;
        for (int scan = 5; p < (uint32_t)kHllRegs && scan-- > 0;) {
            const uint32_t o = opat(L, H, p), nx = p + len(o);
            if (is_val(o) && nx < (uint32_t)kHllRegs) {
                const uint32_t o2 = L.meta[nx];
                if (is_val(o2) && value(o2) == value(o) && len(o) + len(o2) <= 4u) {
                    put(L, p, mkval(value(o), len(o) + len(o2)));
                    clear_start(L, H, nx);
                    H.nbytes -= 1u;
                    continue;  // the merged opcode may merge again
                }
            }
            p = nx;
        }
    }
    return 1u;
}

// exclusive block scan of one value per thread (256 threads); returns the total
__device__ __forceinline__ uint32_t block_scan(Lds &L, uint32_t v, uint32_t &excl) {
    const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
    uint32_t x = v;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const uint32_t y = __shfl_up(x, off, 64);
        if (lane >= (uint32_t)off) x += y;
    }
    if (lane == 63u) L.part[wave] = x;
    __syncthreads();
    uint32_t base = 0;
    for (uint32_t w = 0; w < wave; ++w) base += L.part[w];
    const uint32_t total = L.part[0] + L.part[1] + L.part[2] + L.part[3];
    excl = base + x - v;
    __syncthreads();  // part[] reuse
    return total;
}
}  // namespace sp

// A sufficient condition for a promotion inside the update: the final registers hold a value
// > 32, or even their fewest-bytes sparse form exceeds the limit while the string started within
// it.  (Without a promotion every growth of the string was checked, so the final string would fit
// -- and no encoding of the final registers is shorter than the fewest-bytes one.)  Then the replay is skipped: a large batch
// into fresh keys costs a register scan, not an element-by-element walk.  Thread t scans
// registers [64t, 64t + 64); a run is charged by the thread holding its first register, which
// finds the run's end through a suffix minimum of the threads' first run starts.
__device__ bool must_promote(sp::Lds &L, const uint8_t *regs, uint64_t max_bytes, uint64_t canon_max_bytes,
                             bool &canon) {
    const uint32_t t = threadIdx.x, base = t * 64;
    // r06: the thread's 64 registers in four 16-byte loads issued together, and every run measured from
    // them in registers (r05 read a word per loop trip with the loop kept rolled, then re-read each run's
    // first register: ~20 dependent memory round trips per HLL, 0.41 ms of C4's fresh-key step)
    const u32x4 *w4 = (const u32x4 *)(regs + base);
    const u32x4 a0 = w4[0], a1 = w4[1], a2 = w4[2], a3 = w4[3];
    const uint32_t w[16] = {a0.x, a0.y, a0.z, a0.w, a1.x, a1.y, a1.z, a1.w,
                            a2.x, a2.y, a2.z, a2.w, a3.x, a3.y, a3.z, a3.w};
    uint32_t p = t ? regs[base - 1] : 0xffffffffu;
    // runs that start in this thread: each closed one is charged here; the last one's end comes from the
    // suffix minimum of the threads' first run starts below.  bytes: the fewest-bytes encoding; bbound:
    // B = the zero runs' bytes + one byte per nonzero register (no string of these registers is
    // longer); longrun: a nonzero run longer than 4
    uint32_t first = 16384u, cur = 0xffffffffu, curv = 0, vmax = 0, bytes = 0, bbound = 0, longrun = 0;
#pragma unroll
    for (uint32_t i = 0; i < 64; ++i) {
        const uint32_t r = (w[i >> 2] >> (8 * (i & 3))) & 0xffu;
        if (r != p) {
            if (cur != 0xffffffffu) {
                const uint32_t len = base + i - cur;
                bytes += curv == 0 ? (len > 64 ? 2u : 1u) : (len + 3) / 4;
                bbound += curv == 0 ? (len > 64 ? 2u : 1u) : len;
                longrun |= curv != 0 && len > 4;
            } else {
                first = base + i;
            }
            cur = base + i;
            curv = r;
        }
        vmax = r > vmax ? r : vmax;
        p = r;
    }
    uint32_t *s_first = L.idx;  // free until the updates start
    s_first[t] = first;
    __syncthreads();
    for (uint32_t off = 1; off < 256; off <<= 1) {  // suffix minimum, in place
        const uint32_t o = t + off < 256 ? s_first[t + off] : 16384u;
        __syncthreads();
        s_first[t] = min(s_first[t], o);
        __syncthreads();
    }
    if (cur != 0xffffffffu) {  // the last run starting here ends at the next thread's first start
        const uint32_t len = (t + 1 < 256 ? s_first[t + 1] : 16384u) - cur;
        bytes += curv == 0 ? (len > 64 ? 2u : 1u) : (len + 3) / 4;
        bbound += curv == 0 ? (len > 64 ? 2u : 1u) : len;
        longrun |= curv != 0 && len > 4;
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        bytes += __shfl_down(bytes, off, 64);
        bbound += __shfl_down(bbound, off, 64);
        longrun |= __shfl_down(longrun, off, 64);
        vmax = max(vmax, (uint32_t)__shfl_down(vmax, off, 64));
    }
    if ((t & 63) == 0) {
        L.part[t >> 6] = bytes;
        L.part[4 + (t >> 6)] = vmax;
        L.part[8 + (t >> 6)] = bbound;
        L.part[12 + (t >> 6)] = longrun;
    }
    __syncthreads();
    const uint32_t total = L.part[0] + L.part[1] + L.part[2] + L.part[3];
    const uint32_t mx = max(max(L.part[4], L.part[5]), max(L.part[6], L.part[7]));
    const uint32_t bb = L.part[8] + L.part[9] + L.part[10] + L.part[11];
    const uint32_t lr = L.part[12] | L.part[13] | L.part[14] | L.part[15];
    __syncthreads();  // part[] reuse
    canon = mx <= 32u && !lr && 16u + (uint64_t)bb <= canon_max_bytes;
    return mx > 32u || 16u + (uint64_t)total > max_bytes;
}

// The string as it stands is the normalized one (what hll_sparse_pack would give its registers):
// every zero opcode maximal and canonical (XZERO only past 64 registers) and no two adjacent VALs
// of one value.  (createHLLObject's XZERO over 16384 registers is.)
__device__ bool sparse_normalized(sp::Lds &L, const HllReplay &it) {
    const uint32_t t = threadIdx.x, nent = min(it.state[1], (uint32_t)kHllRegs);
    const uint32_t per = (nent + 255u) / 256u, e0 = min(t * per, nent), e1 = min(e0 + per, nent);
    uint32_t bad = 0;
    for (uint32_t e = e0; e < e1; ++e) {
        const uint32_t op = it.ops[e];
        const bool zero = op < 0x40u || op >= 0x100u;
        if (op >= 0x100u && (op & 0x3fffu) + 1u <= 64u) bad = 1;  // an XZERO a ZERO could hold
        if (e + 1 < nent) {
            const uint32_t nx = it.ops[e + 1];
            const bool nzero = nx < 0x40u || nx >= 0x100u;
            if (zero && nzero) bad = 1;                                               // zero runs not maximal
            if (!zero && !nzero && ((op >> 2) & 31u) == ((nx >> 2) & 31u)) bad = 1;  // VALs of one value
        }
    }
    const uint64_t b = __ballot(bad != 0);
    if ((t & 63) == 0) L.part[t >> 6] = b != 0;
    __syncthreads();
    const bool ok = !(L.part[0] | L.part[1] | L.part[2] | L.part[3]);
    __syncthreads();  // part[] reuse
    return ok;
}

// Writes the normalized string of the registers (every run one opcode: all nonzero runs are <= 4
// long) as the HLL's opcode list and its length words.  Thread t encodes the runs starting in
// registers [64t, 64t + 64).
__device__ void sparse_encode_normalized(sp::Lds &L, const uint8_t *regs, uint16_t *ops, uint32_t *state) {
    const uint32_t t = threadIdx.x, base = t * 64;
    uint32_t p = t ? regs[base - 1] : 0xffffffffu;
    uint64_t starts = 0;
    for (uint32_t q = 0; q < 64; ++q) {
        const uint32_t r = regs[base + q];
        if (r != p) starts |= 1ULL << q;
        p = r;
    }
    uint32_t *s_first = L.idx;
    s_first[t] = starts ? base + (uint32_t)__builtin_ctzll(starts) : 16384u;
    __syncthreads();
    for (uint32_t off = 1; off < 256; off <<= 1) {  // suffix minimum, in place
        const uint32_t o = t + off < 256 ? s_first[t + off] : 16384u;
        __syncthreads();
        s_first[t] = min(s_first[t], o);
        __syncthreads();
    }
    const uint32_t next_after = t + 1 < 256 ? s_first[t + 1] : 16384u;
    uint32_t pos, nbytes = 0;
    const uint32_t nops = sp::block_scan(L, (uint32_t)__builtin_popcountll(starts), pos);
    for (uint64_t m = starts; m; m &= m - 1) {
        const uint32_t j = (uint32_t)__builtin_ctzll(m);
        const uint64_t later = m & (m - 1);
        const uint32_t end = later ? base + (uint32_t)__builtin_ctzll(later) : next_after;
        const uint32_t len = end - (base + j), v = regs[base + j];
        const uint32_t op = v ? sp::mkval(v, len) : sp::mkzero(len);
        ops[pos++] = (uint16_t)op;
        nbytes += sp::bytes(op);
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) nbytes += __shfl_down(nbytes, off, 64);
    if ((t & 63) == 0) L.part[t >> 6] = nbytes;
    __syncthreads();
    if (t == 0) {
        state[1] = nops;
        state[2] = L.part[0] + L.part[1] + L.part[2] + L.part[3];
    }
    __syncthreads();  // part[] reuse
}

template <int ELEN>
__device__ void replay_one(sp::Lds &L, const HllReplay &it, const KeysDev &elems, uint64_t max_bytes) {
    if (__hip_atomic_load(it.state, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) return;  // promoted: uniform
    // (a SET string may already exceed the limit and stay sparse through updates that do not grow
    // it: the length argument holds only for strings that start within the limit)
    const uint64_t len0 = 16u + (it.state[1] ? it.state[2] : 2u);
    bool canon;
    if (must_promote(L, it.final_regs, len0 <= max_bytes ? max_bytes : ~0ULL, max_bytes, canon)) {  // uniform
        if (threadIdx.x == 0) it.state[0] = 1u;
        return;
    }
    // Shortcut (r04): from a normalized string, updates whose final registers have no nonzero run
    // longer than 4 and whose bound B (zero-run bytes + one byte per nonzero register, which no
    // intermediate string exceeds: B only grows as registers are raised) fits the limit end in the
    // normalized string of the final registers, whatever their order -- hllSparseSet's merges
    // always join the runs a split or a raise creates when the result is <= 4 long.  Pinned
    // against the oracle's element-by-element hllSparseSet on random and adversarial update
    // sequences (tests/test_oracle.py::test_sparse_normalized_shortcut).  The element-by-element
    // replay below runs only when a condition fails.
    if (canon && sparse_normalized(L, it)) {  // uniform
        sparse_encode_normalized(L, it.final_regs, it.ops, it.state);
        return;
    }
    const uint32_t t = threadIdx.x, lane = t & 63u, wave = t >> 6;
    // load: opcode list -> run starts (thread t takes a contiguous slice of the list)
    const uint32_t nent = min(it.state[1], (uint32_t)kHllRegs);
    L.bits[t] = 0;
    if (t == 0) {
        L.nbytes = nent ? it.state[2] : 2u;
        L.state = 0;
        L.changed = 0;
    }
    const uint32_t per = (nent + 255u) / 256u, e0 = min(t * per, nent), e1 = min(e0 + per, nent);
    uint32_t span = 0;
    for (uint32_t e = e0; e < e1; ++e) span += sp::len(it.ops[e]);
    uint32_t start;
    sp::block_scan(L, span, start);  // (barriers inside order the bits reset)
    for (uint32_t e = e0; e < e1; ++e) {
        const uint32_t op = it.ops[e];
        if (start < (uint32_t)kHllRegs) {
            atomicOr(&L.bits[start >> 6], 1ULL << (start & 63u));
            sp::put(L, start, op);
        }
        start += sp::len(op);
    }
    if (nent == 0 && t == 0) {  // createHLLObject: XZERO over the 16384 registers
        L.bits[0] = 1ULL;
        L.meta[0] = 0x40u;  // XZERO to the end
    }
    __syncthreads();
    {
        const unsigned long long nz = __ballot(L.bits[t] != 0ULL);
        if (lane == 0) L.sum[wave] = nz;
    }
    __syncthreads();
    // updates in order, 256 at a time
    const bool merge = it.regs != nullptr;
    const uint64_t b0 = merge ? 0 : it.begin, b1 = merge ? (uint64_t)kHllRegs : it.end;
    for (uint64_t base = b0; base < b1; base += 256) {
        const uint64_t e = base + t;
        bool cand = false;
        if (e < b1) {
            uint32_t idx, cnt;
            if (merge) {
                idx = (uint32_t)e;
                cnt = it.regs[e];
            } else {
                const uint64_t h = elem_hash<ELEN>(elems, e);
                idx = (uint32_t)(h & (kHllRegs - 1));
                cnt = hll_count_of(h);
            }
            L.idx[t] = idx;
            L.cnt[t] = cnt;
            cand = cnt > sp::value_at(L, idx);
        }
        const unsigned long long m = __ballot(cand);
        if (lane == 0) L.mask[wave] = m;
        __syncthreads();
        if (t == 0) {
            sp::Hot H{L.sum[0], L.sum[1], L.sum[2], L.sum[3], L.nbytes};
            uint32_t state = 0, changed = 0;
            for (uint32_t w = 0; w < 4u && !state; ++w) {
                for (unsigned long long mm = L.mask[w]; mm; mm &= mm - 1) {
                    const uint32_t i = w * 64u + (uint32_t)__builtin_ctzll(mm);
                    const uint32_t r = sp::set(L, H, L.idx[i], L.cnt[i], max_bytes);
                    if (r == 2u) {
                        state = 1;
                        break;
                    }
                    changed |= r;
                }
            }
            L.sum[0] = H.s0;
            L.sum[1] = H.s1;
            L.sum[2] = H.s2;
            L.sum[3] = H.s3;
            L.nbytes = H.nbytes;
            L.state = state;
            L.changed |= changed;
        }
        __syncthreads();
        if (L.state) break;  // uniform
    }
    if (L.state) {
        if (t == 0) it.state[0] = 1u;  // the registers go on in k_hll_pfadd / k_hll_merge
        return;
    }
    if (!L.changed) return;  // uniform
    // write back: thread t serializes the starts of registers [64t, 64t + 64)
    const unsigned long long w = L.bits[t];
    uint32_t pos;
    const uint32_t total = sp::block_scan(L, (uint32_t)__builtin_popcountll(w), pos);
    for (unsigned long long m = w; m; m &= m - 1)
        it.ops[pos++] = (uint16_t)sp::opat(L, sp::LdsSum{L.sum}, t * 64u + (uint32_t)__builtin_ctzll(m));
    if (t == 0) {
        it.state[1] = total;
        it.state[2] = L.nbytes;
    }
}

// a grid of <= 1792 blocks walks the items: a steady PFADD stream into keys that have been
// promoted (the host learns promotions lazily) costs one state load per key, not one block
template <int ELEN>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(7))) void k_hll_sparse_replay(KeysDev elems, const HllReplay *__restrict__ items,
                                                           uint32_t n, uint64_t max_bytes) {
    __shared__ sp::Lds L;
    for (uint32_t i = blockIdx.x; i < n; i += gridDim.x) {
        replay_one<ELEN>(L, items[i], elems, max_bytes);
        __syncthreads();  // L reuse
    }
}

void launch_hll_sparse_replay(const KeysDev &elems, int elen_fast, const HllReplay *items, uint32_t n,
                              uint64_t max_bytes, hipStream_t st) {
    if (!n) return;
    const dim3 grid(std::min<uint32_t>(n, 7 * 256));  // seven 21 KiB blocks per CU, all resident
    switch (elen_fast) {
    case 16: hipLaunchKernelGGL(k_hll_sparse_replay<16>, grid, dim3(256), 0, st, elems, items, n, max_bytes); break;
    case 32: hipLaunchKernelGGL(k_hll_sparse_replay<32>, grid, dim3(256), 0, st, elems, items, n, max_bytes); break;
    case 64: hipLaunchKernelGGL(k_hll_sparse_replay<64>, grid, dim3(256), 0, st, elems, items, n, max_bytes); break;
    case 8: hipLaunchKernelGGL(k_hll_sparse_replay<8>, grid, dim3(256), 0, st, elems, items, n, max_bytes); break;
    default: hipLaunchKernelGGL(k_hll_sparse_replay<0>, grid, dim3(256), 0, st, elems, items, n, max_bytes); break;
    }
}

// recycled pool slots zeroed in one launch (registers + state words), one block per slot
__global__ __launch_bounds__(256) void k_hll_zero(uint8_t *const *__restrict__ regs, uint32_t *const *__restrict__ state) {
    u8x16 *r = (u8x16 *)regs[blockIdx.x];
#pragma unroll
    for (int i = threadIdx.x; i < kHllRegs / 16; i += 256) r[i] = (u8x16)(0);
    if (threadIdx.x < 4) state[blockIdx.x][threadIdx.x] = 0u;
}

void launch_hll_zero(uint8_t *const *d_regs, uint32_t *const *d_state, uint32_t n, hipStream_t st) {
    if (!n) return;
    hipLaunchKernelGGL(k_hll_zero, dim3(n), dim3(256), 0, st, d_regs, d_state);
}

// ---------------------------------------------------------------------------------
// register exchange: HLL i <-> buf[i * 16384 ..], one block per HLL, 16 B per lane
// ---------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_hll_pack(uint8_t *const *__restrict__ regs, uint8_t *__restrict__ buf,
                                                  int unpack_max) {
    u8x16 *r = (u8x16 *)regs[blockIdx.x];
    u8x16 *b = (u8x16 *)(buf + (size_t)blockIdx.x * kHllRegs);
#pragma unroll
    for (int i = threadIdx.x; i < kHllRegs / 16; i += 256) {
        if (unpack_max) r[i] = __builtin_elementwise_max(r[i], b[i]);
        else b[i] = r[i];
    }
}

void launch_hll_pack(uint8_t *const *d_regs, uint32_t n, uint8_t *buf, bool unpack_max, hipStream_t st) {
    if (!n) return;
    hipLaunchKernelGGL(k_hll_pack, dim3(n), dim3(256), 0, st, d_regs, buf, unpack_max ? 1 : 0);
}

}  // namespace rbx
