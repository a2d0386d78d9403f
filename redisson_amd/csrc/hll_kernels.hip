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
    if (threadIdx.x == 0 && any) atomicOr(&changed[tile.seg], 1u);
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
// sparse-limit check (one block per HLL): would the registers still fit Redis' sparse string?
// Bytes of the fewest-bytes opcode form: a zero run costs 1 byte (ZERO, <= 64) or 2 (XZERO), a
// run of value v <= 32 costs ceil(len / 4) bytes (VAL); a register > 32 forces dense.  Thread t
// owns registers [64t, 64t + 64); a run is charged by the thread holding its first register,
// which finds the run's end through a suffix minimum of the threads' first run starts.
// ---------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_hll_sparse_check(const HllCheck *__restrict__ items, uint64_t max_bytes) {
    const HllCheck it = items[blockIdx.x];
    __shared__ uint32_t s_first[257];
    __shared__ uint32_t s_sum[4], s_max[4];
    if (__hip_atomic_load(it.promoted, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) return;  // sticky, uniform
    const uint32_t t = threadIdx.x, base = t * 64;
    uint8_t r[64];
    const u8x16 *src = (const u8x16 *)(it.regs + base);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const u8x16 v = src[q];
#pragma unroll
        for (int j = 0; j < 16; ++j) r[q * 16 + j] = v[j];
    }
    const uint32_t prev = t ? it.regs[base - 1] : 0xffffffffu;
    uint64_t starts = 0;
    uint32_t vmax = 0;
#pragma unroll
    for (int j = 0; j < 64; ++j) {
        const uint32_t p = j ? (uint32_t)r[j - 1] : prev;
        if (r[j] != p) starts |= 1ULL << j;
        vmax = r[j] > vmax ? r[j] : vmax;
    }
    s_first[t] = starts ? base + (uint32_t)__builtin_ctzll(starts) : 16384u;
    if (t == 0) s_first[256] = 16384u;
    __syncthreads();
    // suffix minimum over the threads' first starts (256 entries, in place)
    for (uint32_t off = 1; off < 256; off <<= 1) {
        const uint32_t o = t + off < 256 ? s_first[t + off] : 16384u;
        __syncthreads();
        s_first[t] = min(s_first[t], o);
        __syncthreads();
    }
    const uint32_t next_after = t + 1 < 256 ? s_first[t + 1] : 16384u;  // first start past my range
    uint32_t bytes = 0;
    for (uint64_t m = starts; m; m &= m - 1) {
        const uint32_t j = (uint32_t)__builtin_ctzll(m);
        const uint64_t later = m & (m - 1);
        const uint32_t end = later ? base + (uint32_t)__builtin_ctzll(later) : next_after;
        const uint32_t len = end - (base + j), v = r[j];
        bytes += v == 0 ? (len > 64 ? 2u : 1u) : (len + 3) / 4;
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        bytes += __shfl_down(bytes, off, 64);
        vmax = max(vmax, (uint32_t)__shfl_down(vmax, off, 64));
    }
    if ((t & 63) == 0) {
        s_sum[t >> 6] = bytes;
        s_max[t >> 6] = vmax;
    }
    __syncthreads();
    if (t == 0) {
        const uint32_t total = s_sum[0] + s_sum[1] + s_sum[2] + s_sum[3];
        const uint32_t mx = max(max(s_max[0], s_max[1]), max(s_max[2], s_max[3]));
        if (mx > 32 || 16 + (uint64_t)total > max_bytes) *it.promoted = 1u;
    }
}

void launch_hll_sparse_check(const HllCheck *items, uint32_t n, uint64_t max_bytes, hipStream_t st) {
    if (!n) return;
    hipLaunchKernelGGL(k_hll_sparse_check, dim3(n), dim3(256), 0, st, items, max_bytes);
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
