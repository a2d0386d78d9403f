// contains_partitioned.hip -- RBloomFilter.contains(Collection) for one large filter
// (M/RedissonBloomFilter.java:153-186) with region-bucketed probes.
//
// Uniformly random 4-byte gathers over a bitmap larger than the caches run at the fabric's
// random-request rate (~55 G/s measured, flat from 64 MiB to 1 GiB), while gathers confined
// to a 1 MiB region that one XCD keeps in its L2 run at ~130-150 G/s.  A key is absent at its
// first 0 bit, and on a lightly filled filter most absent keys fail their first bit, so:
//   K1 stage1 : hash every key, test bit 0 with one random gather; survivors are compacted per
//               8192-key tile (h1, h2, key id) and their k-1 remaining bits counted per region;
//   K2 scan   : per-region exclusive scan of the tile counts (region-major), region bases;
//   K3 emit   : survivors' remaining bits written as (bit-in-region, key) pairs, bucketed by
//               region (LDS cursors per tile);
//   K4 probe  : workgroup b works on regions b%8, b%8+8, ... (an XCD's L2 holds its region --
//               placement only affects speed); a clear bit sets the key's miss bit;
//   K5 final  : present = survived AND NOT missed; count (+ per-key bytes).
// The answer per key is the AND of its k bits, exactly as the direct kernel computes it.
#include "rbx_kernels.h"

namespace rbx {

constexpr int kPcTile = 8192;        // keys per K1/K3 tile
constexpr int kPcRegionShift = 23;   // 2^23 bits = 1 MiB per region
constexpr int kPcMaxRegions = 512;   // bitmaps up to 2^32 bits

template <int KLEN>
__device__ __forceinline__ void pc_hash(const KeysDev &keys, uint64_t i, uint64_t &h1, uint64_t &h2) {
    if constexpr (KLEN > 0) {
        hh128_fixed<KLEN>(keys.bytes + i * (uint64_t)KLEN, h1, h2);
    } else {
        uint64_t a, len;
        if (keys.offsets) {
            a = keys.offsets[i];
            len = keys.offsets[i + 1] - a;
            a -= keys.off_base;
        } else {
            a = i * keys.stride;
            len = keys.stride;
        }
        hh128_bytes(keys.bytes + a, len, h1, h2);
    }
}

// K1 -----------------------------------------------------------------------------------
template <int KLEN, int KMAX>
__global__ __launch_bounds__(256) void k_pc_stage1(KeysDev keys, uint64_t base, uint64_t nchunk,
                                                   const uint32_t *__restrict__ bm, ModParams mp, uint32_t k,
                                                   uint4 *__restrict__ surv_h, uint32_t *__restrict__ surv_key,
                                                   uint32_t *__restrict__ surv_cnt,
                                                   unsigned long long *__restrict__ survive_bits,
                                                   uint32_t *__restrict__ hist, uint32_t ntiles, uint32_t nregions) {
    __shared__ uint32_t s_hist[kPcMaxRegions];
    __shared__ uint32_t s_cnt;
    const uint32_t tile = blockIdx.x;
    for (uint32_t r = threadIdx.x; r < nregions; r += blockDim.x) s_hist[r] = 0;
    if (threadIdx.x == 0) s_cnt = 0;
    __syncthreads();
    const uint64_t t0 = (uint64_t)tile * kPcTile;
    const uint64_t t1 = min<uint64_t>(t0 + kPcTile, nchunk);
    const int lane = threadIdx.x & 63;
    for (uint64_t it = t0; it < t1; it += blockDim.x) {
        const uint64_t t = it + threadIdx.x;
        bool surv = false;
        uint64_t h1 = 0, h2 = 0;
        if (t < t1) {
            pc_hash<KLEN>(keys, base + t, h1, h2);
            const uint32_t idx0 = mod63(h1 & 0x7fffffffffffffffULL, mp);
            surv = (bm[idx0 >> 5] & bit_in_word(idx0)) != 0u;
            if (surv) {
                uint64_t h = h1 + h2;
#pragma unroll
                for (int j = 1; j < KMAX; ++j) {
                    if ((uint32_t)j < k) {
                        const uint32_t idx = mod63(h & 0x7fffffffffffffffULL, mp);
                        atomicAdd(&s_hist[idx >> kPcRegionShift], 1u);
                    }
                    h += (j & 1) ? h1 : h2;
                }
            }
        }
        const uint64_t mask = __ballot(surv);
        if (lane == 0 && t - lane < t1) survive_bits[(t - lane) >> 6] = mask;  // t - lane is 64-aligned
        uint32_t wbase = 0;
        if (lane == 0 && mask) wbase = atomicAdd(&s_cnt, (uint32_t)__popcll(mask));
        wbase = __shfl(wbase, 0, 64);
        if (surv) {
            const uint32_t pos = wbase + (uint32_t)__popcll(mask & ((1ULL << lane) - 1));
            surv_h[t0 + pos] = make_uint4((uint32_t)h1, (uint32_t)(h1 >> 32), (uint32_t)h2, (uint32_t)(h2 >> 32));
            surv_key[t0 + pos] = (uint32_t)t;
        }
    }
    __syncthreads();
    for (uint32_t r = threadIdx.x; r < nregions; r += blockDim.x) hist[(uint64_t)r * ntiles + tile] = s_hist[r];
    if (threadIdx.x == 0) surv_cnt[tile] = s_cnt;
}

// K2 -----------------------------------------------------------------------------------
// one block per region: exclusive scan of hist[r][0..ntiles) in place, row total out
__global__ __launch_bounds__(1024) void k_pc_scan_rows(uint32_t *__restrict__ hist, uint32_t ntiles,
                                                       unsigned long long *__restrict__ totals) {
    __shared__ unsigned long long s_w[16];
    uint32_t *row = hist + (uint64_t)blockIdx.x * ntiles;
    unsigned long long carry = 0;
    for (uint32_t c0 = 0; c0 < ntiles; c0 += blockDim.x) {
        const uint32_t i = c0 + threadIdx.x;
        const unsigned long long v = i < ntiles ? row[i] : 0;
        // block-wide inclusive scan: wave scan + wave totals
        unsigned long long x = v;
        const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
        for (int off = 1; off < 64; off <<= 1) {
            const unsigned long long y = __shfl_up(x, off, 64);
            if (lane >= off) x += y;
        }
        if (lane == 63) s_w[w] = x;
        __syncthreads();
        if (threadIdx.x == 0) {
            unsigned long long acc = 0;
            for (int q = 0; q < (int)(blockDim.x >> 6); ++q) {
                const unsigned long long tq = s_w[q];
                s_w[q] = acc;
                acc += tq;
            }
        }
        __syncthreads();
        const unsigned long long incl = x + s_w[w];
        if (i < ntiles) row[i] = (uint32_t)(carry + incl - v);
        __syncthreads();
        if (threadIdx.x == blockDim.x - 1) s_w[0] = incl;  // block total
        __syncthreads();
        carry += s_w[0];
        __syncthreads();
    }
    if (threadIdx.x == 0) totals[blockIdx.x] = carry;
}

// single block: exclusive scan of the region totals -> region base and size
__global__ __launch_bounds__(64) void k_pc_scan_totals(const unsigned long long *__restrict__ totals,
                                                       uint32_t nregions, unsigned long long *__restrict__ rbase) {
    if (threadIdx.x == 0) {
        unsigned long long acc = 0;
        for (uint32_t r = 0; r < nregions; ++r) {
            rbase[r] = acc;
            acc += totals[r];
        }
        rbase[nregions] = acc;
    }
}

// K3 -----------------------------------------------------------------------------------
// Sub-batches of kPcSub survivors: their (k-1) pairs are counted per region in LDS, scanned,
// placed region-sorted into an LDS image and written out so each region's pairs of the
// sub-batch leave as one contiguous run (coalesced stores instead of one line per pair).
template <int KMAX> constexpr int pc_sub() { return KMAX <= 8 ? 1024 : 512; }

template <int KMAX>
__global__ __launch_bounds__(256) void k_pc_emit(const uint4 *__restrict__ surv_h, const uint32_t *__restrict__ surv_key,
                                                 const uint32_t *__restrict__ surv_cnt, const uint32_t *__restrict__ hist,
                                                 const unsigned long long *__restrict__ rbase, uint32_t ntiles,
                                                 uint32_t nregions, ModParams mp, uint32_t k,
                                                 unsigned long long *__restrict__ pairs) {
    extern __shared__ __attribute__((aligned(16))) unsigned char pc_lds[];
    unsigned long long *s_gcur = (unsigned long long *)pc_lds;                  // [512] global cursor
    uint32_t *s_cnt = (uint32_t *)(pc_lds + kPcMaxRegions * 8);                // [512] per sub-batch
    uint32_t *s_off = s_cnt + kPcMaxRegions;                                    // [512] scan / LDS cursor
    constexpr int kPcSub = pc_sub<KMAX>();
    uint32_t *s_misc = s_off + kPcMaxRegions;                                   // [4]: total
    unsigned long long *s_img = (unsigned long long *)(s_misc + 4);            // [kPcSub * (KMAX-1)]
    uint32_t *s_rid = (uint32_t *)(s_img + kPcSub * (KMAX - 1));               // region of each image slot
    uint32_t &s_tot = s_misc[0];
    const uint32_t tile = blockIdx.x;
    for (uint32_t r = threadIdx.x; r < nregions; r += blockDim.x) s_gcur[r] = rbase[r] + hist[(uint64_t)r * ntiles + tile];
    const uint32_t n = surv_cnt[tile];
    const uint64_t t0 = (uint64_t)tile * kPcTile;
    for (uint32_t s0 = 0; s0 < n; s0 += kPcSub) {
        const uint32_t sn = min<uint32_t>(kPcSub, n - s0);
        for (uint32_t r = threadIdx.x; r < nregions; r += blockDim.x) s_cnt[r] = 0;
        __syncthreads();
        // pass 1: count per region
        for (uint32_t s = threadIdx.x; s < sn; s += blockDim.x) {
            const uint4 hv = surv_h[t0 + s0 + s];
            const uint64_t h1 = w2(hv.x, hv.y), h2 = w2(hv.z, hv.w);
            uint64_t h = h1 + h2;
#pragma unroll
            for (int j = 1; j < KMAX; ++j) {
                if ((uint32_t)j < k) atomicAdd(&s_cnt[mod63(h & 0x7fffffffffffffffULL, mp) >> kPcRegionShift], 1u);
                h += (j & 1) ? h1 : h2;
            }
        }
        __syncthreads();
        if (threadIdx.x == 0) {  // exclusive scan of <= 512 counts (cheap next to the batch)
            uint32_t acc = 0;
            for (uint32_t r = 0; r < nregions; ++r) {
                s_off[r] = acc;
                acc += s_cnt[r];
            }
            s_tot = acc;
        }
        __syncthreads();
        // pass 2: place region-sorted in LDS
        for (uint32_t s = threadIdx.x; s < sn; s += blockDim.x) {
            const uint4 hv = surv_h[t0 + s0 + s];
            const uint64_t h1 = w2(hv.x, hv.y), h2 = w2(hv.z, hv.w);
            const unsigned long long key = surv_key[t0 + s0 + s];
            uint64_t h = h1 + h2;
#pragma unroll
            for (int j = 1; j < KMAX; ++j) {
                if ((uint32_t)j < k) {
                    const uint32_t idx = mod63(h & 0x7fffffffffffffffULL, mp);
                    const uint32_t r = idx >> kPcRegionShift;
                    const uint32_t slot = atomicAdd(&s_off[r], 1u);
                    s_img[slot] = ((unsigned long long)(idx & ((1u << kPcRegionShift) - 1)) << 32) | key;
                    s_rid[slot] = r;
                }
                h += (j & 1) ? h1 : h2;
            }
        }
        __syncthreads();
        // s_off[r] now = end of region r in the image; its start = end - s_cnt[r]
        const uint32_t tot = s_tot;
        for (uint32_t q = threadIdx.x; q < tot; q += blockDim.x) {
            const uint32_t r = s_rid[q];
            const uint32_t start = s_off[r] - s_cnt[r];
            pairs[s_gcur[r] + (q - start)] = s_img[q];
        }
        __syncthreads();
        for (uint32_t r = threadIdx.x; r < nregions; r += blockDim.x) s_gcur[r] += s_cnt[r];
        __syncthreads();
    }
}

// K4 -----------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_pc_probe(const unsigned long long *__restrict__ pairs,
                                                  const unsigned long long *__restrict__ rbase, uint32_t nregions,
                                                  const uint32_t *__restrict__ bm, uint32_t *__restrict__ miss) {
    const uint32_t xcd = blockIdx.x & 7, local = blockIdx.x >> 3, nlocal = gridDim.x >> 3;
    for (uint32_t r = xcd; r < nregions; r += 8) {
        const uint32_t *region = bm + ((uint64_t)r << (kPcRegionShift - 5));
        const unsigned long long p0 = rbase[r], p1 = rbase[r + 1];
        const unsigned long long step = (unsigned long long)nlocal * blockDim.x;
        unsigned long long p = p0 + (unsigned long long)local * blockDim.x + threadIdx.x;
        // 8 pairs per lane in flight
        for (; p + 7 * step < p1; p += 8 * step) {
            unsigned long long e[8];
            uint32_t w[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) e[u] = __builtin_nontemporal_load(pairs + p + u * step);
#pragma unroll
            for (int u = 0; u < 8; ++u) w[u] = region[(uint32_t)(e[u] >> 32) >> 5];
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                const uint32_t li = (uint32_t)(e[u] >> 32), key = (uint32_t)e[u];
                if ((w[u] & bit_in_word(li)) == 0u) atomicOr(&miss[key >> 5], 1u << (key & 31));
            }
        }
        for (; p < p1; p += step) {
            const unsigned long long e = pairs[p];
            const uint32_t li = (uint32_t)(e >> 32), key = (uint32_t)e;
            if ((region[li >> 5] & bit_in_word(li)) == 0u) atomicOr(&miss[key >> 5], 1u << (key & 31));
        }
    }
}

// K5 -----------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_pc_final(const unsigned long long *__restrict__ survive_bits,
                                                  const unsigned long long *__restrict__ miss, uint64_t nchunk,
                                                  uint64_t base, uint8_t *__restrict__ out,
                                                  unsigned long long *__restrict__ count) {
    __shared__ unsigned long long s_part[4];
    unsigned long long c = 0;
    const uint64_t ngroups = (nchunk + 63) >> 6;
    for (uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; g < ngroups; g += (uint64_t)gridDim.x * blockDim.x) {
        unsigned long long pres = survive_bits[g] & ~miss[g];
        const uint64_t rem = nchunk - (g << 6);
        if (rem < 64) pres &= (1ULL << rem) - 1;
        c += __popcll(pres);
        if (out) {
            const uint64_t n = rem < 64 ? rem : 64;
            for (uint64_t b = 0; b < n; ++b) out[base + (g << 6) + b] = (pres >> b) & 1;
        }
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) c += __shfl_down(c, off, 64);
    if ((threadIdx.x & 63) == 0) s_part[threadIdx.x >> 6] = c;
    __syncthreads();
    if (threadIdx.x == 0) {
        const unsigned long long t = s_part[0] + s_part[1] + s_part[2] + s_part[3];
        if (t && count) atomicAdd(count, t);
    }
}

// launcher -------------------------------------------------------------------------------
template <int KLEN, int KMAX>
static void pc_chunk(const PcArgs &a, hipStream_t st) {
    const uint32_t ntiles = (uint32_t)((a.nchunk + kPcTile - 1) / kPcTile);
    hipLaunchKernelGGL((k_pc_stage1<KLEN, KMAX>), dim3(ntiles), dim3(256), 0, st, a.keys, a.base, a.nchunk, a.bm, a.mp,
                       a.k, a.surv_h, a.surv_key, a.surv_cnt, a.survive_bits, a.hist, ntiles, a.nregions);
    hipLaunchKernelGGL(k_pc_scan_rows, dim3(a.nregions), dim3(1024), 0, st, a.hist, ntiles, a.totals);
    hipLaunchKernelGGL(k_pc_scan_totals, dim3(1), dim3(64), 0, st, a.totals, a.nregions, a.rbase);
    const size_t lds = kPcMaxRegions * 16 + 16 + (size_t)pc_sub<KMAX>() * (KMAX - 1) * 12;
    hipLaunchKernelGGL((k_pc_emit<KMAX>), dim3(ntiles), dim3(256), lds, st, a.surv_h, a.surv_key, a.surv_cnt, a.hist,
                       a.rbase, ntiles, a.nregions, a.mp, a.k, a.pairs);
    hipLaunchKernelGGL(k_pc_probe, dim3(a.probe_grid), dim3(256), 0, st, a.pairs, a.rbase, a.nregions, a.bm,
                       (uint32_t *)a.miss);
    hipLaunchKernelGGL(k_pc_final, dim3(grid_for_pc(a.nchunk)), dim3(256), 0, st, a.survive_bits, a.miss, a.nchunk,
                       a.base, a.out, a.count);
}

template <int KLEN>
static void pc_chunk_len(const PcArgs &a, hipStream_t st) {
    if (a.k <= 8) pc_chunk<KLEN, 8>(a, st);
    else pc_chunk<KLEN, 16>(a, st);
}

void launch_contains_partitioned_chunk(const PcArgs &a, int klen_fast, hipStream_t st) {
    switch (klen_fast) {
    case 16: pc_chunk_len<16>(a, st); break;
    case 32: pc_chunk_len<32>(a, st); break;
    case 64: pc_chunk_len<64>(a, st); break;
    default: pc_chunk_len<0>(a, st); break;
    }
}

}  // namespace rbx
