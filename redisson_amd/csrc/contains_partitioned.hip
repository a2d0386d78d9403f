// contains_partitioned.hip -- RBloomFilter.contains(Collection) for one large filter
// (M/RedissonBloomFilter.java:153-186) with the bitmap probed from LDS instead of HBM.
//
// Why: a uniformly random 4-byte gather that misses L2 costs one fabric request (measured
// ~55 G requests/s chip-wide, flat from 64 MiB to 1 GiB working sets), the same request rate a
// 128-byte streaming read gets.  A 100M-key batch issues ~4e8 such gathers into a 512 MiB bitmap
// (4.2M cache lines), i.e. ~100 requests per line.  Routing the probes through two streaming
// radix passes turns almost all of them into 8-byte slots of 128-byte streaming requests, and
// the bitmap itself is read once, a 64 KiB region at a time, into LDS.
//
//   K1 stage1 : hash every key, test bit 0 with one random gather (a key is absent at its first
//               0 bit, and on a lightly filled filter most absent keys fail here); `alive` bit per
//               key; the survivors' k-1 remaining bits become (bit index, key id) pairs, bucketed
//               in LDS by coarse bucket (<= 64 buckets of 2^FB regions, each split into kBkSub
//               sub-partitions with their own counters) and written as runs.
//   K3 emit2  : each coarse bucket's pairs re-bucketed by region (2^FB fine buckets).
//   K4 probe  : one workgroup per 64 KiB region: region -> LDS, then every pair of the region
//               tests its bit there; a clear bit (only keys that survived stage 1 by chance)
//               records the key id, bucketed by 2^19-key range.
//   K5 misses : records -> LDS image of the range's miss words -> OR-ed into `miss`.
//   K6 final  : present = alive AND NOT miss; count (+ per-key bytes).
// Measured bound (rocprof PMC, C2): every kernel runs at ~50 G memory requests/s at the L2->EA
// interface (a read moves 128 B, a write 64 B, an atomic is one request), the same rate the
// direct kernel's random gathers get; this path issues ~2.8e8 requests per 1e8 keys where the
// direct kernel issues ~4.4e8.
// Buckets have fixed capacities sized for "every key survives"; a pair that does not fit (only
// for adversarial batches, e.g. one key repeated 1e8 times) is probed directly from HBM where it
// overflows, so the answer is exact in every case.  The answer per key is the AND of its k bits,
// exactly as the direct kernel (bloom_kernels.hip) computes it.
#include "bucket_common.h"

namespace rbx {

constexpr uint32_t kBkRegionWords = 1u << (kBkRegionBits - 5);  // 16384 words = 64 KiB
// Each coarse bucket is split into kBkSub sub-partitions with their own reservation counters;
// stage-1 block b writes to sub-partition b % kBkSub (one counter per bucket would take every
// block's reservation: ~1e5 same-address atomics per counter per 1e8 keys).

// a pair whose bucket is full: test its bit in HBM
__device__ __forceinline__ void bk_direct(unsigned long long e, const uint32_t *__restrict__ bm,
                                          unsigned long long *__restrict__ miss) {
    const uint32_t idx = (uint32_t)(e >> 32), key = (uint32_t)e;
    if ((bm[idx >> 5] & bit_in_word(idx)) == 0u) atomicOr(&miss[key >> 6], 1ULL << (key & 63));
}

// Region pairs (emit2 -> probe) are 6 bytes, split into two arrays: lo = offset in the region
// (19 bits) << 13 | key bits 0-12, hi = key bits 13-26 (chunks hold < 2^27 keys).  Against 8-byte
// pairs this saves a quarter of emit2's write requests and of the probe's read requests.
constexpr uint32_t kBkKeyLoBits = 13;
static_assert(kBkRegionBits + kBkKeyLoBits == 32, "lo word = region offset | low key bits");

__device__ __forceinline__ void bk_put6(unsigned long long e, uint64_t gp, uint32_t *__restrict__ lo,
                                        uint16_t *__restrict__ hi, uint64_t cap, const uint32_t *__restrict__ bm,
                                        unsigned long long *__restrict__ miss) {
    if (gp < cap) {
        const uint32_t idx = (uint32_t)(e >> 32), key = (uint32_t)e;
        run_store(((idx & ((1u << kBkRegionBits) - 1)) << kBkKeyLoBits) |
                                        (key & ((1u << kBkKeyLoBits) - 1)), lo + gp);
        run_store((uint16_t)(key >> kBkKeyLoBits), hi + gp);
    } else {
        bk_direct(e, bm, miss);
    }
}

// Whole-line runs.  A run written at an arbitrary position touches a partial 64-byte line at
// each end, and a partial line costs a full write request: at C2 that was ~1/3 of all write
// requests.  So every reservation is a multiple of the line's entry count (8 pairs of 8 bytes;
// 32 region pairs = 2 lines of lo words + 1 line of hi halves), the remainder of a run carries
// in LDS to the block's next tile, and a block's last remainder is padded to a whole line with
// copies of its last pair (a copy is probed again and sets the same miss bit: no effect).
constexpr uint32_t kBkLine1 = 8, kBkLine2 = 32;

// K1 -----------------------------------------------------------------------------------
// Tile = NT * PER keys.  Hash, test bit 0 (one random gather per key), then the survivors'
// k-1 remaining bits are counted per coarse bucket in LDS, scanned, placed bucket-sorted in an
// LDS image and written out as one run per bucket (one global reservation per bucket per tile).
template <int KMAX> constexpr int bk_per() { return KMAX <= 8 ? 2 : 1; }

template <int KLEN, int KMAX, int NT, int PER>
__global__ __launch_bounds__(NT) void k_bk_stage1(KeysDev keys, uint64_t base, uint64_t nchunk,
                                                   const uint32_t *__restrict__ bm, ModParams mp, uint32_t k,
                                                   uint32_t cshift, uint32_t ncoarse, uint64_t cap1,
                                                   unsigned long long *__restrict__ pairs1, uint32_t *__restrict__ cnt1,
                                                   unsigned long long *__restrict__ alive,
                                                   unsigned long long *__restrict__ miss, uint32_t flags) {
    if (!kDiag) flags = 0;  // wrong-answer diagnostics exist in the profiling build only (rbx_kernels.h)
    constexpr int TILE = NT * PER;
    // dynamic LDS (bk_stage1_lds): image of a tile's pairs with each bucket's carried pairs in
    // front of its new ones, the bucket id of every image slot, the carries, the counters
    extern __shared__ __attribute__((aligned(16))) unsigned char bk_lds[];
    // new pairs + carries (<= 7 per bucket) + line rounding (<= 7 per bucket), ncoarse <= 64
    const uint32_t nimg = TILE * (k - 1) + 128 * (kBkLine1 - 1);
    unsigned long long *s_img = (unsigned long long *)bk_lds;   // [nimg]
    unsigned long long *s_car = s_img + nimg;                     // [128 * kBkLine1] carried pairs
    uint32_t *s_cnt = (uint32_t *)(s_car + 128 * kBkLine1);       // [128]
    uint32_t *s_start = s_cnt + 128, *s_pos = s_start + 128, *s_gb = s_pos + 128, *s_full = s_gb + 128,
             *s_cn = s_full + 128, *s_ncn = s_cn + 128;
    uint8_t *s_bkt = (uint8_t *)(s_ncn + 128);                    // [nimg]
    const uint64_t ntiles = (nchunk + TILE - 1) / TILE;
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint32_t sub = blockIdx.x % kBkSub;
    if (threadIdx.x < 128) s_cn[threadIdx.x] = 0;  // visible after the loop's first barrier
    // Software-pipelined over tiles: tile t+1's hash and bit-0 gather are issued between tile
    // t's bucket scan (whose reservation atomics are then in flight) and tile t's placement,
    // so the VALU-heavy hash overlaps the reservation round trip and the gather has a whole
    // placement + store phase to land.
    uint64_t h1[PER], h2[PER];
    uint32_t w[PER], m[PER];
    auto hash_tile = [&](uint64_t tl) {
        const uint64_t tt0 = tl * TILE + threadIdx.x;
#pragma unroll
        for (int q = 0; q < PER; ++q) {
            const uint64_t t = tt0 + q * NT;
            h1[q] = h2[q] = 0;
            if (t < nchunk) bk_hash<KLEN>(keys, base + t, h1[q], h2[q]);
        }
#pragma unroll
        for (int q = 0; q < PER; ++q) {
            const uint64_t t = tt0 + q * NT;
            w[q] = 0;
            m[q] = 0;
            if (t < nchunk) {
                const uint32_t idx = mod63(h1[q] & 0x7fffffffffffffffULL, mp);
                m[q] = bit_in_word(idx);
                // diagnostics (flags 32, wrong answers): no bit-0 gather; ~54% of keys survive
                if (flags & 32) w[q] = (uint32_t)(h2[q] >> 40) % 100u < 54u ? m[q] : 0u;
                else w[q] = bm[idx >> 5];
            }
        }
    };
    if ((uint64_t)blockIdx.x < ntiles) hash_tile(blockIdx.x);
    if (threadIdx.x < 128) s_cnt[threadIdx.x] = 0;  // later tiles: reset during the placement
    __syncthreads();
    for (uint64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
        const uint64_t t0 = tile * TILE + threadIdx.x;
        uint32_t idx[PER][KMAX - 1];
        bool surv[PER];
#pragma unroll
        for (int q = 0; q < PER; ++q) {
            const uint64_t t = t0 + q * NT;
            surv[q] = (w[q] & m[q]) != 0u;
            const uint64_t mask = __ballot(surv[q]);
            if (lane == 0 && t < nchunk) alive[t >> 6] = mask;  // t is 64-aligned for lane 0
            if (surv[q] && !(flags & 4)) {
                uint64_t h = h1[q] + h2[q];
#pragma unroll
                for (int j = 1; j < KMAX; ++j) {
                    if ((uint32_t)j < k) {
                        idx[q][j - 1] = mod63(h & 0x7fffffffffffffffULL, mp);
                        atomicAdd(&s_cnt[idx[q][j - 1] >> cshift], 1u);
                    }
                    h += (j & 1) ? h1[q] : h2[q];
                }
            }
        }
        __syncthreads();
        if (threadIdx.x < 64) bk_scan128c_al(s_cnt, s_cn, ncoarse, kBkLine1, s_start, s_pos);
        else if (threadIdx.x >= 128 && threadIdx.x - 128 < ncoarse) {
            const uint32_t b = threadIdx.x - 128;
            const uint32_t tot = s_cn[b] + s_cnt[b];
            const uint32_t full = tot & ~(kBkLine1 - 1);
            s_full[b] = full;
            s_ncn[b] = tot - full;
            s_gb[b] = full ? atomicAdd(&cnt1[b * kBkSub + sub], full) : 0u;
        }
        if (tile + gridDim.x < ntiles) hash_tile(tile + gridDim.x);  // the next tile (see above)
        __syncthreads();
        // s_cnt was last read by the scan and the reservations above: reset for the next tile
        // (visible to its counting after this tile's last barrier)
        if (threadIdx.x < 128) s_cnt[threadIdx.x] = 0;
        // the carried pairs go in front of their bucket's new ones; the slots that round each
        // bucket's extent up to a whole line are marked empty (0xff: ncoarse <= 64)
        for (uint32_t j = threadIdx.x; j < ncoarse * kBkLine1; j += NT) {
            const uint32_t b = j / kBkLine1, t = j % kBkLine1;
            if (t < s_cn[b]) {
                s_img[s_start[b] + t] = s_car[j];
                s_bkt[s_start[b] + t] = (uint8_t)b;
            }
            const uint32_t tot = s_full[b] + s_ncn[b];
            if (t < ((kBkLine1 - tot) & (kBkLine1 - 1))) s_bkt[s_start[b] + tot + t] = 0xff;
        }
#pragma unroll
        for (int q = 0; q < PER; ++q) {
            if (surv[q] && !(flags & 4)) {
                const unsigned long long key = (uint32_t)(t0 + q * NT);
#pragma unroll
                for (int j = 1; j < KMAX; ++j) {
                    if ((uint32_t)j < k) {
                        const uint32_t b = idx[q][j - 1] >> cshift;
                        const uint32_t slot = atomicAdd(&s_pos[b], 1u);
                        s_img[slot] = ((unsigned long long)idx[q][j - 1] << 32) | key;
                        s_bkt[slot] = (uint8_t)b;
                    }
                }
            }
        }
        __syncthreads();
        // slot-linear: each bucket's first `full` entries (whole lines) go to its reservation, the
        // rest become its carry; all lanes store, consecutive lanes to consecutive addresses
        const uint32_t total = s_start[ncoarse - 1] + s_full[ncoarse - 1] + s_ncn[ncoarse - 1];
        if (threadIdx.x < ncoarse) s_cn[threadIdx.x] = s_ncn[threadIdx.x];  // carries were placed above
        for (uint32_t i = threadIdx.x; i < total; i += NT) {
            const uint32_t b = s_bkt[i];
            if (b == 0xffu) continue;  // alignment gap
            const uint32_t pos = i - s_start[b];
            const unsigned long long e = s_img[i];
            if (pos < s_full[b]) {
                const uint64_t gp = (uint64_t)s_gb[b] + pos;
                if (gp < cap1) run_store(e, pairs1 + (uint64_t)(b * kBkSub + sub) * cap1 + gp);
                else bk_direct(e, bm, miss);
            } else {
                s_car[b * kBkLine1 + pos - s_full[b]] = e;
            }
        }
        __syncthreads();  // LDS reuse
    }
    // the block's last remainders, padded to whole lines
    for (uint32_t b = wave; b < ncoarse; b += NT / 64) {
        const uint32_t cn = s_cn[b];
        if (cn == 0) continue;  // uniform over the wave
        uint32_t gb = 0;
        if (lane == 0) gb = atomicAdd(&cnt1[b * kBkSub + sub], kBkLine1);
        gb = __shfl(gb, 0, 64);
        if (lane < kBkLine1) {
            const unsigned long long e = s_car[b * kBkLine1 + min(lane, cn - 1)];
            if ((uint64_t)gb + lane < cap1)
                run_store(e, pairs1 + (uint64_t)(b * kBkSub + sub) * cap1 + gb + lane);
            else bk_direct(e, bm, miss);
        }
    }
}

// K3 -----------------------------------------------------------------------------------
// One block per (coarse bucket c, sub-partition) work item, over its 2*PER*NT-pair tiles in order;
// fine bucket = region within c.  Items are numbered c-minor so the blocks running at one time
// reserve from different buckets' region counters.  Runs are whole lines (kBkLine2 pairs), the
// remainder carries to the next tile (s_car), the item's last remainders are padded.
template <int NT, int PER, bool STAMP>
__global__ __launch_bounds__(NT) void k_bk_emit2(const unsigned long long *__restrict__ pairs1,
                                                  const uint32_t *__restrict__ cnt1, uint64_t cap1, uint32_t ncoarse,
                                                  uint32_t fb, uint32_t nregions, uint64_t cap2,
                                                  uint32_t *__restrict__ p2lo, uint16_t *__restrict__ p2hi,
                                                  uint32_t *__restrict__ cnt2,
                                                  const uint32_t *__restrict__ bm, unsigned long long *__restrict__ miss,
                                                  uint32_t flags, unsigned long long *__restrict__ stamps) {
    if (!kDiag) flags = 0;  // wrong-answer diagnostics exist in the profiling build only (rbx_kernels.h)
    PhaseStamps<STAMP, 4> ps;
    ps.start();
    // PER u32x4 (two pairs each) per thread
    constexpr uint32_t TILE = 2 * PER * NT;
    __shared__ __attribute__((aligned(16))) unsigned long long s_img[TILE];
    __shared__ unsigned long long s_car[128 * kBkLine2];
    // s_cnt is double-buffered: a tile counts into one buffer while the other (read by the previous
    // tile's stores) is cleared, which saves the barrier a reset at the top of the tile needed
    __shared__ uint32_t s_cnt2[2][128], s_start[128], s_pos[128], s_gb[128], s_full[128], s_cn[128];
    const uint32_t nf = 1u << fb, fmask = nf - 1;
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint32_t nparts = ncoarse * kBkSub;
    for (uint32_t item = blockIdx.x; item < nparts; item += gridDim.x) {
        const uint32_t c = item % ncoarse, cs = c * kBkSub + item / ncoarse;
        const uint64_t nc = min<uint64_t>(cnt1[cs], cap1);
        if (threadIdx.x < 128) {
            s_cn[threadIdx.x] = 0;
            s_cnt2[0][threadIdx.x] = 0;
        }
        uint32_t par = 0;
        // an item with no pairs goes straight to the remainder loop, whose waves read the
        // counters zeroed above by waves 0-1: LDS holds the previous kernel's bytes otherwise
        __syncthreads();
        // cap1 and TILE are multiples of 64 pairs: every tile is 16-byte aligned
        const u32x4 *src0 = (const u32x4 *)(pairs1 + (uint64_t)cs * cap1);
        u32x4 v[PER];  // the next tile, loaded while the current one is bucketed and written
        auto load = [&](uint64_t st) {
            const uint32_t mm = (uint32_t)min<uint64_t>(TILE, nc - st);
#pragma unroll
            for (int p = 0; p < PER; ++p) {
                v[p] = u32x4{0u, 0u, 0u, 0u};
                if (2 * (p * NT + threadIdx.x) < mm) v[p] = __builtin_nontemporal_load(src0 + st / 2 + p * NT + threadIdx.x);
            }
        };
        if (nc) load(0);
        for (uint64_t start = 0; start < nc; start += TILE) {
            const uint32_t m = (uint32_t)min<uint64_t>(TILE, nc - start);
            uint32_t *s_cnt = s_cnt2[par];
            if (threadIdx.x < 128) s_cnt2[par ^ 1][threadIdx.x] = 0;  // the next tile's (visible after this tile's last barrier)
            unsigned long long e[2 * PER];
#pragma unroll
            for (int p = 0; p < PER; ++p) {
                e[2 * p] = w2(v[p].x, v[p].y);
                e[2 * p + 1] = w2(v[p].z, v[p].w);
            }
#pragma unroll
            for (int p = 0; p < 2 * PER; ++p) {
                const uint32_t q = 2 * ((p >> 1) * NT + threadIdx.x) + (p & 1);
                if (q < m) atomicAdd(&s_cnt[(uint32_t)(e[p] >> (32 + kBkRegionBits)) & fmask], 1u);
            }
            __syncthreads();
            ps.mark(0);
            // the reservation atomics are issued here and their results stored to LDS only after
            // the placement below, which overlaps their round trip (one 1024-thread block per CU:
            // a blocking reservation idled the CU); the next tile's loads follow the atomics
            uint32_t gb = 0;
            if (threadIdx.x < 64) bk_scan128(s_cnt, nf, s_start, s_pos);
            else if (threadIdx.x >= 128 && threadIdx.x - 128 < nf) {
                const uint32_t f = threadIdx.x - 128;
                const uint32_t r = (c << fb) + f;
                const uint32_t full = (s_cn[f] + s_cnt[f]) & ~(kBkLine2 - 1);
                s_full[f] = full;
                if (full && r < nregions) gb = atomicAdd(&cnt2[r], full);
            }
            if (start + TILE < nc) load(start + TILE);
            __syncthreads();
            ps.mark(1);
#pragma unroll
            for (int p = 0; p < 2 * PER; ++p) {
                const uint32_t q = 2 * ((p >> 1) * NT + threadIdx.x) + (p & 1);
                if (q < m) {
                    const uint32_t slot = atomicAdd(&s_pos[(uint32_t)(e[p] >> (32 + kBkRegionBits)) & fmask], 1u);
                    s_img[slot] = e[p];
                }
            }
            if (threadIdx.x >= 128 && threadIdx.x - 128 < nf) s_gb[threadIdx.x - 128] = gb;
            __syncthreads();
            ps.mark(2);
            for (uint32_t f = wave; f < nf; f += NT / 64) {
                const uint32_t n = s_cnt[f], cn = s_cn[f], full = s_full[f], st = s_start[f];
                const uint64_t rb = (uint64_t)((c << fb) + f) * cap2;
                for (uint32_t t = lane; t < full; t += 64) {
                    const unsigned long long v = t < cn ? s_car[f * kBkLine2 + t] : s_img[st + t - cn];
                    bk_put6(v, (uint64_t)s_gb[f] + t, p2lo + rb, p2hi + rb, cap2, bm, miss);
                }
                if (full == 0) {
                    for (uint32_t t = lane; t < n; t += 64) s_car[f * kBkLine2 + cn + t] = s_img[st + t];
                } else {
                    for (uint32_t t = lane; t < cn + n - full; t += 64)
                        s_car[f * kBkLine2 + t] = s_img[st + full - cn + t];
                }
                if (lane == 0) s_cn[f] = cn + n - full;
            }
            par ^= 1u;
            __syncthreads();
            ps.mark(3);
        }
        for (uint32_t f = wave; f < nf; f += NT / 64) {  // the item's last remainders, padded
            const uint32_t cn = s_cn[f];
            if (cn == 0) continue;
            const uint32_t r = (c << fb) + f;
            uint32_t gb = 0;
            if (lane == 0) gb = atomicAdd(&cnt2[r], kBkLine2);
            gb = __shfl(gb, 0, 64);
            if (lane < kBkLine2)
                bk_put6(s_car[f * kBkLine2 + min(lane, cn - 1)], (uint64_t)gb + lane, p2lo + (uint64_t)r * cap2,
                        p2hi + (uint64_t)r * cap2, cap2, bm, miss);
        }
        __syncthreads();  // s_cn / s_car reuse by the next item
        ps.mark(3);
    }
    ps.flush(stamps);
}

// K4 -----------------------------------------------------------------------------------
// A clear bit means the key is absent.  Its key id goes to an LDS record list (one LDS atomic);
// at the end of the region the list is bucketed by 2^19-key range and written as runs, one
// reservation per (region, range), for K5 to turn into miss bits.  A scattered 64-bit
// atomicOr per clear bit (~21M per 1e8 C2 keys: keys that passed bit 0 by chance, ~5.5 clear
// bits each) cost one memory request each; the runs cost ~1 per 13 records.
constexpr uint32_t kBkMissBuf = 3000;  // records per region held in LDS (C2: ~2.6k); beyond: direct atomicOr

__device__ __forceinline__ void bk_miss_direct(uint32_t key, unsigned long long *miss) {
    atomicOr(&miss[key >> 6], 1ULL << (key & 63));
}

__device__ __forceinline__ void bk_test6(const uint32_t *s_bm, uint32_t lo, uint32_t hi, unsigned long long *miss,
                                         uint32_t *s_mrec, uint32_t *s_mn, uint32_t flags) {
    const uint32_t off = lo >> kBkKeyLoBits;
    if ((s_bm[off >> 5] & bit_in_word(off)) == 0u) {  // regions are word-aligned: off's low bits = idx's
        const uint32_t key = (hi << kBkKeyLoBits) | (lo & ((1u << kBkKeyLoBits) - 1));
        if (flags & 8) {
            miss[0] = 0;  // diagnostics: one fixed store instead of the miss
        } else if (flags & 16) {
            bk_miss_direct(key, miss);  // diagnostics: the direct atomic per clear bit (A/B)
        } else {
            const uint32_t slot = atomicAdd(s_mn, 1u);
            if (slot < kBkMissBuf) s_mrec[slot] = key;
            else bk_miss_direct(key, miss);
        }
    }
}

// One block per region; a lane reads 4 pairs at a time (16 B of lo words + 8 B of hi halves),
// 6 groups per round trip, the first round issued together with the region's bitmap load.
template <bool STAMP>
__global__ __launch_bounds__(1024) __attribute__((amdgpu_waves_per_eu(8))) void k_bk_probe(const uint32_t *__restrict__ p2lo,
                                                   const uint16_t *__restrict__ p2hi,
                                                   const uint32_t *__restrict__ cnt2, uint64_t cap2, uint32_t nregions,
                                                   const uint32_t *__restrict__ bm, uint64_t nwords4,
                                                   unsigned long long *__restrict__ miss, uint32_t *__restrict__ mrec,
                                                   uint32_t *__restrict__ mcnt, uint64_t capm, uint32_t nmranges,
                                                   uint32_t flags, unsigned long long *__restrict__ stamps) {
    if (!kDiag) flags = 0;  // wrong-answer diagnostics exist in the profiling build only (rbx_kernels.h)
    PhaseStamps<STAMP, 4> ps;
    ps.start();
    __shared__ __attribute__((aligned(16))) uint32_t s_bm[kBkRegionWords];
    // <= 80 KiB so two blocks share a CU: the bucketed image of the miss records reuses the
    // region bitmap's LDS once the region's probes are done
    __shared__ uint32_t s_mrec[kBkMissBuf];
    uint32_t *s_mimg = s_bm;
    __shared__ uint32_t s_mc[256], s_mst[256], s_mpos[256], s_mgb[256], s_mn;
    constexpr uint32_t NT = 1024, G = 2;
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    for (uint32_t r = blockIdx.x; r < nregions; r += gridDim.x) {
        const uint32_t n = (uint32_t)min<uint64_t>(cnt2[r], cap2);
        if (n == 0) continue;  // uniform
        if (threadIdx.x == 0) s_mn = 0;  // ordered before the probes by the barrier below
        // region bitmap (nwords4 = bitmap words rounded up to 4; the allocation covers them)
        const uint64_t w0 = (uint64_t)r * kBkRegionWords;
        const uint32_t nv = (uint32_t)min<uint64_t>(kBkRegionWords, nwords4 - w0) / 4;
        const u32x4 *srcv = (const u32x4 *)(bm + w0);
        // the region's bitmap goes straight to LDS (global_load_lds, 16 B per lane, lane-linear):
        // no VGPRs held for it, which also removed the kernel's register spills
#pragma unroll
        for (uint32_t i = 0; i < kBkRegionWords / 4 / NT; ++i) {
            const uint32_t j = i * NT + threadIdx.x;
            if (j < nv)
                __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void *)(srcv + j),
                                                 (__attribute__((address_space(3))) void *)((u32x4 *)s_bm + i * NT + wave * 64),
                                                 16, 0, 0);
        }
        // cap2 is a multiple of 64 pairs: the region's lo words are 16-byte and hi halves 8-byte aligned
        const u32x4 *slo = (const u32x4 *)(p2lo + (uint64_t)r * cap2);
        const u32x2 *shi = (const u32x2 *)(p2hi + (uint64_t)r * cap2);
        const uint32_t n4 = (n + 3) >> 2;
        u32x4 vl[G];
        u32x2 vh[G];
#pragma unroll
        for (uint32_t u = 0; u < G; ++u) {
            const uint32_t q = u * NT + threadIdx.x;
            if (q < n4) {
                vl[u] = __builtin_nontemporal_load(slo + q);
                vh[u] = __builtin_nontemporal_load(shi + q);
            }
        }
        __syncthreads();  // waits for the bitmap DMA (and the first pair loads)
        ps.mark(0);
        for (uint32_t base = 0;;) {
#pragma unroll
            for (uint32_t u = 0; u < G; ++u) {
                const uint32_t q = base + u * NT + threadIdx.x;
                if (q < n4) {
                    const uint32_t p0 = 4 * q;
                    bk_test6(s_bm, vl[u].x, vh[u].x & 0xffffu, miss, s_mrec, &s_mn, flags);
                    if (p0 + 1 < n) bk_test6(s_bm, vl[u].y, vh[u].x >> 16, miss, s_mrec, &s_mn, flags);
                    if (p0 + 2 < n) bk_test6(s_bm, vl[u].z, vh[u].y & 0xffffu, miss, s_mrec, &s_mn, flags);
                    if (p0 + 3 < n) bk_test6(s_bm, vl[u].w, vh[u].y >> 16, miss, s_mrec, &s_mn, flags);
                }
            }
            base += G * NT;
            if (base >= n4) break;
#pragma unroll
            for (uint32_t u = 0; u < G; ++u) {
                const uint32_t q = base + u * NT + threadIdx.x;
                if (q < n4) {
                    vl[u] = __builtin_nontemporal_load(slo + q);
                    vh[u] = __builtin_nontemporal_load(shi + q);
                }
            }
        }
        __syncthreads();
        ps.mark(1);
        const uint32_t nm = min(s_mn, kBkMissBuf);
        if (nm) {  // uniform: bucket the region's miss records by key range
            if (threadIdx.x < 256) s_mc[threadIdx.x] = 0;
            __syncthreads();
            for (uint32_t i = threadIdx.x; i < nm; i += NT) atomicAdd(&s_mc[s_mrec[i] >> kBkMissRangeBits], 1u);
            __syncthreads();
            if (threadIdx.x < 64) bk_scan256(s_mc, nmranges, s_mst, s_mpos);
            else if (threadIdx.x >= 256 && threadIdx.x - 256 < nmranges) {
                const uint32_t q = threadIdx.x - 256;
                s_mgb[q] = s_mc[q] ? atomicAdd(&mcnt[q], s_mc[q]) : 0u;
            }
            __syncthreads();
            for (uint32_t i = threadIdx.x; i < nm; i += NT) {
                const uint32_t key = s_mrec[i];
                s_mimg[atomicAdd(&s_mpos[key >> kBkMissRangeBits], 1u)] = key;
            }
            __syncthreads();
            for (uint32_t q = wave; q < nmranges; q += NT / 64) {
                const uint32_t cq = s_mc[q], st = s_mst[q];
                const uint64_t gb = s_mgb[q];
                for (uint32_t t = lane; t < cq; t += 64) {
                    const uint32_t key = s_mimg[st + t];
                    if (gb + t < capm) run_store(key, mrec + (uint64_t)q * capm + gb + t);
                    else bk_miss_direct(key, miss);
                }
            }
        }
        __syncthreads();  // s_bm / s_mrec / s_mn reuse
        ps.mark(2);
    }
    ps.flush(stamps);
}

// K5 -----------------------------------------------------------------------------------
// Miss records -> miss bits.  Item = (key range q, slice of kBkMissSlice records): the slice's
// key ids set bits of a 64 KiB LDS image of the range's miss words, whose nonzero words are
// OR-ed into `miss` (consecutive words: one 64-B atomic request per 16 words).  Many small
// items, not one block per range: one block walking a range's ~1e5 records was latency-bound
// at ~0.5e9 records/s (0.23 ms at C2).
constexpr uint32_t kBkMissSlice = 32768;

__global__ __launch_bounds__(1024) void k_bk_misses(const uint32_t *__restrict__ mrec,
                                                    const uint32_t *__restrict__ mcnt, uint64_t capm,
                                                    uint32_t nmranges, unsigned long long *__restrict__ miss) {
    constexpr uint32_t NT = 1024, W = 1u << (kBkMissRangeBits - 5), PER = kBkMissSlice / NT;
    constexpr uint32_t KM = (1u << kBkMissRangeBits) - 1;
    __shared__ uint32_t s_m[W];  // 64 KiB
    const uint32_t nslices = (uint32_t)((capm + kBkMissSlice - 1) / kBkMissSlice);
    for (uint32_t item = blockIdx.x; item < nmranges * nslices; item += gridDim.x) {
        const uint32_t q = item % nmranges, sl = item / nmranges;
        const uint64_t n = min<uint64_t>(mcnt[q], capm), start = (uint64_t)sl * kBkMissSlice;
        if (start >= n) continue;  // uniform
        const uint32_t m = (uint32_t)min<uint64_t>(kBkMissSlice, n - start);
        const uint32_t *src = mrec + (uint64_t)q * capm + start;
        uint32_t kk[PER];
#pragma unroll
        for (uint32_t u = 0; u < PER; ++u) {
            const uint32_t i = u * NT + threadIdx.x;
            kk[u] = i < m ? __builtin_nontemporal_load(src + i) : 0xffffffffu;
        }
        for (uint32_t w = threadIdx.x; w < W; w += NT) s_m[w] = 0u;
        __syncthreads();
#pragma unroll
        for (uint32_t u = 0; u < PER; ++u)
            if (kk[u] != 0xffffffffu) atomicOr(&s_m[(kk[u] & KM) >> 5], 1u << (kk[u] & 31));
        __syncthreads();
        uint32_t *dst = (uint32_t *)miss + ((uint64_t)q << (kBkMissRangeBits - 5));  // u64 words as LE u32 pairs
        for (uint32_t w = threadIdx.x; w < W; w += NT) {
            const uint32_t v = s_m[w];
            if (v) atomicOr(&dst[w], v);
        }
        __syncthreads();  // s_m reuse
    }
}

// K6 -----------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_bk_final(const unsigned long long *__restrict__ alive,
                                                  const unsigned long long *__restrict__ miss, uint64_t nchunk,
                                                  uint64_t base, uint8_t *__restrict__ out,
                                                  unsigned long long *__restrict__ count) {
    __shared__ unsigned long long s_part[4];
    unsigned long long c = 0;
    const uint64_t ngroups = (nchunk + 63) >> 6;
    for (uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; g < ngroups; g += (uint64_t)gridDim.x * blockDim.x) {
        unsigned long long pres = alive[g] & ~miss[g];
        const uint64_t rem = nchunk - (g << 6);
        if (rem < 64) pres &= (1ULL << rem) - 1;
        c += __popcll(pres);
    }
    if (out) {  // one byte per key, coalesced
        for (uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; t < nchunk; t += (uint64_t)gridDim.x * blockDim.x)
            out[base + t] = (uint8_t)(((alive[t >> 6] & ~miss[t >> 6]) >> (t & 63)) & 1ULL);
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
template <int KLEN, int KMAX, int NT1, int PER>
static void bk_stage1(const PcArgs &a, hipStream_t st) {
    constexpr int TILE = NT1 * PER;
    const uint64_t ntiles1 = (a.nchunk + TILE - 1) / TILE;
    const unsigned g1 = (unsigned)std::min<uint64_t>(ntiles1, 4096);
    const size_t nimg = (size_t)TILE * (a.k - 1) + 128 * (kBkLine1 - 1);
    const size_t lds1 = nimg * 8 + 128 * kBkLine1 * 8 + 7 * 128 * 4 + nimg;
    hipLaunchKernelGGL((k_bk_stage1<KLEN, KMAX, NT1, PER>), dim3(g1), dim3(NT1), lds1, st, a.keys, a.base, a.nchunk, a.bm,
                       a.mp, a.k, a.cshift, a.ncoarse, a.cap1, a.pairs1, a.cnt1, a.alive, a.miss, a.flags);
}

template <int NT2, int PER>
static void bk_emit2(const PcArgs &a, hipStream_t st) {
    // one block per (coarse bucket, sub-partition); tiles start 16-byte aligned (cap1 is a multiple of 8192)
    if (a.stamps)
        hipLaunchKernelGGL((k_bk_emit2<NT2, PER, true>), dim3(a.ncoarse * kBkSub), dim3(NT2), 0, st, a.pairs1, a.cnt1,
                           a.cap1, a.ncoarse, a.fb, a.nregions, a.cap2, a.p2lo, a.p2hi, a.cnt2, a.bm, a.miss, a.flags,
                           a.stamps);
    else
        hipLaunchKernelGGL((k_bk_emit2<NT2, PER, false>), dim3(a.ncoarse * kBkSub), dim3(NT2), 0, st, a.pairs1, a.cnt1,
                           a.cap1, a.ncoarse, a.fb, a.nregions, a.cap2, a.p2lo, a.p2hi, a.cnt2, a.bm, a.miss, a.flags,
                           nullptr);
}

// Shapes: stage 1 at 512 threads with bk_per<KMAX>() keys per thread (1024-key tiles at k <= 8, ~75 KiB
// of LDS, two blocks per CU); emit2 at 1024 threads with 12K-pair tiles (131 KiB, one block per CU; C2
// 4.84 -> 4.74 ms against 8K, profiles/r02/r02u_abt_c2_emit2_tiles.jsonl).  (The A/B shapes behind
// rbx_tune "contains_emit2_nt" / "contains_stage1_per" were removed in r06.)
template <int KLEN, int KMAX>
static void bk_chunk(const PcArgs &a, hipStream_t st) {
    bk_stage1<KLEN, KMAX, 512, bk_per<KMAX>()>(a, st);
    bk_emit2<1024, 6>(a, st);
    if (kDiag && a.stamps)
        hipLaunchKernelGGL((k_bk_probe<true>), dim3(std::min<uint32_t>(a.nregions, 2048)), dim3(1024), 0, st, a.p2lo,
                           a.p2hi, a.cnt2, a.cap2, a.nregions, a.bm, a.nwords4, a.miss, a.mrec, a.mcnt, a.capm, a.nmranges,
                           a.flags, a.stamps + 8);
    else
        hipLaunchKernelGGL((k_bk_probe<false>), dim3(std::min<uint32_t>(a.nregions, 2048)), dim3(1024), 0, st, a.p2lo,
                           a.p2hi, a.cnt2, a.cap2, a.nregions, a.bm, a.nwords4, a.miss, a.mrec, a.mcnt, a.capm, a.nmranges,
                           a.flags, nullptr);
    hipLaunchKernelGGL(k_bk_misses, dim3(2048), dim3(1024), 0, st, a.mrec, a.mcnt, a.capm, a.nmranges, a.miss);
    hipLaunchKernelGGL(k_bk_final, dim3(grid_for_pc(a.nchunk)), dim3(256), 0, st, a.alive, a.miss, a.nchunk, a.base,
                       a.out, a.count);
}

template <int KLEN>
static void bk_chunk_len(const PcArgs &a, hipStream_t st) {
    if (a.k <= 8) bk_chunk<KLEN, 8>(a, st);
    else bk_chunk<KLEN, 16>(a, st);
}

void launch_contains_partitioned_chunk(const PcArgs &a, int klen_fast, hipStream_t st) {
    switch (klen_fast) {
    case 16: bk_chunk_len<16>(a, st); break;
    case 32: bk_chunk_len<32>(a, st); break;
    case 64: bk_chunk_len<64>(a, st); break;
    default: bk_chunk_len<0>(a, st); break;
    }
}

}  // namespace rbx
