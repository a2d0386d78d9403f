// add_partitioned.hip -- RBloomFilter.add(Collection) for one large filter
// (M/RedissonBloomFilter.java:104-137) with first-setter resolution in LDS.
//
// The reference executes n*k SETBITs in submission order (CommandBatchService.java:115-134,
// :335, :600-602) and counts a key as new iff one of its replies was 0.  So key i is new iff
// some bit b of key i was 0 before the batch and i is the smallest key id touching b.  The
// table path (bloom_kernels.hip) resolves that with ~28 random memory requests per key (gathers,
// CAS into a first-setter table, lookups, atomicOr).  Here every (bit, key) pair is routed
// through three streaming radix passes to its 32K-bit region, and one workgroup per region
// resolves the owners in LDS:
//   A  k_ba_stage1  : hash, all k pairs per key -> level-1 buckets (<= 64, kBkSub sub-partitions)
//   B  k_ba_rebucket: level 1 -> level 2 (idx >> s2), then level 2 -> regions (idx >> s3)
//   C  k_ba_region  : region bitmap (4 KiB) + owner array (32K x u32, 128 KiB) in LDS; every
//                     initially-0 bit gets owner = atomicMin(key id); owners set the bit; records
//                     (key ids, bucketed by 2^20-key range) name either the owner pairs or the
//                     non-owner pairs (k_ba_mode); bitmap written back
//   D  k_ba_keys    : per key range, owner records -> LDS bitmap -> atomicOr into new_bits, or
//                     non-owner records -> LDS byte counters -> key is new iff its count < k
//   E  k_ba_final   : out_new bytes and the count
// Record kinds: a key is new iff at least one of its k pairs owns its bit.  Into a mostly empty
// filter nearly every pair owns (~n*k owner records, 4 B written + read each) while non-owners
// are only the in-batch collisions (~4% of pairs at 2.7K pairs per 32K-bit region), so there the
// region kernel records the non-owners and the key test becomes "fewer than k non-owner pairs".
// k_ba_mode samples 4096 bitmap words per chunk and picks the kind expected to be rarer (fill
// below 1/2: non-owners).  Both kinds are bounded by k records per key, so capacities and
// results do not depend on the choice.
// Chunks run strictly one after another (each chunk's regions are updated before the next
// chunk's pairs are examined), so the in-order semantics hold across chunks.  Capacities are
// sized for uniform bits; a batch that overflows one (adversarial repeats) sets `overflow`, the
// region/keys/final kernels then do nothing, and the host reruns the chunk on the table path --
// the bitmap is untouched until C, and C checks the flag before writing, so the result is exact
// either way.
#include "bucket_common.h"

namespace rbx {

constexpr uint32_t kBaRegionWords = 1u << (kBaRegionBits - 5);  // 1024
constexpr uint32_t kBaRangeWords = 1u << (kBaKeyRangeBits - 5);  // 32768

__device__ __forceinline__ void ba_write_run(const unsigned long long *s_img, uint32_t st, uint32_t n, uint64_t gb,
                                             unsigned long long *__restrict__ dst, uint64_t cap, uint32_t lane,
                                             uint32_t *__restrict__ overflow) {
    for (uint32_t t = lane; t < n; t += 64) {
        const uint64_t gp = gb + t;
        if (gp < cap) run_store(s_img[st + t], dst + gp);
        else *overflow = 1u;
    }
}

// A ------------------------------------------------------------------------------------
template <int KMAX> constexpr int ba_per() { return KMAX <= 8 ? 2 : 1; }

template <int KLEN, int KMAX>
__global__ __launch_bounds__(512) void k_ba_stage1(KeysDev keys, uint64_t base, uint64_t nchunk, FilterDesc f,
                                                   uint32_t s1, uint32_t ncoarse, uint64_t cap1,
                                                   unsigned long long *__restrict__ p1, uint32_t *__restrict__ cnt1,
                                                   uint32_t *__restrict__ overflow) {
    constexpr int NT = 512, PER = ba_per<KMAX>(), TILE = NT * PER;
    __shared__ __attribute__((aligned(16))) unsigned long long s_img[TILE * KMAX];
    __shared__ uint32_t s_cnt[128], s_start[128], s_pos[128], s_gb[128];
    const uint64_t ntiles = (nchunk + TILE - 1) / TILE;
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint32_t sub = blockIdx.x % kBkSub;
    uint32_t maxidx = 0;
    for (uint64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
        if (threadIdx.x < 128) s_cnt[threadIdx.x] = 0;
        const uint64_t t0 = tile * TILE + threadIdx.x;
        uint32_t idx[PER][KMAX];
#pragma unroll
        for (int q = 0; q < PER; ++q) {
            const uint64_t t = t0 + q * NT;
            uint64_t h1 = 0, h2 = 0;
            if (t < nchunk) bk_hash<KLEN>(keys, base + t, h1, h2);
            uint64_t h = h1;
#pragma unroll
            for (int j = 0; j < KMAX; ++j) {
                if ((uint32_t)j < f.k) idx[q][j] = mod63(h & 0x7fffffffffffffffULL, f.mp);
                h += (j & 1) ? h1 : h2;
            }
        }
        __syncthreads();  // s_cnt reset visible
#pragma unroll
        for (int q = 0; q < PER; ++q) {
            if (t0 + q * NT < nchunk) {
#pragma unroll
                for (int j = 0; j < KMAX; ++j) {
                    if ((uint32_t)j < f.k) {
                        atomicAdd(&s_cnt[idx[q][j] >> s1], 1u);
                        maxidx = idx[q][j] > maxidx ? idx[q][j] : maxidx;
                    }
                }
            }
        }
        __syncthreads();
        if (threadIdx.x < 64) bk_scan128(s_cnt, ncoarse, s_start, s_pos);
        else if (threadIdx.x >= 128 && threadIdx.x - 128 < ncoarse) {
            const uint32_t b = threadIdx.x - 128;
            s_gb[b] = s_cnt[b] ? atomicAdd(&cnt1[b * kBkSub + sub], s_cnt[b]) : 0u;
        }
        __syncthreads();
#pragma unroll
        for (int q = 0; q < PER; ++q) {
            const uint64_t t = t0 + q * NT;
            if (t < nchunk) {
#pragma unroll
                for (int j = 0; j < KMAX; ++j) {
                    if ((uint32_t)j < f.k) {
                        const uint32_t slot = atomicAdd(&s_pos[idx[q][j] >> s1], 1u);
                        s_img[slot] = ((unsigned long long)idx[q][j] << 32) | (uint32_t)t;
                    }
                }
            }
        }
        __syncthreads();
        for (uint32_t b = wave; b < ncoarse; b += NT / 64)
            ba_write_run(s_img, s_start[b], s_cnt[b], s_gb[b], p1 + (uint64_t)(b * kBkSub + sub) * cap1, cap1, lane,
                         overflow);
        __syncthreads();  // LDS reuse
    }
    // Redis string length: every SETBIT grows it to idx/8 + 1 (one atomic per wave)
    uint64_t wmax = maxidx;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        const uint64_t o = __shfl_down(wmax, off, 64);
        wmax = o > wmax ? o : wmax;
    }
    if (lane == 0 && nchunk) {
        const unsigned long long v = (unsigned long long)(wmax >> 3) + 1ULL;
        if (v > __hip_atomic_load(f.redis_len, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) atomicMax(f.redis_len, v);
    }
}

// B ------------------------------------------------------------------------------------
// Input partitions part = parent * sub_div + s (sub_div = kBkSub for level 1, 1 for level 2);
// a pair's output partition = (parent << fo) + ((idx >> shift_out) & (2^fo - 1)).  Work items
// are numbered so that the blocks running at one time read different parents.
__global__ __launch_bounds__(512) void k_ba_rebucket(const unsigned long long *__restrict__ pin,
                                                     const uint32_t *__restrict__ cnt_in, uint64_t cap_in,
                                                     uint32_t nparents, uint32_t sub_div, uint32_t items_per_part,
                                                     uint32_t shift_out, uint32_t fo, uint32_t nparts_out,
                                                     unsigned long long *__restrict__ pout,
                                                     uint32_t *__restrict__ cnt_out, uint64_t cap_out,
                                                     uint32_t *__restrict__ overflow) {
    constexpr int NT = 512, PER = 8, TILE = 16 * NT;  // PER uint4 = two pairs each
    __shared__ __attribute__((aligned(16))) unsigned long long s_img[TILE];
    __shared__ uint32_t s_cnt[128], s_start[128], s_pos[128], s_gb[128];
    const uint32_t nf = 1u << fo, fmask = nf - 1;
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint32_t nparts = nparents * sub_div;
    const uint32_t nitems = nparts * items_per_part;
    for (uint32_t item = blockIdx.x; item < nitems; item += gridDim.x) {
        const uint32_t it = item / nparts, ix = item - it * nparts;
        const uint32_t parent = ix % nparents, part = parent * sub_div + ix / nparents;
        const uint64_t nc = min<uint64_t>(cnt_in[part], cap_in);
        const uint64_t start = (uint64_t)it * TILE;
        if (start >= nc) continue;  // uniform over the block
        const uint32_t m = (uint32_t)min<uint64_t>(TILE, nc - start);
        if (threadIdx.x < 128) s_cnt[threadIdx.x] = 0;
        __syncthreads();
        // cap_in is a multiple of TILE: the tile is 16-byte aligned
        const u32x4 *src = (const u32x4 *)(pin + (uint64_t)part * cap_in + start);
        unsigned long long e[2 * PER];
#pragma unroll
        for (int p = 0; p < PER; ++p) {
            const uint32_t q = 2 * (p * NT + threadIdx.x);
            u32x4 v = {0u, 0u, 0u, 0u};
            if (q < m) v = __builtin_nontemporal_load(src + p * NT + threadIdx.x);
            e[2 * p] = w2(v.x, v.y);
            e[2 * p + 1] = w2(v.z, v.w);
        }
#pragma unroll
        for (int p = 0; p < 2 * PER; ++p) {
            const uint32_t q = 2 * ((p >> 1) * NT + threadIdx.x) + (p & 1);
            if (q < m) atomicAdd(&s_cnt[(uint32_t)(e[p] >> (32 + shift_out)) & fmask], 1u);
        }
        __syncthreads();
        if (threadIdx.x < 64) bk_scan128(s_cnt, nf, s_start, s_pos);
        else if (threadIdx.x >= 128 && threadIdx.x - 128 < nf) {
            const uint32_t f = threadIdx.x - 128;
            const uint32_t r = (parent << fo) + f;
            s_gb[f] = (s_cnt[f] && r < nparts_out) ? atomicAdd(&cnt_out[r], s_cnt[f]) : 0u;
        }
        __syncthreads();
#pragma unroll
        for (int p = 0; p < 2 * PER; ++p) {
            const uint32_t q = 2 * ((p >> 1) * NT + threadIdx.x) + (p & 1);
            if (q < m) {
                const uint32_t slot = atomicAdd(&s_pos[(uint32_t)(e[p] >> (32 + shift_out)) & fmask], 1u);
                s_img[slot] = e[p];
            }
        }
        __syncthreads();
        for (uint32_t f = wave; f < nf; f += NT / 64)
            ba_write_run(s_img, s_start[f], s_cnt[f], s_gb[f], pout + (uint64_t)((parent << fo) + f) * cap_out,
                         cap_out, lane, overflow);
        __syncthreads();
    }
}

// mode -----------------------------------------------------------------------------------
__global__ __launch_bounds__(1024) void k_ba_mode(const uint32_t *__restrict__ bm, uint64_t nwords4, uint32_t policy,
                                                  uint32_t *__restrict__ mode) {
    __shared__ uint32_t s_sum[16];
    uint32_t c = 0;
    if (policy == 2) {
        constexpr uint32_t kSamples = 4096;
#pragma unroll
        for (uint32_t u = 0; u < kSamples / 1024; ++u) {
            const uint64_t i = (uint64_t)(u * 1024 + threadIdx.x);
            c += __popc(bm[i * nwords4 / kSamples]);
        }
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) c += __shfl_down(c, off, 64);
        if ((threadIdx.x & 63) == 0) s_sum[threadIdx.x >> 6] = c;
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        uint32_t m = policy == 3 ? 2u : policy;
        if (policy == 2) {
            uint32_t t = 0;
            for (int w = 0; w < 16; ++w) t += s_sum[w];
            // sampled fill f: below 1/16 the non-owner pairs (~f of all plus ~4% in-batch
            // collisions) are few enough for direct counter atomics; below 1/2 they are still
            // rarer than owners
            m = t < 4096u * 2u ? 2u : t < 4096u * 16u ? 1u : 0u;
        }
        *mode = m;
    }
}

// C ------------------------------------------------------------------------------------
// One block per region at a time (the 128 KiB owner array allows one block per CU); the next
// region's pairs and bitmap word are loaded into registers while the current one is resolved.
// (Measured alternative: touched-once/touched-again bitsets plus a small LDS table for shared
// bits, 70 KiB and two blocks per CU -- no faster.)
constexpr uint32_t kBaRegionThreads = kBaRegionBits >= 15 ? 1024 : 512;

__global__ __launch_bounds__(kBaRegionThreads) void k_ba_region(const unsigned long long *__restrict__ p3,
                                                    const uint32_t *__restrict__ cnt3, uint64_t cap3, uint32_t nregions,
                                                    uint32_t *__restrict__ bm, uint64_t nwords4,
                                                    uint32_t *__restrict__ recs, uint32_t *__restrict__ rec_cnt,
                                                    uint64_t cap_rec, uint32_t nranges,
                                                    const uint32_t *__restrict__ overflow,
                                                    const uint32_t *__restrict__ mode,
                                                    uint32_t *__restrict__ ctr, uint32_t diag) {
    constexpr uint32_t NT = kBaRegionThreads, PER = kBaMaxRegionPairs / NT;
    __shared__ uint32_t s_owner[1u << kBaRegionBits];  // 128 KiB
    __shared__ uint32_t s_bm[kBaRegionWords];          // 4 KiB
    __shared__ uint32_t s_rec[kBaMaxRegionPairs];      // 24 KiB
    __shared__ uint32_t s_rc[128], s_rstart[128], s_rpos[128], s_rgb[128];
    if (*overflow) return;
    const uint32_t md = *mode;
    const bool losers = md != 0;    // records (or counters) name the non-owner pairs
    const bool counters = md == 2;  // non-owner pairs bump their key's byte counter directly
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    constexpr uint32_t kOff = (1u << kBaRegionBits) - 1;
    // Owner entries are epoch-tagged, (62 - epoch) << 26 | key id (key ids < 2^26 per chunk), so
    // an entry left by an earlier region of this block compares larger than any of the current
    // region's and no per-region initialisation (and its barrier) is needed; the array is reset
    // to all-ones at the start and every 63 regions.
    uint32_t epoch = 62;
    auto reset_owners = [&]() {
        for (uint32_t w = threadIdx.x; w < (1u << kBaRegionBits) / 4; w += NT)
            ((u32x4 *)s_owner)[w] = u32x4{~0u, ~0u, ~0u, ~0u};
    };
    // prefetched state of the next two regions (A = r, B = r + grid): two regions' loads stay in
    // flight while one is resolved (one block per CU: the kernel is bound by load latency)
    uint32_t r = blockIdx.x, nA = 0, nB = 0, wA = 0, wB = 0;
    unsigned long long eA[PER], eB[PER];
    auto fetch = [&](uint32_t rr, uint32_t &n, uint32_t &word, unsigned long long (&e)[PER]) {
        n = (uint32_t)min<uint64_t>(cnt3[rr], cap3);
        const uint64_t w0 = (uint64_t)rr * kBaRegionWords;
        if (n && w0 + threadIdx.x < nwords4) word = bm[w0 + threadIdx.x];
        const unsigned long long *src = p3 + (uint64_t)rr * cap3;
#pragma unroll
        for (uint32_t p = 0; p < PER; ++p) {
            const uint32_t q = p * NT + threadIdx.x;
            e[p] = q < n ? __builtin_nontemporal_load(src + q) : 0ULL;
        }
    };
    if (r < nregions) fetch(r, nA, wA, eA);
    if (r + gridDim.x < nregions) fetch(r + gridDim.x, nB, wB, eB);
    while (r < nregions) {
        const uint32_t cur = r, cn = nA;
        const uint64_t w0 = (uint64_t)cur * kBaRegionWords;
        const uint32_t nw = (uint32_t)min<uint64_t>(kBaRegionWords, nwords4 - w0);
        unsigned long long ec[PER];
#pragma unroll
        for (uint32_t p = 0; p < PER; ++p) {
            ec[p] = eA[p];
            eA[p] = eB[p];
        }
        const uint32_t wc = wA;
        nA = nB;
        wA = wB;
        r += gridDim.x;
        if (r + gridDim.x < nregions && !(diag & 8)) fetch(r + gridDim.x, nB, wB, eB);  // two regions ahead
        if (diag & 16) {  // diagnostics: loads only
            unsigned long long acc = wc;
#pragma unroll
            for (uint32_t p = 0; p < PER; ++p) acc ^= ec[p];
            if (acc == 0x9e3779b97f4a7c15ULL) bm[0] = 0u;
            continue;
        }
        if (cn == 0) continue;       // uniform
        if (++epoch == 63) {         // uniform: first region, or 63 regions since the last reset
            epoch = 0;
            reset_owners();
        }
        const uint32_t tag = (62u - epoch) << 26;
        if (threadIdx.x < nw) s_bm[threadIdx.x] = wc;
        if (threadIdx.x < 128) s_rc[threadIdx.x] = 0;
        __syncthreads();
        bool z[PER];
#pragma unroll
        for (uint32_t p = 0; p < PER; ++p) {
            const uint32_t idx = (uint32_t)(ec[p] >> 32);
            z[p] = p * NT + threadIdx.x < cn && (s_bm[(idx & kOff) >> 5] & bit_in_word(idx)) == 0u;
            if (z[p]) atomicMin(&s_owner[idx & kOff], tag | (uint32_t)ec[p]);
        }
        __syncthreads();
        bool any = false, anyrec = false;
#pragma unroll
        for (uint32_t p = 0; p < PER; ++p) {
            const uint32_t idx = (uint32_t)(ec[p] >> 32), key = (uint32_t)ec[p];
            const bool own = z[p] && s_owner[idx & kOff] == (tag | key);  // owner: this pair's SETBIT replies 0
            if (own) {
                any = true;
                atomicOr(&s_bm[(idx & kOff) >> 5], bit_in_word(idx));
            }
            z[p] = losers ? (p * NT + threadIdx.x < cn && !own) : own;  // z = "record this pair"
            if (z[p]) {
                if (counters) {
                    atomicAdd(&ctr[key >> 2], 1u << (8 * (key & 3)));  // no return: not waited on here
                } else {
                    anyrec = true;
                    atomicAdd(&s_rc[key >> kBaKeyRangeBits], 1u);
                }
            }
        }
        // uniform: nothing owned and nothing to record.  Past this point the region's words are
        // written back even if none changed (only a region whose pairs all met set bits, with
        // non-owner records: rare, those are chosen for fills below 1/2).
        if (!__syncthreads_or(any || anyrec)) continue;
        if (counters || (diag & 4)) {  // counters, or diagnostics: bitmap write-back only, no records
            if (threadIdx.x < nw) bm[w0 + threadIdx.x] = s_bm[threadIdx.x];
            __syncthreads();
            continue;
        }
        uint32_t gb = 0;
        const uint32_t qown = threadIdx.x - 128;
        const bool reserver = threadIdx.x >= 128 && qown < nranges;
        if (threadIdx.x < 64) bk_scan128(s_rc, nranges, s_rstart, s_rpos);
        else if (reserver && s_rc[qown]) gb = atomicAdd(&rec_cnt[qown], s_rc[qown]);
        if (threadIdx.x < nw) bm[w0 + threadIdx.x] = s_bm[threadIdx.x];  // region words are this block's
        __syncthreads();
#pragma unroll
        for (uint32_t p = 0; p < PER; ++p) {
            if (z[p]) {
                const uint32_t key = (uint32_t)ec[p];
                s_rec[atomicAdd(&s_rpos[key >> kBaKeyRangeBits], 1u)] = key;
            }
        }
        if (reserver) s_rgb[qown] = gb;  // the reservation's round trip overlapped the placement
        __syncthreads();
        // records per range <= 2^20 keys x k: cap_rec bounds them exactly, no overflow.  (Splitting
        // the range counters 16 ways by block, as stage A does, measured no faster here.)
        for (uint32_t q = wave; q < nranges; q += NT / 64) {
            const uint32_t rn = s_rc[q], st = s_rstart[q];
            uint32_t *dst = recs + (uint64_t)q * cap_rec + s_rgb[q];
            for (uint32_t t = lane; t < rn; t += 64) run_store(s_rec[st + t], dst + t);
        }
        __syncthreads();
    }
}

// D ------------------------------------------------------------------------------------
// Non-owner records: item = (key range q, eighth e of its keys).  The item reads all of range
// q's records and counts those of its 2^17 keys in LDS bytes (a count never exceeds k <= 16);
// a key is new iff its count < k.  The item owns its new_bits words and writes them whole.
__device__ void ba_keys_losers(const uint32_t *__restrict__ recs, const uint32_t *__restrict__ rec_cnt,
                               uint64_t cap_rec, uint32_t nranges, uint32_t k, uint32_t *__restrict__ new_bits,
                               uint32_t *s_cnt) {
    constexpr uint32_t NT = 1024, kSubBits = kBaKeyRangeBits - 3, kSubWords = 1u << (kSubBits - 2);
    const uint32_t nitems = nranges * 8;
    for (uint32_t item = blockIdx.x; item < nitems; item += gridDim.x) {
        const uint32_t q = item % nranges, e = item / nranges;
        const uint32_t m = (uint32_t)min<uint64_t>(rec_cnt[q], cap_rec);
        for (uint32_t w = threadIdx.x; w < kSubWords; w += NT) s_cnt[w] = 0u;
        __syncthreads();
        const uint32_t *src = recs + (uint64_t)q * cap_rec;
        uint32_t i = threadIdx.x;
        for (; i + 3 * NT < m; i += 4 * NT) {
            uint32_t kk[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) kk[u] = __builtin_nontemporal_load(src + i + u * NT);
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const uint32_t l = kk[u] & ((1u << kBaKeyRangeBits) - 1);
                if ((l >> kSubBits) == e) atomicAdd(&s_cnt[(l & ((1u << kSubBits) - 1)) >> 2], 1u << (8 * (l & 3)));
            }
        }
        for (; i < m; i += NT) {
            const uint32_t l = src[i] & ((1u << kBaKeyRangeBits) - 1);
            if ((l >> kSubBits) == e) atomicAdd(&s_cnt[(l & ((1u << kSubBits) - 1)) >> 2], 1u << (8 * (l & 3)));
        }
        __syncthreads();
        // new_bits word w of this eighth covers keys 32w .. 32w+31 = count words 8w .. 8w+7
        uint32_t *dst = new_bits + (uint64_t)q * kBaRangeWords + (uint64_t)e * (kSubWords / 8);
        for (uint32_t w = threadIdx.x; w < kSubWords / 8; w += NT) {
            uint32_t v = 0;
#pragma unroll
            for (uint32_t j = 0; j < 8; ++j) {
                const uint32_t c = s_cnt[8 * w + ((j + w) & 7)];  // rotated: fewer bank conflicts
                const uint32_t jj = (j + w) & 7;
#pragma unroll
                for (uint32_t b = 0; b < 4; ++b) v |= (((c >> (8 * b)) & 0xffu) < k ? 1u : 0u) << (4 * jj + b);
            }
            dst[w] = v;
        }
        __syncthreads();
    }
}

// Owner records: item = (key range q, slice s of 2^20 records): records -> LDS bitmap -> global atomicOr
__global__ __launch_bounds__(1024) void k_ba_keys(const uint32_t *__restrict__ recs,
                                                  const uint32_t *__restrict__ rec_cnt, uint64_t cap_rec,
                                                  uint32_t nranges, uint32_t nslices, uint32_t *__restrict__ new_bits,
                                                  const uint32_t *__restrict__ overflow,
                                                  const uint32_t *__restrict__ mode, uint32_t k,
                                                  uint32_t *__restrict__ ctr) {
    constexpr uint32_t NT = 1024;
    __shared__ uint32_t s_bits[kBaRangeWords];  // 128 KiB
    if (*overflow) return;
    const uint32_t md = *mode;
    if (md == 2) {  // counters: new iff count < k; the counters read are zeroed for the next call
        const uint64_t nw = (uint64_t)nranges << (kBaKeyRangeBits - 5);
        for (uint64_t w = (uint64_t)blockIdx.x * NT + threadIdx.x; w < nw; w += (uint64_t)gridDim.x * NT) {
            u32x4 *src = (u32x4 *)(ctr + 8 * w);
            const u32x4 a = src[0], b = src[1];
            const uint32_t c8[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
            uint32_t v = 0;
#pragma unroll
            for (uint32_t j = 0; j < 8; ++j)
#pragma unroll
                for (uint32_t t = 0; t < 4; ++t) v |= (((c8[j] >> (8 * t)) & 0xffu) < k ? 1u : 0u) << (4 * j + t);
            new_bits[w] = v;
            if (a.x | a.y | a.z | a.w) src[0] = u32x4{0u, 0u, 0u, 0u};
            if (b.x | b.y | b.z | b.w) src[1] = u32x4{0u, 0u, 0u, 0u};
        }
        return;
    }
    if (md == 1) {
        ba_keys_losers(recs, rec_cnt, cap_rec, nranges, k, new_bits, s_bits);
        return;
    }
    const uint32_t nitems = nranges * nslices;
    for (uint32_t item = blockIdx.x; item < nitems; item += gridDim.x) {
        const uint32_t q = item % nranges, s = item / nranges;
        const uint64_t nrec = rec_cnt[q];
        const uint64_t start = (uint64_t)s << kBaKeyRangeBits;
        if (start >= nrec) continue;  // uniform
        const uint32_t m = (uint32_t)min<uint64_t>(1ULL << kBaKeyRangeBits, nrec - start);
        for (uint32_t w = threadIdx.x; w < kBaRangeWords; w += NT) s_bits[w] = 0u;
        __syncthreads();
        const uint32_t *src = recs + (uint64_t)q * cap_rec + start;
        uint32_t i = threadIdx.x;
        for (; i + 7 * NT < m; i += 8 * NT) {
            uint32_t kk[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) kk[u] = __builtin_nontemporal_load(src + i + u * NT);
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                const uint32_t l = kk[u] & ((1u << kBaKeyRangeBits) - 1);
                atomicOr(&s_bits[l >> 5], 1u << (l & 31));
            }
        }
        for (; i < m; i += NT) {
            const uint32_t l = src[i] & ((1u << kBaKeyRangeBits) - 1);
            atomicOr(&s_bits[l >> 5], 1u << (l & 31));
        }
        __syncthreads();
        uint32_t *dst = new_bits + (uint64_t)q * kBaRangeWords;
        for (uint32_t w = threadIdx.x; w < kBaRangeWords; w += NT) {
            const uint32_t v = s_bits[w];
            if (v) atomicOr(&dst[w], v);
        }
        __syncthreads();
    }
}

// E ------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_ba_final(const uint32_t *__restrict__ new_bits, uint64_t nchunk,
                                                  uint64_t base, uint8_t *__restrict__ out_new,
                                                  unsigned long long *__restrict__ count,
                                                  const uint32_t *__restrict__ overflow) {
    __shared__ unsigned long long s_part[4];
    if (*overflow) return;
    unsigned long long c = 0;
    const uint64_t nwords = (nchunk + 31) >> 5;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; g < nwords; g += stride) {
        uint32_t v = new_bits[g];
        const uint64_t rem = nchunk - (g << 5);
        if (rem < 32) v &= (1u << rem) - 1u;
        c += __popc(v);
    }
    if (out_new)
        for (uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; t < nchunk; t += stride)
            out_new[base + t] = (uint8_t)((new_bits[t >> 5] >> (t & 31)) & 1u);
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) c += __shfl_down(c, off, 64);
    if ((threadIdx.x & 63) == 0) s_part[threadIdx.x >> 6] = c;
    __syncthreads();
    if (threadIdx.x == 0) {
        const unsigned long long t = s_part[0] + s_part[1] + s_part[2] + s_part[3];
        if (t && count) atomicAdd(count, t);
    }
}

// launcher ---------------------------------------------------------------------------------
template <int KLEN, int KMAX>
static void ba_chunk(const BaArgs &a, hipStream_t st) {
    constexpr int TILE = 512 * ba_per<KMAX>();
    const uint64_t ntiles = (a.nchunk + TILE - 1) / TILE;
    hipLaunchKernelGGL(k_ba_mode, dim3(1), dim3(1024), 0, st, (const uint32_t *)a.f.bm, a.nwords4, a.record_policy,
                       a.mode);
    hipLaunchKernelGGL((k_ba_stage1<KLEN, KMAX>), dim3((unsigned)std::min<uint64_t>(ntiles, 4096)), dim3(512), 0, st,
                       a.keys, a.base, a.nchunk, a.f, a.s1, a.ncoarse, a.cap1, a.p1, a.cnt1, a.overflow);
    const uint32_t it1 = (uint32_t)((a.cap1 + 8191) / 8192), it2 = (uint32_t)((a.cap2 + 8191) / 8192);
    hipLaunchKernelGGL(k_ba_rebucket, dim3(2048), dim3(512), 0, st, a.p1, a.cnt1, a.cap1, a.ncoarse, kBkSub, it1, a.s2,
                       a.f2, a.n2, a.p2, a.cnt2, a.cap2, a.overflow);
    hipLaunchKernelGGL(k_ba_rebucket, dim3(2048), dim3(512), 0, st, a.p2, a.cnt2, a.cap2, a.n2, 1u, it2, a.s3, a.f3,
                       a.nregions, a.p3, a.cnt3, a.cap3, a.overflow);
    hipLaunchKernelGGL(k_ba_region, dim3(std::min<uint32_t>(a.nregions, 4096)), dim3(kBaRegionThreads), 0, st, a.p3, a.cnt3, a.cap3,
                       a.nregions, a.f.bm, a.nwords4, a.recs, a.rec_cnt, a.cap_rec, a.nranges, a.overflow, a.mode, a.ctr,
                       a.diag);
    hipLaunchKernelGGL(k_ba_keys, dim3(std::min<uint32_t>(a.nranges * std::max<uint32_t>(a.f.k, 8), 2048)), dim3(1024),
                       0, st, a.recs, a.rec_cnt, a.cap_rec, a.nranges, a.f.k, a.new_bits, a.overflow, a.mode, a.f.k, a.ctr);
    hipLaunchKernelGGL(k_ba_final, dim3(grid_for_pc(a.nchunk)), dim3(256), 0, st, a.new_bits, a.nchunk, a.base,
                       a.out_new, a.count, a.overflow);
}

template <int KLEN>
static void ba_chunk_len(const BaArgs &a, hipStream_t st) {
    if (a.f.k <= 8) ba_chunk<KLEN, 8>(a, st);
    else ba_chunk<KLEN, 16>(a, st);
}

void launch_add_partitioned_chunk(const BaArgs &a, int klen_fast, hipStream_t st) {
    switch (klen_fast) {
    case 16: ba_chunk_len<16>(a, st); break;
    case 32: ba_chunk_len<32>(a, st); break;
    case 64: ba_chunk_len<64>(a, st); break;
    default: ba_chunk_len<0>(a, st); break;
    }
}

}  // namespace rbx
