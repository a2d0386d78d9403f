// bloom_kernels.hip -- RBloomFilter hot path on gfx950.
//
// Replaces, per key: Hash.hash128 (M/misc/Hash.java:53-74) -> hash(h1,h2,k,size)
// (M/RedissonBloomFilter.java:139-151) -> k pipelined SETBIT/GETBIT commands through
// CommandBatchService (:112-118, :161-167) executed by redis-server's bitops.c.
//
// contains: one lane per key, k independent 4-byte gathers in flight per lane.
// add: the reference counts a key as new iff one of its k SETBIT replies was 0, with
//   the batch executed strictly in submission order (CommandBatchService.java:115-134,
//   :335, :600-602).  So key i is new iff some bit b of key i was 0 before the batch
//   and no earlier key j < i of the batch touches b.  Three steps reproduce that
//   exactly under full parallelism:
//     probe : gather the k bits; for every bit that is 0, insert (bit, key) into a
//             first-setter table with a 64-bit atomicMin on the key id;
//     commit: a key owning (= minimum id of) any of its zero bits is new; owners
//             atomicOr their bits into the bitmap.
//   Keys are processed in chunks that each finish before the next probes, so chunking
//   preserves the in-order semantics.
// M/ = /root/reference/redisson/src/main/java/org/redisson/
#include "bloom_common.h"

#include <atomic>

namespace rbx {

// ---------------------------------------------------------------------------------
// contains
// ---------------------------------------------------------------------------------
// Loads bits [J0, J1) of the key (h already advanced to hash J0) and returns their AND.
template <int J0, int J1>
__device__ __forceinline__ bool probe_range(const uint32_t *__restrict__ bm, const ModParams &mp, uint32_t k,
                                            uint64_t &h, uint64_t h1, uint64_t h2) {
    uint32_t word[J1 - J0], mask[J1 - J0];
#pragma unroll
    for (int j = J0; j < J1; ++j) {
        if ((uint32_t)j < k) {
            const uint32_t idx = mod63(h & 0x7fffffffffffffffULL, mp);
            word[j - J0] = bm[idx >> 5];
            mask[j - J0] = bit_in_word(idx);
        }
        h += (j & 1) ? h1 : h2;
    }
    bool all = true;
#pragma unroll
    for (int j = J0; j < J1; ++j)
        if ((uint32_t)j < k) all &= (word[j - J0] & mask[j - J0]) != 0u;
    return all;
}

// Tests the k bits of one key (KMAX >= k, unrolled).  All loads of a stage issue before any
// is used.  A key is absent as soon as one bit is 0, so later stages run only while every
// bit so far is set (early exit; the result is identical).  Schedules (SCHED):
//   0: one stage of k loads          1: 1, then k-1        2: 2, then k-2
//   3: 3, then k-3                   4: doubling 1, 2, 4, 8 ...
// On a filter with fill f an absent key costs ~1 + (k-1) f gathers under schedule 1 and
// ~1 + 2f + 4f^3 under schedule 4 (the better one when f is large, e.g. 0.5 at design load).
template <int KMAX, int SCHED = 0>
__device__ __forceinline__ bool probe_all_set(const uint32_t *__restrict__ bm, const ModParams &mp,
                                              uint32_t k, uint64_t h1, uint64_t h2) {
    if constexpr (KMAX > 0) {
        uint64_t h = h1;
        if constexpr (SCHED == 0 || KMAX <= 1) {
            return probe_range<0, KMAX>(bm, mp, k, h, h1, h2);
        } else if constexpr (SCHED >= 1 && SCHED <= 3) {
            constexpr int S = SCHED < KMAX ? SCHED : KMAX;
            if (!probe_range<0, S>(bm, mp, k, h, h1, h2)) return false;
            if (k <= (uint32_t)S) return true;
            return probe_range<S, KMAX>(bm, mp, k, h, h1, h2);
        } else {  // doubling
            if (!probe_range<0, 1>(bm, mp, k, h, h1, h2)) return false;
            if (k <= 1) return true;
            if constexpr (KMAX > 1) {
                constexpr int E2 = KMAX < 3 ? KMAX : 3;
                if (!probe_range<1, E2>(bm, mp, k, h, h1, h2)) return false;
                if (k <= (uint32_t)E2) return true;
            }
            if constexpr (KMAX > 3) {
                constexpr int E3 = KMAX < 7 ? KMAX : 7;
                if (!probe_range<3, E3>(bm, mp, k, h, h1, h2)) return false;
                if (k <= (uint32_t)E3) return true;
            }
            if constexpr (KMAX > 7) return probe_range<7, KMAX>(bm, mp, k, h, h1, h2);
            return true;
        }
    } else {
        // any k: 8 loads in flight per round, stop after the first round with a zero bit
        bool all = true;
        uint64_t h = h1;
        for (uint32_t j0 = 0; j0 < k && all; j0 += 8) {
            uint32_t word[8], mask[8];
#pragma unroll
            for (int t = 0; t < 8; ++t) {
                const uint32_t j = j0 + t;
                if (j < k) {
                    const uint32_t idx = mod63(h & 0x7fffffffffffffffULL, mp);
                    word[t] = bm[idx >> 5];
                    mask[t] = bit_in_word(idx);
                    h += (j & 1) ? h1 : h2;
                }
            }
#pragma unroll
            for (int t = 0; t < 8; ++t)
                if (j0 + t < k) all &= (word[t] & mask[t]) != 0u;
        }
        return all;
    }
}

template <int KLEN, int KMAX, int S1>
__global__ __launch_bounds__(256) void k_bloom_contains(KeysDev keys, const uint32_t *__restrict__ bm,
                                                        ModParams mp, uint32_t k,
                                                        uint8_t *__restrict__ out,
                                                        unsigned long long *__restrict__ count) {
    uint64_t present = 0;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < keys.n; i += stride) {
        uint64_t h1, h2;
        hash_key<KLEN>(keys, i, h1, h2);
        const bool p = probe_all_set<KMAX, S1>(bm, mp, k, h1, h2);
        if (out) out[i] = p;
        present += p;
    }
    if (count) block_add_u64(present, count);
}

// tile_seg0[t] = segment of key t*256 (one parallel binary search per 256-key tile)
__global__ __launch_bounds__(256) void k_tile_seg0(const uint64_t *__restrict__ seg_off, uint32_t nseg,
                                                   uint64_t ntiles, uint32_t *__restrict__ tile_seg0) {
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t < ntiles) tile_seg0[t] = upper_seg(seg_off, nseg, t * 256);
}


template <int KLEN, int KMAX, int S1>
__global__ __launch_bounds__(256) void k_bloom_contains_multi(KeysDev keys, const FilterDesc *__restrict__ filt,
                                                              const uint64_t *__restrict__ seg_off, uint32_t nseg,
                                                              const uint32_t *__restrict__ tile_seg0,
                                                              uint8_t *__restrict__ out,
                                                              unsigned long long *__restrict__ counts) {
    // No LDS staging and no block barrier: each lane finds its segment by a binary search of
    // seg_off between the segments of its own and the next 256-key tile (L2-resident; 0-1 steps
    // for C3-sized segments), so waves run independently and a lane's early-exit depth never
    // holds up the other waves of its block.
    const uint64_t nkeys = keys.n;
    const uint64_t ntiles = (nkeys + 255) >> 8;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    // grid-stride over whole waves: every lane of a wave takes the same trip count
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i - (threadIdx.x & 63) < nkeys; i += stride) {
        const bool active = i < nkeys;
        uint32_t seg = 0;
        bool p = false;
        if (active) {
            const uint64_t t = i >> 8;
            uint32_t lo = tile_seg0[t];                                   // seg_off[lo] <= i
            uint32_t hi = t + 1 < ntiles ? tile_seg0[t + 1] + 1 : nseg;  // i < seg_off[hi]
            while (hi - lo > 1) {
                const uint32_t mid = (lo + hi) >> 1;
                if (seg_off[mid] <= i) lo = mid;
                else hi = mid;
            }
            seg = lo;
            const FilterDesc f = filt[seg];
            uint64_t h1, h2;
            hash_key<KLEN>(keys, i, h1, h2);
            p = probe_all_set<KMAX, S1>(f.bm, f.mp, f.k, h1, h2);
            if (out) out[i] = p;
        }
        if (counts) wave_seg_add(active, seg, p, counts);
    }
}

// ---------------------------------------------------------------------------------
// contains with per-lane key slots (rbx_tune("contains_stage1", 5))
// ---------------------------------------------------------------------------------
// Each lane keeps P keys in flight and tests ONE bit per key per round trip, so a key costs
// exactly as many gathers as the bits read before its first 0 (~2 on a filter at fill 0.5,
// the minimum) while the lane still has P independent gathers outstanding.  A key that
// finishes frees its slot; free slots are refilled, in key order, from a per-wave queue that the
// whole wave fills convergently (hash, segment, first bit index of 64*Q consecutive keys, one
// coalesced pass) -- so the divergent part is only a 32-byte LDS read.  Two queue buffers per
// wave: while one is consumed the other holds the next range.  Results are identical to the
// staged kernels (same bits, same AND); only the number of gathers changes.
template <int KLEN, bool MULTI, int P, int Q>
__global__ __launch_bounds__(256) void k_bloom_contains_q(KeysDev keys, const FilterDesc *__restrict__ filt,
                                                          const uint64_t *__restrict__ seg_off, uint32_t nseg,
                                                          const uint32_t *__restrict__ tile_seg0, FilterDesc single,
                                                          uint8_t *__restrict__ out,
                                                          unsigned long long *__restrict__ counts) {
    constexpr uint32_t RANGE = 64 * Q, WAVES = 4;
    struct alignas(16) QEnt {
        uint64_t h1, h2;
        const uint32_t *bm;
        uint32_t seg, idx0;
    };
    __shared__ QEnt s_q[WAVES][2][RANGE];
    const uint32_t wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    QEnt *qb = &s_q[wave][0][0];
    const uint64_t nkeys = keys.n;
    const uint64_t nranges = (nkeys + RANGE - 1) / RANGE;
    const uint64_t ntiles = (nkeys + 255) >> 8;
    const uint64_t nw = (uint64_t)gridDim.x * WAVES;
    uint64_t rnext = (uint64_t)blockIdx.x * WAVES + wave;  // next range this wave hashes
    uint64_t qbase[2] = {0, 0};
    uint32_t qlen[2] = {0, 0};
    auto fill = [&](uint32_t b) {  // wave-uniform: hash range rnext into buffer b
        qlen[b] = 0;
        if (rnext >= nranges) return;
        const uint64_t rb = rnext * RANGE;
        qbase[b] = rb;
        qlen[b] = (uint32_t)min<uint64_t>(RANGE, nkeys - rb);
#pragma unroll
        for (uint32_t q = 0; q < Q; ++q) {
            const uint32_t pos = q * 64 + lane;
            const uint64_t i = rb + pos;
            if (i < nkeys) {
                QEnt e;
                hash_key<KLEN>(keys, i, e.h1, e.h2);
                e.seg = 0;
                ModParams mp = single.mp;
                e.bm = single.bm;
                if constexpr (MULTI) {
                    const uint64_t t = i >> 8;
                    uint32_t lo = tile_seg0[t];
                    uint32_t hi = t + 1 < ntiles ? tile_seg0[t + 1] + 1 : nseg;
                    while (hi - lo > 1) {
                        const uint32_t mid = (lo + hi) >> 1;
                        if (seg_off[mid] <= i) lo = mid;
                        else hi = mid;
                    }
                    e.seg = lo;
                    mp = filt[lo].mp;
                    e.bm = filt[lo].bm;
                }
                e.idx0 = mod63(e.h1 & 0x7fffffffffffffffULL, mp);
                qb[b * RANGE + pos] = e;
            }
        }
        rnext += nw;
        __builtin_amdgcn_wave_barrier();
    };
    bool act[P];
    uint64_t sh1[P], sh2[P], sh[P];
    uint32_t si[P], sjk[P], sseg[P], sidx[P];  // key index (< 2^32, host-checked), j | k << 16
    const uint32_t *sbm[P];
    ModC smp[P];
    const ModC single_mc = mod_compact(single.mp);
#pragma unroll
    for (int s = 0; s < P; ++s) act[s] = false;
    uint32_t cur = 0, qpos = 0;
    int stale = -1;  // a consumed buffer, refilled after the next gathers are issued
    fill(0);
    fill(1);
    uint64_t present = 0;
    for (;;) {
        // refill free slots in key order (lanes by rank)
#pragma unroll
        for (int s = 0; s < P; ++s) {
            bool need = !act[s];
            for (;;) {
                const uint64_t nm = __ballot(need);
                if (!nm) break;
                if (qpos >= qlen[cur]) {
                    if (stale == (int)(cur ^ 1)) {  // both buffers consumed in one refill: fill now
                        fill(cur ^ 1);
                        stale = -1;
                    }
                    if (qlen[cur ^ 1] == 0) break;  // queue exhausted
                    stale = (int)cur;
                    cur ^= 1;
                    qpos = 0;
                    continue;
                }
                const uint32_t avail = qlen[cur] - qpos;
                const uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(nm >> 32),
                                                                __builtin_amdgcn_mbcnt_lo((uint32_t)nm, 0u));
                if (need && rank < avail) {
                    const QEnt e = qb[cur * RANGE + qpos + rank];
                    act[s] = true;
                    need = false;
                    sh1[s] = e.h1;
                    sh2[s] = e.h2;
                    sh[s] = e.h1 + e.h2;  // hash 1 (h advances by h2 after j = 0)
                    si[s] = (uint32_t)(qbase[cur] + qpos + rank);
                    sidx[s] = e.idx0;
                    sbm[s] = e.bm;
                    sseg[s] = e.seg;
                    if constexpr (MULTI) {  // needed only after the first gather returns
                        smp[s] = mod_compact(filt[e.seg].mp);
                        sjk[s] = filt[e.seg].k << 16;
                    } else {
                        sjk[s] = single.k << 16;
                    }
                }
                qpos += min<uint32_t>((uint32_t)__popcll(nm), avail);
            }
        }
        bool any = false;
#pragma unroll
        for (int s = 0; s < P; ++s) any |= act[s];
        if (!__ballot(any)) break;  // every slot drained and the queue is empty
        uint32_t w[P];
#pragma unroll
        for (int s = 0; s < P; ++s)
            if (act[s]) w[s] = sbm[s][sidx[s] >> 5];
        if (stale >= 0) {  // hash the next range while this round's gathers are in flight
            fill((uint32_t)stale);
            stale = -1;
        }
#pragma unroll
        for (int s = 0; s < P; ++s) {
            bool fin_p = false;
            if (act[s]) {
                bool fin = false;
                if ((w[s] & bit_in_word(sidx[s])) == 0u) {
                    fin = true;
                } else if (((++sjk[s]) & 0xffffu) >= (sjk[s] >> 16)) {
                    fin = fin_p = true;
                } else {
                    sidx[s] = mod63c(sh[s] & 0x7fffffffffffffffULL, MULTI ? smp[s] : single_mc);
                    sh[s] += (sjk[s] & 1) ? sh1[s] : sh2[s];
                }
                if (fin) {
                    act[s] = false;
                    if (out) out[si[s]] = fin_p;
                }
            }
            if constexpr (MULTI) {
                if (counts && __ballot(fin_p)) wave_seg_add(fin_p, sseg[s], 1u, counts);
            } else {
                present += fin_p;
            }
        }
    }
    if constexpr (!MULTI) {
        if (counts) block_add_u64(present, counts);
    }
}

// Probe: gathers the k bits, records which are zero (zmask, bit j <-> hash j) and
// registers each zero bit in the first-setter table.  Tracks the Redis string length
// (every SETBIT grows it to idx/8+1, whatever the old bit).
template <int KLEN, int KMAX>
__global__ __launch_bounds__(256) void k_bloom_add_probe(KeysDev keys, uint64_t base, uint64_t nchunk,
                                                         const FilterDesc *__restrict__ filt,
                                                         const uint64_t *__restrict__ seg_off, uint32_t nseg,
                                                         const uint32_t *__restrict__ tile_seg0,
                                                         FilterDesc single, HTEntry *__restrict__ T,
                                                         uint32_t log2cap, uint32_t epoch,
                                                         uint32_t *__restrict__ zmask) {
    static_assert(KMAX > 0 && KMAX <= 32, "probe mask holds 32 hashes");
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; t < nchunk; t += stride) {
        const uint64_t i = base + t;
        FilterDesc f = single;
        if (filt) f = filt[seg_from(seg_off, nseg, tile_seg0[i >> 8], i)];
        uint64_t h1, h2;
        hash_key<KLEN>(keys, i, h1, h2);
        uint32_t word[KMAX], idxs[KMAX];
        uint32_t maxidx = 0;
        uint64_t h = h1;
#pragma unroll
        for (int j = 0; j < KMAX; ++j) {
            if ((uint32_t)j < f.k) {
                const uint32_t idx = mod63(h & 0x7fffffffffffffffULL, f.mp);
                idxs[j] = idx;
                word[j] = f.bm[idx >> 5];
                maxidx = idx > maxidx ? idx : maxidx;
            }
            h += (j & 1) ? h1 : h2;
        }
        uint32_t zm = 0;
#pragma unroll
        for (int j = 0; j < KMAX; ++j) {
            if ((uint32_t)j < f.k && (word[j] & bit_in_word(idxs[j])) == 0u) {
                zm |= 1u << j;
                ht_insert(T, log2cap, epoch, ((uint64_t)f.fid << 32) | idxs[j], (uint32_t)t);
            }
        }
        zmask[t] = zm;
        raise_redis_len(f.redis_len, (unsigned long long)(maxidx >> 3) + 1ULL);
    }
}

template <int KLEN, int KMAX>
__global__ __launch_bounds__(256) void k_bloom_add_commit(KeysDev keys, uint64_t base, uint64_t nchunk,
                                                          const FilterDesc *__restrict__ filt,
                                                          const uint64_t *__restrict__ seg_off, uint32_t nseg,
                                                          const uint32_t *__restrict__ tile_seg0,
                                                          FilterDesc single, const HTEntry *__restrict__ T,
                                                          uint32_t log2cap, uint32_t epoch,
                                                          const uint32_t *__restrict__ zmask,
                                                          uint8_t *__restrict__ out_new,
                                                          unsigned long long *__restrict__ count,
                                                          unsigned long long *__restrict__ seg_counts) {
    uint64_t added = 0;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; t < nchunk; t += stride) {
        const uint64_t i = base + t;
        const uint32_t zm = zmask[t];
        bool isnew = false;
        if (zm) {
            uint32_t seg = 0;
            FilterDesc f = single;
            if (filt) {
                seg = seg_from(seg_off, nseg, tile_seg0[i >> 8], i);
                f = filt[seg];
            }
            uint64_t h1, h2;
            hash_key<KLEN>(keys, i, h1, h2);
            uint64_t h = h1;
#pragma unroll
            for (int j = 0; j < KMAX; ++j) {
                if ((zm >> j) & 1u) {
                    const uint32_t idx = mod63(h & 0x7fffffffffffffffULL, f.mp);
                    if (ht_owner(T, log2cap, epoch, ((uint64_t)f.fid << 32) | idx) == (uint32_t)t) {
                        isnew = true;
                        atomicOr(&f.bm[idx >> 5], bit_in_word(idx));
                    }
                }
                h += (j & 1) ? h1 : h2;
            }
            if (isnew && seg_counts) atomicAdd(&seg_counts[seg], 1ULL);
        }
        if (out_new) out_new[i] = isnew;
        added += isnew;
    }
    if (count) block_add_u64(added, count);
}

// ---- single-filter fast path: 8-byte entries (bit << 32 | key id), empty = ~0 ------------
// The table is cleared (memset 0xff) before every chunk, so a claim is one CAS on an empty
// slot; a slot already holding the same bit takes the 64-bit atomicMin (same high word, so
// the minimum is the smallest key id); a lookup is one 8-byte load per probe.
__device__ __forceinline__ void ht8_insert(unsigned long long *__restrict__ T, uint32_t log2cap, uint32_t idx,
                                           uint32_t id) {
    const uint64_t mask = (1ULL << log2cap) - 1;
    const unsigned long long mine = ((unsigned long long)idx << 32) | id;
    uint64_t slot = ht_slot(idx, log2cap);
    for (uint64_t probes = 0; probes <= mask; ++probes) {
        const unsigned long long old = atomicCAS(&T[slot], ~0ULL, mine);
        if (old == ~0ULL) return;
        if ((uint32_t)(old >> 32) == idx) {
            if ((uint32_t)old > id) atomicMin(&T[slot], mine);
            return;
        }
        slot = (slot + 1) & mask;
    }
}

__device__ __forceinline__ uint32_t ht8_owner(const unsigned long long *__restrict__ T, uint32_t log2cap,
                                              uint32_t idx) {
    const uint64_t mask = (1ULL << log2cap) - 1;
    uint64_t slot = ht_slot(idx, log2cap);
    for (uint64_t probes = 0; probes <= mask; ++probes) {
        const unsigned long long e = T[slot];
        if ((uint32_t)(e >> 32) == idx) return (uint32_t)e;
        slot = (slot + 1) & mask;
    }
    return 0xffffffffu;
}

template <int KLEN, int KMAX>
__global__ __launch_bounds__(256) void k_bloom_add_probe8(KeysDev keys, uint64_t base, uint64_t nchunk,
                                                          FilterDesc f, unsigned long long *__restrict__ T,
                                                          uint32_t log2cap, uint32_t *__restrict__ zmask) {
    uint32_t maxidx = 0;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; t < nchunk; t += stride) {
        uint64_t h1, h2;
        hash_key<KLEN>(keys, base + t, h1, h2);
        uint32_t word[KMAX], idxs[KMAX];
        uint64_t h = h1;
#pragma unroll
        for (int j = 0; j < KMAX; ++j) {
            if ((uint32_t)j < f.k) {
                const uint32_t idx = mod63(h & 0x7fffffffffffffffULL, f.mp);
                idxs[j] = idx;
                word[j] = f.bm[idx >> 5];
                maxidx = idx > maxidx ? idx : maxidx;
            }
            h += (j & 1) ? h1 : h2;
        }
        uint32_t zm = 0;
#pragma unroll
        for (int j = 0; j < KMAX; ++j) {
            if ((uint32_t)j < f.k && (word[j] & bit_in_word(idxs[j])) == 0u) {
                zm |= 1u << j;
                ht8_insert(T, log2cap, idxs[j], (uint32_t)t);
            }
        }
        zmask[t] = zm;
    }
    // Redis string length: one atomic per wave (every SETBIT grows it to idx/8 + 1)
    const uint64_t wmax = wave_max_u64(maxidx);
    if ((threadIdx.x & 63) == 0 && nchunk) raise_redis_len(f.redis_len, (unsigned long long)(wmax >> 3) + 1ULL);
}

template <int KLEN, int KMAX>
__global__ __launch_bounds__(256) void k_bloom_add_commit8(KeysDev keys, uint64_t base, uint64_t nchunk,
                                                           FilterDesc f, const unsigned long long *__restrict__ T,
                                                           uint32_t log2cap, const uint32_t *__restrict__ zmask,
                                                           uint8_t *__restrict__ out_new,
                                                           unsigned long long *__restrict__ count) {
    uint64_t added = 0;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; t < nchunk; t += stride) {
        const uint32_t zm = zmask[t];
        bool isnew = false;
        if (zm) {
            uint64_t h1, h2;
            hash_key<KLEN>(keys, base + t, h1, h2);
            uint64_t h = h1;
#pragma unroll
            for (int j = 0; j < KMAX; ++j) {
                if ((zm >> j) & 1u) {
                    const uint32_t idx = mod63(h & 0x7fffffffffffffffULL, f.mp);
                    if (ht8_owner(T, log2cap, idx) == (uint32_t)t) {
                        isnew = true;
                        atomicOr(&f.bm[idx >> 5], bit_in_word(idx));
                    }
                }
                h += (j & 1) ? h1 : h2;
            }
        }
        if (out_new) out_new[base + t] = isnew;
        added += isnew;
    }
    if (count) block_add_u64(added, count);
}

// Generic-k add (k > 32): per-pair zero flags in a byte array zflag[t*k + j].
template <int KLEN>
__global__ __launch_bounds__(256) void k_bloom_add_probe_anyk(KeysDev keys, uint64_t base, uint64_t nchunk,
                                                              const FilterDesc *__restrict__ filt,
                                                              const uint64_t *__restrict__ seg_off, uint32_t nseg,
                                                              const uint32_t *__restrict__ tile_seg0,
                                                              FilterDesc single, HTEntry *__restrict__ T,
                                                              uint32_t log2cap, uint32_t epoch,
                                                              uint8_t *__restrict__ zflag, uint32_t kstride) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; t < nchunk; t += stride) {
        const uint64_t i = base + t;
        FilterDesc f = single;
        if (filt) f = filt[seg_from(seg_off, nseg, tile_seg0[i >> 8], i)];
        uint64_t h1, h2;
        hash_key<KLEN>(keys, i, h1, h2);
        uint64_t h = h1;
        uint32_t maxidx = 0;
        for (uint32_t j = 0; j < f.k; ++j) {
            const uint32_t idx = mod63(h & 0x7fffffffffffffffULL, f.mp);
            maxidx = idx > maxidx ? idx : maxidx;
            const bool z = (f.bm[idx >> 5] & bit_in_word(idx)) == 0u;
            zflag[t * kstride + j] = z;
            if (z) ht_insert(T, log2cap, epoch, ((uint64_t)f.fid << 32) | idx, (uint32_t)t);
            h += (j & 1) ? h1 : h2;
        }
        raise_redis_len(f.redis_len, (unsigned long long)(maxidx >> 3) + 1ULL);
    }
}

template <int KLEN>
__global__ __launch_bounds__(256) void k_bloom_add_commit_anyk(KeysDev keys, uint64_t base, uint64_t nchunk,
                                                               const FilterDesc *__restrict__ filt,
                                                               const uint64_t *__restrict__ seg_off, uint32_t nseg,
                                                               const uint32_t *__restrict__ tile_seg0,
                                                               FilterDesc single, const HTEntry *__restrict__ T,
                                                               uint32_t log2cap, uint32_t epoch,
                                                               const uint8_t *__restrict__ zflag, uint32_t kstride,
                                                               uint8_t *__restrict__ out_new,
                                                               unsigned long long *__restrict__ count,
                                                               unsigned long long *__restrict__ seg_counts) {
    uint64_t added = 0;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; t < nchunk; t += stride) {
        const uint64_t i = base + t;
        uint32_t seg = 0;
        FilterDesc f = single;
        if (filt) {
            seg = seg_from(seg_off, nseg, tile_seg0[i >> 8], i);
            f = filt[seg];
        }
        uint64_t h1, h2;
        hash_key<KLEN>(keys, i, h1, h2);
        uint64_t h = h1;
        bool isnew = false;
        for (uint32_t j = 0; j < f.k; ++j) {
            if (zflag[t * kstride + j]) {
                const uint32_t idx = mod63(h & 0x7fffffffffffffffULL, f.mp);
                if (ht_owner(T, log2cap, epoch, ((uint64_t)f.fid << 32) | idx) == (uint32_t)t) {
                    isnew = true;
                    atomicOr(&f.bm[idx >> 5], bit_in_word(idx));
                }
            }
            h += (j & 1) ? h1 : h2;
        }
        if (isnew && seg_counts) atomicAdd(&seg_counts[seg], 1ULL);
        if (out_new) out_new[i] = isnew;
        added += isnew;
    }
    if (count) block_add_u64(added, count);
}

// ---------------------------------------------------------------------------------
// BITCOUNT over nbytes of the bitmap string (RedissonBitSet.cardinalityAsync :482-484)
// ---------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_bitcount(const uint8_t *__restrict__ bytes, uint64_t nbytes,
                                                  unsigned long long *__restrict__ out) {
    uint64_t c = 0;
    const uint64_t nvec = nbytes >> 4;
    const uint4 *v = (const uint4 *)bytes;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    const uint64_t tid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    for (uint64_t i = tid; i < nvec; i += stride) {
        const uint4 x = ld_nt16(v + i);
        c += __popc(x.x) + __popc(x.y) + __popc(x.z) + __popc(x.w);
    }
    for (uint64_t i = (nvec << 4) + tid; i < nbytes; i += stride) c += __popc((uint32_t)bytes[i]);
    block_add_u64(c, out);
}

// Order-independent 64-bit digest of the Redis string's bytes: sum over 16-byte vectors v of
// mix(v, position).  Replicas compare digests (one word per GPU over the collective) instead of
// whole bitmaps.  The tail bytes past nbytes of the last vector are zero (bitmap invariant).
__device__ __forceinline__ uint64_t mix64(uint64_t x) {
    x ^= x >> 31;
    x *= 0x7fb5d329728ea185ULL;
    x ^= x >> 27;
    x *= 0x81dadef4bc2dd44dULL;
    x ^= x >> 33;
    return x;
}

__global__ __launch_bounds__(256) void k_digest(const uint8_t *__restrict__ bytes, uint64_t nbytes,
                                                unsigned long long *__restrict__ out) {
    uint64_t d = 0;
    const uint64_t nvec = (nbytes + 15) >> 4;
    const uint4 *v = (const uint4 *)bytes;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nvec; i += stride) {
        const uint4 x = ld_nt16(v + i);
        const uint64_t lo = ((uint64_t)x.y << 32) | x.x, hi = ((uint64_t)x.w << 32) | x.z;
        d += mix64(lo ^ mix64(2 * i + 0x9E3779B97F4A7C15ULL)) + mix64(hi ^ mix64(2 * i + 1));
    }
    block_add_u64(d, out);
}

// ---------------------------------------------------------------------------------
// launchers
// ---------------------------------------------------------------------------------

// Early-exit width for contains (rbx_tune("contains_stage1", n)); 0 disables.
static std::atomic<int> g_stage1{4};
void set_contains_stage1(int v) { g_stage1 = v; }
int get_contains_stage1() { return g_stage1; }

template <int KLEN, int KMAX, int S1>
static void launch_contains_s(const KeysDev &keys, const uint32_t *bm, const ModParams &mp, uint32_t k,
                              uint8_t *out, unsigned long long *count, hipStream_t st, unsigned grid) {
    hipLaunchKernelGGL((k_bloom_contains<KLEN, KMAX, S1>), dim3(grid), dim3(256), 0, st, keys, bm, mp, k, out, count);
}

// slot kernel grid (grid-stride over 64*Q-key ranges), rbx_tune "contains_qgrid".  Its shape is P = 2
// slots and Q = 2 queued keys per lane (r02-r05 also compiled 24/32/34/42/44 for A/Bs: none faster,
// removed in r06; profiles/r03/r03u_c5sweep_qshape_qgrid.jsonl).
static std::atomic<unsigned> g_qgrid{2048};
void set_contains_qgrid(int v) { g_qgrid = (unsigned)v; }

template <int KLEN, bool MULTI>
static void launch_contains_q(const KeysDev &keys, const FilterDesc *filt, const uint64_t *seg_off, uint32_t nseg,
                              const uint32_t *tile_seg0, const FilterDesc &single, uint8_t *out,
                              unsigned long long *counts, hipStream_t st, unsigned grid) {
    hipLaunchKernelGGL((k_bloom_contains_q<KLEN, MULTI, 2, 2>), dim3(std::min(grid, g_qgrid.load())), dim3(256), 0, st,
                       keys, filt, seg_off, nseg, tile_seg0, single, out, counts);
}

template <int KLEN, int KMAX>
static void launch_contains_km(const KeysDev &keys, const uint32_t *bm, const ModParams &mp, uint32_t k,
                               uint8_t *out, unsigned long long *count, hipStream_t st, unsigned grid) {
    const int stage1 = g_stage1.load();  // read once per call
    if (stage1 == 5 && keys.n < (1ULL << 32)) {  // slot kernel: u32 key indexes
        FilterDesc f{};
        f.bm = const_cast<uint32_t *>(bm);
        f.mp = mp;
        f.k = k;
        launch_contains_q<KLEN, false>(keys, nullptr, nullptr, 0u, nullptr, f, out, count, st, grid);
        return;
    }
    switch (stage1) {
    case 0: launch_contains_s<KLEN, KMAX, 0>(keys, bm, mp, k, out, count, st, grid); break;
    case 2: launch_contains_s<KLEN, KMAX, 2>(keys, bm, mp, k, out, count, st, grid); break;
    case 3: launch_contains_s<KLEN, KMAX, 3>(keys, bm, mp, k, out, count, st, grid); break;
    case 4: launch_contains_s<KLEN, KMAX, 4>(keys, bm, mp, k, out, count, st, grid); break;
    default: launch_contains_s<KLEN, KMAX, 1>(keys, bm, mp, k, out, count, st, grid); break;
    }
}

template <int KLEN>
static void launch_contains_k(const KeysDev &keys, const uint32_t *bm, const ModParams &mp, uint32_t k,
                              uint8_t *out, unsigned long long *count, hipStream_t st, unsigned grid) {
    if (k <= 8) launch_contains_km<KLEN, 8>(keys, bm, mp, k, out, count, st, grid);
    else if (k <= 16) launch_contains_km<KLEN, 16>(keys, bm, mp, k, out, count, st, grid);
    else launch_contains_s<KLEN, 0, 0>(keys, bm, mp, k, out, count, st, grid);
}

void launch_bloom_contains(const KeysDev &keys, int klen_fast, const uint32_t *bm, const ModParams &mp,
                           uint32_t k, uint8_t *out, unsigned long long *count, hipStream_t st) {
    const unsigned grid = grid_for(keys.n, kMaxGrid);
    switch (klen_fast) {
    case 16: launch_contains_k<16>(keys, bm, mp, k, out, count, st, grid); break;
    case 32: launch_contains_k<32>(keys, bm, mp, k, out, count, st, grid); break;
    case 64: launch_contains_k<64>(keys, bm, mp, k, out, count, st, grid); break;
    default: launch_contains_k<0>(keys, bm, mp, k, out, count, st, grid); break;
    }
}

template <int KLEN>
static void launch_contains_multi_k(const KeysDev &keys, const FilterDesc *filt, const uint64_t *seg_off,
                                    uint32_t nseg, const uint32_t *tile_seg0, uint32_t kmax, uint8_t *out,
                                    unsigned long long *counts, hipStream_t st, unsigned grid, bool slots) {
    const int stage1 = g_stage1.load();  // read once per call
    const bool dbl = stage1 == 4;
    if ((slots || stage1 == 5) && keys.n < (1ULL << 32)) {  // slot kernel: u32 key indexes
        launch_contains_q<KLEN, true>(keys, filt, seg_off, nseg, tile_seg0, FilterDesc{}, out, counts, st, grid);
        return;
    }
    if (kmax <= 8) {
        if (dbl) hipLaunchKernelGGL((k_bloom_contains_multi<KLEN, 8, 4>), dim3(grid), dim3(256), 0, st, keys, filt, seg_off, nseg, tile_seg0, out, counts);
        else hipLaunchKernelGGL((k_bloom_contains_multi<KLEN, 8, 1>), dim3(grid), dim3(256), 0, st, keys, filt, seg_off, nseg, tile_seg0, out, counts);
    } else if (kmax <= 16) {
        if (dbl) hipLaunchKernelGGL((k_bloom_contains_multi<KLEN, 16, 4>), dim3(grid), dim3(256), 0, st, keys, filt, seg_off, nseg, tile_seg0, out, counts);
        else hipLaunchKernelGGL((k_bloom_contains_multi<KLEN, 16, 1>), dim3(grid), dim3(256), 0, st, keys, filt, seg_off, nseg, tile_seg0, out, counts);
    }
    else hipLaunchKernelGGL((k_bloom_contains_multi<KLEN, 0, 0>), dim3(grid), dim3(256), 0, st, keys, filt, seg_off, nseg, tile_seg0, out, counts);
}

void launch_tile_seg0(const uint64_t *seg_off, uint32_t nseg, uint64_t nkeys, uint32_t *tile_seg0,
                      hipStream_t st) {
    const uint64_t ntiles = (nkeys + 255) / 256;
    if (!ntiles) return;
    hipLaunchKernelGGL(k_tile_seg0, dim3((unsigned)((ntiles + 255) / 256)), dim3(256), 0, st, seg_off, nseg, ntiles,
                       tile_seg0);
}

void launch_bloom_contains_multi(const KeysDev &keys, int klen_fast, const FilterDesc *filt,
                                 const uint64_t *seg_off, uint32_t nseg, const uint32_t *tile_seg0, uint32_t kmax,
                                 uint8_t *out, unsigned long long *counts, hipStream_t st, bool slots) {
    const unsigned grid = grid_for(keys.n, kMaxGrid);
    switch (klen_fast) {
    case 16: launch_contains_multi_k<16>(keys, filt, seg_off, nseg, tile_seg0, kmax, out, counts, st, grid, slots); break;
    case 32: launch_contains_multi_k<32>(keys, filt, seg_off, nseg, tile_seg0, kmax, out, counts, st, grid, slots); break;
    case 64: launch_contains_multi_k<64>(keys, filt, seg_off, nseg, tile_seg0, kmax, out, counts, st, grid, slots); break;
    default: launch_contains_multi_k<0>(keys, filt, seg_off, nseg, tile_seg0, kmax, out, counts, st, grid, slots); break;
    }
}

template <int KLEN, int KMAX>
static void launch_add_chunk_k(const AddChunkArgs &a, hipStream_t st) {
    const unsigned grid = grid_for(a.nchunk, kMaxGrid);
    if (a.narrow) {
        auto *T = (unsigned long long *)a.table;
        hipLaunchKernelGGL((k_bloom_add_probe8<KLEN, KMAX>), dim3(grid), dim3(256), 0, st, a.keys, a.base, a.nchunk,
                           a.single, T, a.log2cap, a.zmask);
        hipLaunchKernelGGL((k_bloom_add_commit8<KLEN, KMAX>), dim3(grid), dim3(256), 0, st, a.keys, a.base, a.nchunk,
                           a.single, (const unsigned long long *)T, a.log2cap, a.zmask, a.out_new, a.count);
        return;
    }
    hipLaunchKernelGGL((k_bloom_add_probe<KLEN, KMAX>), dim3(grid), dim3(256), 0, st, a.keys, a.base, a.nchunk,
                       a.filt, a.seg_off, a.nseg, a.tile_seg0, a.single, a.table, a.log2cap, a.epoch, a.zmask);
    hipLaunchKernelGGL((k_bloom_add_commit<KLEN, KMAX>), dim3(grid), dim3(256), 0, st, a.keys, a.base, a.nchunk,
                       a.filt, a.seg_off, a.nseg, a.tile_seg0, a.single, a.table, a.log2cap, a.epoch, a.zmask, a.out_new,
                       a.count, a.seg_counts);
}

template <int KLEN>
static void launch_add_chunk_len(const AddChunkArgs &a, hipStream_t st) {
    if (a.kmax <= 8) launch_add_chunk_k<KLEN, 8>(a, st);
    else if (a.kmax <= 16) launch_add_chunk_k<KLEN, 16>(a, st);
    else if (a.kmax <= 32) launch_add_chunk_k<KLEN, 32>(a, st);
    else {
        const unsigned grid = grid_for(a.nchunk, kMaxGrid);
        hipLaunchKernelGGL((k_bloom_add_probe_anyk<KLEN>), dim3(grid), dim3(256), 0, st, a.keys, a.base, a.nchunk,
                           a.filt, a.seg_off, a.nseg, a.tile_seg0, a.single, a.table, a.log2cap, a.epoch,
                           (uint8_t *)a.zmask, a.kmax);
        hipLaunchKernelGGL((k_bloom_add_commit_anyk<KLEN>), dim3(grid), dim3(256), 0, st, a.keys, a.base,
                           a.nchunk, a.filt, a.seg_off, a.nseg, a.tile_seg0, a.single, a.table, a.log2cap, a.epoch,
                           (const uint8_t *)a.zmask, a.kmax, a.out_new, a.count, a.seg_counts);
    }
}

void launch_bloom_add_chunk(const AddChunkArgs &a, int klen_fast, hipStream_t st) {
    switch (klen_fast) {
    case 16: launch_add_chunk_len<16>(a, st); break;
    case 32: launch_add_chunk_len<32>(a, st); break;
    case 64: launch_add_chunk_len<64>(a, st); break;
    default: launch_add_chunk_len<0>(a, st); break;
    }
}

// add(T) (M/RedissonBloomFilter.java:99-102): SETBIT of the key's k bits, new iff one of them was 0.  One
// key has no earlier key of its batch to lose a bit to, so it needs no first-setter table: one lane reads
// the Redis length and the k words, ORs every zero bit in (non-returning atomics), writes the reply and
// raises the length.  The context's call order keeps every other writer of the bitmap out meanwhile.
// (A 1-key call through the one-segment kernel spends ~10 us on the GPU, through this one ~5 us.)
// `done` (nullable, coherent host memory): the lane's last store is seq there, after every other access of
// the call (a system-scope release), so the host can spin on it instead of waiting for the stream (§3.10)
template <int KLEN, int KMAX>
__global__ __launch_bounds__(64) void k_bloom_add_one(KeysDev keys, FilterDesc f, uint8_t *__restrict__ out,
                                                      unsigned long long *__restrict__ count, uint32_t *done,
                                                      uint32_t seq) {
    if (threadIdx.x != 0) return;
    const unsigned long long len0 = __hip_atomic_load(f.redis_len, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    uint64_t h1, h2;
    hash_key<KLEN>(keys, 0, h1, h2);
    uint32_t idxs[KMAX], word[KMAX], maxidx = 0;
    uint64_t h = h1;
#pragma unroll
    for (int j = 0; j < KMAX; ++j) {
        if ((uint32_t)j < f.k) {
            const uint32_t idx = mod63(h & 0x7fffffffffffffffULL, f.mp);
            idxs[j] = idx;
            word[j] = f.bm[idx >> 5];
            maxidx = idx > maxidx ? idx : maxidx;
        }
        h += (j & 1) ? h1 : h2;
    }
    bool isnew = false;
#pragma unroll
    for (int j = 0; j < KMAX; ++j) {
        if ((uint32_t)j < f.k && (word[j] & bit_in_word(idxs[j])) == 0u) {
            isnew = true;
            atomicOr(&f.bm[idxs[j] >> 5], bit_in_word(idxs[j]));
        }
    }
    if (out) out[0] = isnew;
    if (count && isnew) atomicAdd(count, 1ULL);
    const unsigned long long len = (unsigned long long)(maxidx >> 3) + 1ULL;  // every SETBIT grows the string
    if (len > len0) atomicMax(f.redis_len, len);
    if (done) __hip_atomic_store(done, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// contains(T): one key, one lane, every word gathered at once; `done` as in k_bloom_add_one
template <int KLEN, int KMAX>
__global__ __launch_bounds__(64) void k_bloom_contains_one(KeysDev keys, const uint32_t *__restrict__ bm, ModParams mp,
                                                           uint32_t k, uint8_t *__restrict__ out, uint32_t *done,
                                                           uint32_t seq) {
    if (threadIdx.x != 0) return;
    uint64_t h1, h2;
    hash_key<KLEN>(keys, 0, h1, h2);
    uint32_t idxs[KMAX], word[KMAX];
    uint64_t h = h1;
#pragma unroll
    for (int j = 0; j < KMAX; ++j) {
        if ((uint32_t)j < k) {
            idxs[j] = mod63(h & 0x7fffffffffffffffULL, mp);
            word[j] = bm[idxs[j] >> 5];
        }
        h += (j & 1) ? h1 : h2;
    }
    bool all = true;
#pragma unroll
    for (int j = 0; j < KMAX; ++j)
        if ((uint32_t)j < k) all &= (word[j] & bit_in_word(idxs[j])) != 0u;
    if (out) out[0] = all;
    if (done) __hip_atomic_store(done, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

template <int KLEN>
static void launch_one_len(bool add, const KeysDev &keys, const FilterDesc &f, uint8_t *out, unsigned long long *count,
                           uint32_t *done, uint32_t seq, hipStream_t st) {
    if (add && f.k <= 8)
        hipLaunchKernelGGL((k_bloom_add_one<KLEN, 8>), dim3(1), dim3(64), 0, st, keys, f, out, count, done, seq);
    else if (add)
        hipLaunchKernelGGL((k_bloom_add_one<KLEN, 16>), dim3(1), dim3(64), 0, st, keys, f, out, count, done, seq);
    else if (f.k <= 8)
        hipLaunchKernelGGL((k_bloom_contains_one<KLEN, 8>), dim3(1), dim3(64), 0, st, keys, f.bm, f.mp, f.k, out, done, seq);
    else
        hipLaunchKernelGGL((k_bloom_contains_one<KLEN, 16>), dim3(1), dim3(64), 0, st, keys, f.bm, f.mp, f.k, out, done, seq);
}

void launch_bloom_one(bool add, const KeysDev &keys, int klen_fast, const FilterDesc &f, uint8_t *out,
                      unsigned long long *count, uint32_t *done, uint32_t seq, hipStream_t st) {
    switch (klen_fast) {
    case 16: launch_one_len<16>(add, keys, f, out, count, done, seq, st); break;
    case 32: launch_one_len<32>(add, keys, f, out, count, done, seq, st); break;
    case 64: launch_one_len<64>(add, keys, f, out, count, done, seq, st); break;
    default: launch_one_len<0>(add, keys, f, out, count, done, seq, st); break;
    }
}

// the completion word of a tiny host call whose work is several kernels or workgroups: stream order puts it
// after all of them (bloom_host_tiny; 9.6 vs 11.5 us for a stream sync, tools/syncbench.hip)
__global__ void k_done_word(uint32_t *done, uint32_t seq) {
    if (threadIdx.x == 0) __hip_atomic_store(done, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

void launch_done_word(uint32_t *done, uint32_t seq, hipStream_t st) {
    hipLaunchKernelGGL(k_done_word, dim3(1), dim3(64), 0, st, done, seq);
}

void launch_bitcount(const uint8_t *bytes, uint64_t nbytes, unsigned long long *out, hipStream_t st) {
    const unsigned grid = grid_for((nbytes + 15) / 16, kMaxGrid);
    hipLaunchKernelGGL(k_bitcount, dim3(grid), dim3(256), 0, st, bytes, nbytes, out);
}

void launch_digest(const uint8_t *bytes, uint64_t nbytes, unsigned long long *out, hipStream_t st) {
    const unsigned grid = grid_for((nbytes + 15) / 16, 4096);
    hipLaunchKernelGGL(k_digest, dim3(grid), dim3(256), 0, st, bytes, nbytes, out);
}

}  // namespace rbx

// ---------------------------------------------------------------------------------
// Random-gather roofline probe: the contains kernel's memory pattern with the hashing
// removed.  Each lane issues k independent 4-byte loads at pseudo-random word offsets
// of a `nwords`-word table (same MLP structure as k_bloom_contains), XOR-reduced to a
// sink so nothing is dead-code eliminated.
// ---------------------------------------------------------------------------------
namespace rbx {
template <int K>
__global__ __launch_bounds__(256) void k_gather_probe(const uint32_t *__restrict__ tbl, uint64_t nwords,
                                                      uint64_t nkeys, uint64_t seed, uint32_t *__restrict__ sink) {
    uint32_t acc = 0;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nkeys; i += stride) {
        uint64_t z = (seed + i) * 0x9E3779B97F4A7C15ULL;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
        z ^= z >> 27;
        uint32_t w[K];
#pragma unroll
        for (int j = 0; j < K; ++j) {
            const uint32_t r = (uint32_t)(z >> (j & 1 ? 32 : 0)) ^ (uint32_t)(j * 0x9E3779B9u);
            z += 0x632BE59BD9B4E019ULL;
            w[j] = tbl[(uint64_t)r * nwords >> 32];
        }
#pragma unroll
        for (int j = 0; j < K; ++j) acc ^= w[j];
    }
    if (acc == 0x9E3779B9u) sink[0] = acc;  // practically never taken; keeps the loads live
}

void launch_gather_probe(const uint32_t *tbl, uint64_t nwords, uint64_t nkeys, uint32_t k, uint32_t *sink,
                         hipStream_t st) {
    const unsigned grid = grid_for(nkeys, kMaxGrid);
    switch (k) {
    case 10: hipLaunchKernelGGL(k_gather_probe<10>, dim3(grid), dim3(256), 0, st, tbl, nwords, nkeys, 0x5EEDull, sink); break;
    default: hipLaunchKernelGGL(k_gather_probe<7>, dim3(grid), dim3(256), 0, st, tbl, nwords, nkeys, 0x5EEDull, sink); break;
    }
}
}  // namespace rbx

// ---------------------------------------------------------------------------------
// Region-local gather probe: the table is cut into regions of `region_words`; workgroup b
// works on regions b%8, b%8+8, ... in order (blocks b and b+8 share an XCD under the
// observed round-robin placement -- speed only), each lane doing k random loads inside the
// current region.  Measures the L2-resident gather rate a region-bucketed probe can reach.
// ---------------------------------------------------------------------------------
namespace rbx {
__global__ __launch_bounds__(256) void k_gather_regions(const uint32_t *__restrict__ tbl, uint64_t nregions,
                                                        uint64_t region_words, uint64_t per_region,
                                                        uint32_t *__restrict__ sink) {
    const uint32_t xcd = blockIdx.x & 7, local = blockIdx.x >> 3, nlocal = gridDim.x >> 3;
    uint32_t acc = 0;
    for (uint64_t r = xcd; r < nregions; r += 8) {
        const uint32_t *base = tbl + r * region_words;
        for (uint64_t i = (uint64_t)local * blockDim.x + threadIdx.x; i < per_region; i += (uint64_t)nlocal * blockDim.x) {
            uint64_t z = (r * 0x9E3779B97F4A7C15ULL) ^ (i * 0xBF58476D1CE4E5B9ULL);
            z ^= z >> 31;
            z *= 0x94D049BB133111EBULL;
            uint32_t w[6];
#pragma unroll
            for (int j = 0; j < 6; ++j) {
                w[j] = base[(uint64_t)(uint32_t)(z >> (j & 1 ? 32 : 0) ^ (j * 0x9E3779B9u)) * region_words >> 32];
                z += 0x632BE59BD9B4E019ULL;
            }
#pragma unroll
            for (int j = 0; j < 6; ++j) acc ^= w[j];
        }
    }
    if (acc == 0x9E3779B9u) sink[0] = acc;
}

// Segment-local gather probe (the locality of a multi-tenant batch, BASELINE C3): key i belongs
// to segment i / keys_per_seg, segments are consecutive slices of seg_words words (wrapping over
// the table), and every key does K random 4-byte loads inside its own segment.
template <int K>
__global__ __launch_bounds__(256) void k_gather_segments(const uint32_t *__restrict__ tbl, uint64_t nwords,
                                                         uint64_t seg_words, uint64_t keys_per_seg, uint64_t nkeys,
                                                         uint32_t *__restrict__ sink) {
    uint32_t acc = 0;
    const uint64_t nseg_tbl = nwords / seg_words;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nkeys; i += stride) {
        const uint32_t *base = tbl + ((i / keys_per_seg) % nseg_tbl) * seg_words;
        uint64_t z = (i + 0x5EEDull) * 0x9E3779B97F4A7C15ULL;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
        z ^= z >> 27;
        uint32_t w[K];
#pragma unroll
        for (int j = 0; j < K; ++j) {
            const uint32_t r = (uint32_t)(z >> (j & 1 ? 32 : 0)) ^ (uint32_t)(j * 0x9E3779B9u);
            z += 0x632BE59BD9B4E019ULL;
            w[j] = base[(uint64_t)r * seg_words >> 32];
        }
#pragma unroll
        for (int j = 0; j < K; ++j) acc ^= w[j];
    }
    if (acc == 0x9E3779B9u) sink[0] = acc;
}

void launch_gather_segments(const uint32_t *tbl, uint64_t nwords, uint64_t seg_words, uint64_t keys_per_seg,
                            uint64_t nkeys, uint32_t *sink, hipStream_t st) {
    const unsigned grid = grid_for(nkeys, kMaxGrid);
    hipLaunchKernelGGL(k_gather_segments<4>, dim3(grid), dim3(256), 0, st, tbl, nwords, seg_words, keys_per_seg,
                       nkeys, sink);
}

// Streaming-read roofline probe: 16-byte loads of a whole buffer, 4 in flight per lane.
__global__ __launch_bounds__(256) void k_stream_read(const u32x4 *__restrict__ src, uint64_t n16,
                                                     uint32_t *__restrict__ sink) {
    uint32_t acc = 0;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    for (; i + 3 * stride < n16; i += 4 * stride) {
        u32x4 v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) v[u] = __builtin_nontemporal_load(src + i + u * stride);
#pragma unroll
        for (int u = 0; u < 4; ++u) acc ^= v[u].x ^ v[u].y ^ v[u].z ^ v[u].w;
    }
    for (; i < n16; i += stride) {
        const u32x4 v = src[i];
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    if (acc == 0x9E3779B9u) sink[0] = acc;
}

void launch_stream_read(const void *buf, uint64_t bytes, uint32_t *sink, hipStream_t st) {
    hipLaunchKernelGGL(k_stream_read, dim3(4096), dim3(256), 0, st, (const u32x4 *)buf, bytes / 16, sink);
}

// Streaming-write roofline probe: 16-byte nontemporal stores over a whole buffer (whole 64-byte
// write requests, the form the partition passes' runs take).
__global__ __launch_bounds__(256) void k_stream_write(u32x4 *__restrict__ dst, uint64_t n16, uint32_t seed) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += stride) {
        const uint32_t x = (uint32_t)i ^ seed;
        __builtin_nontemporal_store(u32x4{x, x + 1u, x + 2u, x + 3u}, dst + i);
    }
}

void launch_stream_write(void *buf, uint64_t bytes, hipStream_t st) {
    hipLaunchKernelGGL(k_stream_write, dim3(4096), dim3(256), 0, st, (u32x4 *)buf, bytes / 16, 0x9E3779B9u);
}

// Slice-probe roofline: the bitmap is cut into nbuckets slices of 2^slice_log2 bytes; bucket b's
// entries (8 bytes: word offset in the slice, payload) are streamed and each tests one word of
// slice b.  Workgroup w takes the buckets w % 8, w % 8 + 8, ... (blocks b and b + 8 share an XCD
// under the observed round-robin placement: speed only), so one XCD's workgroups gather inside
// one slice at a time and the slice can stay in that XCD's L2.
__global__ __launch_bounds__(256) void k_bench_slice_probe(const u32x2 *__restrict__ ent, uint64_t per_bucket,
                                                           uint32_t nbuckets, const uint32_t *__restrict__ bm,
                                                           uint32_t slice_words_log2, uint32_t *__restrict__ sink) {
    const uint32_t x = blockIdx.x & 7, local = blockIdx.x >> 3, nlocal = gridDim.x >> 3;
    uint32_t acc = 0;
    for (uint32_t b = x; b < nbuckets; b += 8) {
        const u32x2 *e = ent + (uint64_t)b * per_bucket;
        const uint32_t *slice = bm + ((uint64_t)b << slice_words_log2);
        const uint64_t step = (uint64_t)nlocal * 256;
        uint64_t i = (uint64_t)local * 256 + threadIdx.x;
        for (; i + 3 * step < per_bucket; i += 4 * step) {
            u32x2 v[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) v[u] = __builtin_nontemporal_load(e + i + u * step);
#pragma unroll
            for (int u = 0; u < 4; ++u) acc ^= slice[v[u].x & ((1u << slice_words_log2) - 1)] ^ v[u].y;
        }
        for (; i < per_bucket; i += step) {
            const u32x2 v = e[i];
            acc ^= slice[v.x & ((1u << slice_words_log2) - 1)] ^ v.y;
        }
    }
    if (acc == 0x9E3779B9u) sink[0] = acc;
}

void launch_bench_slice_probe(const void *ent, uint64_t per_bucket, uint32_t nbuckets, const uint32_t *bm,
                              uint32_t slice_words_log2, unsigned grid, uint32_t *sink, hipStream_t st) {
    hipLaunchKernelGGL(k_bench_slice_probe, dim3(grid), dim3(256), 0, st, (const u32x2 *)ent, per_bucket, nbuckets, bm,
                       slice_words_log2, sink);
}

void launch_gather_regions(const uint32_t *tbl, uint64_t nwords, uint64_t region_words, uint64_t total_lanes,
                           uint32_t *sink, hipStream_t st, unsigned grid) {
    const uint64_t nregions = nwords / region_words;
    hipLaunchKernelGGL(k_gather_regions, dim3(grid), dim3(256), 0, st, tbl, nregions, region_words,
                       total_lanes / nregions, sink);
}

// ---------------------------------------------------------------------------------
// Filters past the Redis offset limit: |size| > 2^32, reachable only through tryInit with a
// negative expectedInsertions (M/RedissonBloomFilter.java:262-277).  The reference's indexes are
// (h & Long.MAX_VALUE) % size in 64 bits (:139-151); a SETBIT / GETBIT at an offset past 2^32 - 1
// is an error reply that leaves the key alone while the batch's other commands still run, and the
// batch then throws (include/rbx.h RBX_E_REDIS).  A correctness path, not a hot one: plain 64-bit
// remainders, and a first-setter hash table (min key per initially-zero bit) for the in-order add
// replies -- a key is new iff it is the first setter of one of its bits.
// ---------------------------------------------------------------------------------
constexpr unsigned long long kWideEmpty = ~0ULL;
constexpr uint64_t kMaxOffset = 0xFFFFFFFFULL;

__device__ __forceinline__ uint32_t wide_slot(uint64_t idx, uint32_t tlog2) {
    return (uint32_t)((idx * 0x9E3779B97F4A7C15ULL) >> (64 - tlog2));
}

// add pass 1: every in-range bit that is 0 before the chunk gets its smallest key (entry = bit << 32 | key)
__global__ __launch_bounds__(256) void k_wide_claim(KeysDev keys, uint64_t m, uint32_t k, const uint32_t *__restrict__ bm,
                                                    unsigned long long *__restrict__ T, uint32_t tlog2) {
    const uint32_t mask = (1u << tlog2) - 1u;
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < keys.n; i += (uint64_t)gridDim.x * 256) {
        uint64_t h1, h2;
        hash_key<0>(keys, i, h1, h2);
        uint64_t h = h1;
        for (uint32_t j = 0; j < k; ++j) {
            const uint64_t idx = (h & 0x7fffffffffffffffULL) % m;
            h += (j & 1) ? h1 : h2;
            if (idx > kMaxOffset || (bm[idx >> 5] & bit_in_word((uint32_t)idx))) continue;
            const unsigned long long e = (unsigned long long)idx << 32 | i;
            for (uint32_t s = wide_slot(idx, tlog2);; s = (s + 1u) & mask) {
                const unsigned long long prev = atomicCAS(&T[s], kWideEmpty, e);
                if (prev == kWideEmpty) break;
                if ((prev >> 32) == idx) {  // same bit: the smaller key wins (equal high halves)
                    atomicMin(&T[s], e);
                    break;
                }
            }
        }
    }
}

// add pass 2: replies, the first setters' SETBITs (and the Redis string length), the error flag
__global__ __launch_bounds__(256) void k_wide_resolve(KeysDev keys, uint64_t m, uint32_t k, uint32_t *__restrict__ bm,
                                                      unsigned long long *__restrict__ len,
                                                      const unsigned long long *__restrict__ T, uint32_t tlog2,
                                                      uint8_t *__restrict__ out, unsigned long long *__restrict__ count,
                                                      unsigned long long *__restrict__ oob) {
    const uint32_t mask = (1u << tlog2) - 1u;
    uint64_t added = 0;
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < keys.n; i += (uint64_t)gridDim.x * 256) {
        uint64_t h1, h2;
        hash_key<0>(keys, i, h1, h2);
        uint64_t h = h1;
        bool fresh = false, bad = false;
        for (uint32_t j = 0; j < k; ++j) {
            const uint64_t idx = (h & 0x7fffffffffffffffULL) % m;
            h += (j & 1) ? h1 : h2;
            if (idx > kMaxOffset) {
                bad = true;
                continue;
            }
            for (uint32_t s = wide_slot(idx, tlog2);; s = (s + 1u) & mask) {
                const unsigned long long e = T[s];
                if (e == kWideEmpty) break;  // the bit was already 1
                if ((e >> 32) == idx) {
                    if ((uint32_t)e == (uint32_t)i) {  // this key's SETBIT is the one that replied 0
                        fresh = true;
                        atomicOr(&bm[idx >> 5], bit_in_word((uint32_t)idx));
                        raise_redis_len(len, (idx >> 3) + 1);
                    }
                    break;
                }
            }
        }
        if (out) out[i] = fresh;
        added += fresh;
        if (bad) *oob = 1;
    }
    block_add_u64(added, count);
}

// contains: every in-range bit set; an index past the limit flags the call (GETBIT's error reply)
__global__ __launch_bounds__(256) void k_wide_contains(KeysDev keys, uint64_t m, uint32_t k,
                                                       const uint32_t *__restrict__ bm, uint8_t *__restrict__ out,
                                                       unsigned long long *__restrict__ count,
                                                       unsigned long long *__restrict__ oob) {
    uint64_t present = 0;
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < keys.n; i += (uint64_t)gridDim.x * 256) {
        uint64_t h1, h2;
        hash_key<0>(keys, i, h1, h2);
        uint64_t h = h1;
        bool all = true, bad = false;
        for (uint32_t j = 0; j < k; ++j) {
            const uint64_t idx = (h & 0x7fffffffffffffffULL) % m;
            h += (j & 1) ? h1 : h2;
            if (idx > kMaxOffset) bad = true;
            else if (!bm || !(bm[idx >> 5] & bit_in_word((uint32_t)idx))) all = false;  // no key: GETBIT reads 0
        }
        if (out) out[i] = all;
        present += all;
        if (bad) *oob = 1;
    }
    block_add_u64(present, count);
}

void launch_bloom_wide(const KeysDev &keys, uint64_t m, uint32_t k, uint32_t *bm, unsigned long long *len,
                       unsigned long long *table, uint32_t tlog2, bool is_add, uint8_t *out,
                       unsigned long long *count, unsigned long long *oob, hipStream_t st) {
    const unsigned grid = grid_for(keys.n, kMaxGrid);
    if (!is_add) {
        hipLaunchKernelGGL(k_wide_contains, dim3(grid), dim3(256), 0, st, keys, m, k, bm, out, count, oob);
        return;
    }
    hipLaunchKernelGGL(k_wide_claim, dim3(grid), dim3(256), 0, st, keys, m, k, bm, table, tlog2);
    hipLaunchKernelGGL(k_wide_resolve, dim3(grid), dim3(256), 0, st, keys, m, k, bm, len, table, tlog2, out, count,
                       oob);
}
}  // namespace rbx
