// stream_kernels.hip -- the ordered mixed contains/add stream (C5, rbx_bloom_stream[_dev]) and the
// multi-tenant add (rbx_bloom_add_multi[_dev]) on gfx950; split from bloom_kernels.hip in r05 so
// the two compile in parallel.  Semantics: M/RedissonBloomFilter.java:99-137,198-201 with
// M/command/CommandBatchService.java:115-134's in-order execution.
// M/ = /root/reference/redisson/src/main/java/org/redisson/
#include "bloom_common.h"

namespace rbx {

// Looks keypart up; ~0u when absent (linear probing never leaves an unclaimed slot before an
// entry, so the first slot not claimed in this epoch ends the search).
__device__ __forceinline__ uint32_t ht_find(const HTEntry *__restrict__ T, uint32_t log2cap, uint32_t epoch,
                                            uint64_t keypart) {
    const uint64_t mask = (1ULL << log2cap) - 1;
    const uint64_t mytag = ((uint64_t)epoch << 56) | keypart;
    uint64_t slot = ht_slot(keypart, log2cap);
    for (uint64_t probes = 0; probes <= mask; ++probes) {
        const HTEntry e = T[slot];
        if (e.tag == mytag) return (uint32_t)e.idw;
        if ((uint32_t)(e.tag >> 56) != epoch) return 0xffffffffu;
        slot = (slot + 1) & mask;
    }
    return 0xffffffffu;
}

// 8-byte stream first-setter entries (r04; see k_stream_probe8)
__device__ __forceinline__ uint64_t t8_slot(uint64_t key, uint32_t lg) {
    return ((key + 1) * 0x9E3779B97F4A7C15ULL) >> (64 - lg);
}

// returns the slot that holds key's entry
__device__ __forceinline__ uint32_t t8_insert(unsigned long long *__restrict__ T, uint32_t lg, uint32_t pb, uint64_t key,
                                              uint32_t pos) {
    const uint64_t mask = (1ULL << lg) - 1;
    const unsigned long long mine = ((unsigned long long)key << pb) | pos;
    uint64_t slot = t8_slot(key, lg);
    for (uint64_t probes = 0; probes <= mask; ++probes) {
        const unsigned long long old = atomicCAS(&T[slot], ~0ULL, mine);
        if (old == ~0ULL) return (uint32_t)slot;
        if ((old >> pb) == key) {
            if (old > mine) atomicMin(&T[slot], mine);
            return (uint32_t)slot;
        }
        slot = (slot + 1) & mask;
    }
    return (uint32_t)slot;
}

// the first setter's chunk position of key, ~0u when no add of the chunk meets it at 0
__device__ __forceinline__ uint32_t t8_find(const unsigned long long *__restrict__ T, uint32_t lg, uint32_t pb,
                                            uint64_t key) {
    const uint64_t mask = (1ULL << lg) - 1;
    uint64_t slot = t8_slot(key, lg);
    for (uint64_t probes = 0; probes <= mask; ++probes) {
        const unsigned long long e = T[slot];
        if (e == ~0ULL) return 0xffffffffu;
        if ((e >> pb) == key) return (uint32_t)(e & ((1ULL << pb) - 1));
        slot = (slot + 1) & mask;
    }
    return 0xffffffffu;
}

// The zero bits' claims of one add (position t) in the 8-byte table; returns the slot of the first
// zero bit's entry.  batch: every home-slot CAS in flight at once (a C5 add of the fresh stream meets
// ~5 zero bits; one CAS round trip after another was a serial chain per lane), then the rare
// occupied home slot of another bit probes on serially; 0: one insert after another.
template <int KMAX>
__device__ __forceinline__ uint32_t t8_claim(unsigned long long *__restrict__ T, uint32_t lg, uint32_t bb, uint32_t pb,
                                             uint32_t fid, const uint32_t (&idxs)[KMAX], uint32_t zm, uint32_t t,
                                             uint32_t batch) {
    const uint32_t j0 = zm ? (uint32_t)(__ffs(zm) - 1) : 0u;
    uint32_t fs = 0;
    if (batch) {
        const uint64_t mask = (1ULL << lg) - 1;
        unsigned long long old[KMAX];
#pragma unroll
        for (int j = 0; j < KMAX; ++j) {
            if (zm & (1u << j)) {
                const uint64_t key = ((uint64_t)fid << bb) | idxs[j];
                old[j] = atomicCAS(&T[t8_slot(key, lg)], ~0ULL, ((unsigned long long)key << pb) | t);
            }
        }
#pragma unroll
        for (int j = 0; j < KMAX; ++j) {
            if (!(zm & (1u << j))) continue;
            const uint64_t key = ((uint64_t)fid << bb) | idxs[j];
            const unsigned long long mine = ((unsigned long long)key << pb) | t;
            uint64_t slot = t8_slot(key, lg);
            unsigned long long o = old[j];
            for (uint64_t probes = 0; probes <= mask; ++probes) {
                if (o == ~0ULL) break;
                if ((o >> pb) == key) {
                    if (o > mine) atomicMin(&T[slot], mine);
                    break;
                }
                slot = (slot + 1) & mask;
                o = atomicCAS(&T[slot], ~0ULL, mine);
            }
            if ((uint32_t)j == j0) fs = (uint32_t)slot;
        }
    } else {
#pragma unroll
        for (int j = 0; j < KMAX; ++j)
            if (zm & (1u << j)) {
                const uint32_t sl = t8_insert(T, lg, pb, ((uint64_t)fid << bb) | idxs[j], t);
                if ((uint32_t)j == j0) fs = sl;
            }
    }
    return fs;
}

// ---- ordered mixed stream (C5): key i is a single-key contains (op 0) or add (op 1) on
// filters[kf[i]], executed in key order.  Per chunk: compact the adds' positions, probe the adds
// (first-setter table of add positions per initially-zero bit, plus a prefilter bitset of the
// (filter, bit) pairs they touch), then the contains -- a zero bit counts as set iff an add at
// an earlier position of the chunk touches it; the table is consulted only when the prefilter
// bit is set -- then commit the adds.  Earlier chunks are committed before later ones probe, so
// chunking keeps the order.  The add list is unordered: owners are resolved by atomicMin.
// prefilter of 2^pbits bits (rbx_tune "stream_prefilter", default 2^23 = 1 MiB: L2-resident while
// the contains run, beside the Zipf-hot bitmaps); pshift = 64 - pbits
__device__ __forceinline__ uint32_t prefilter_bit(uint32_t fid, uint32_t idx, uint32_t pshift) {
    return (uint32_t)(((((uint64_t)fid << 32) | idx) * 0x9E3779B97F4A7C15ULL) >> pshift);
}

// May this clear bit have been set by an earlier add of the chunk (look it up in the table)?
// pshift 0 (r04, with the 8-byte table): `filter` is the occupancy bitmap of the table's slots
// (k_stream_occ) -- linear probing puts a key at or after its home slot, so an empty home slot
// means the key is absent; else `filter` is the (fid, bit) prefilter the adds set; NULL: always.
__device__ __forceinline__ bool maybe_claimed(const uint32_t *__restrict__ filter, uint32_t pshift, uint32_t fid,
                                              uint32_t idx, uint64_t key8, uint32_t lg8) {
    if (!filter) return true;
    const uint64_t b = pshift ? (uint64_t)prefilter_bit(fid, idx, pshift) : t8_slot(key8, lg8);
    return (filter[b >> 5] >> (b & 31)) & 1u;
}

// adds[0 .. *nadds) = chunk-local positions of the chunk's adds (any order)
constexpr uint32_t kCompactPer = 64, kCompactBlock = 256 * kCompactPer;  // commands per lane / per block
__global__ __launch_bounds__(256) void k_stream_compact(const uint8_t *__restrict__ op, uint64_t base, uint64_t nchunk,
                                                        uint32_t *__restrict__ adds, uint32_t *__restrict__ nadds) {
    // One pass, kCompactBlock commands per block, kCompactPer consecutive per lane: a block scan of the
    // lanes' add counts and ONE reservation per block.  The reservations of a chunk all go to one
    // counter, which serialises them (~88 per us): 4096-command blocks -- 2K reservations per 8.4M-command
    // chunk -- took 33 us a chunk; 16K-command blocks take a quarter of them (r05).  (A reservation per
    // 1024-command tile, or a block walking a long slice, left the kernel latency-bound: 79 / 38 us for
    // 6.7M commands.)
    __shared__ uint32_t s_w[4], s_base;
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint64_t t0 = (uint64_t)blockIdx.x * kCompactBlock + threadIdx.x * kCompactPer;
    uint64_t bits = 0;
    if (t0 + kCompactPer <= nchunk && ((uintptr_t)(op + base + t0) & 15) == 0) {  // 16 op bytes per load
        using u8x16v = uint8_t __attribute__((ext_vector_type(16)));
#pragma unroll
        for (uint32_t g = 0; g < kCompactPer / 16; ++g) {
            const u8x16v v = *(const u8x16v *)(op + base + t0 + 16 * g);
#pragma unroll
            for (int q = 0; q < 16; ++q)
                if (v[q]) bits |= 1ULL << (16 * g + q);
        }
    } else {
        for (uint32_t q = 0; q < kCompactPer; ++q)
            if (t0 + q < nchunk && op[base + t0 + q]) bits |= 1ULL << q;
    }
    const uint32_t c = (uint32_t)__popcll(bits);
    uint32_t x = c;  // inclusive scan over the wave
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const uint32_t y = __shfl_up(x, off, 64);
        if (lane >= (uint32_t)off) x += y;
    }
    if (lane == 63) s_w[wave] = x;
    __syncthreads();
    if (threadIdx.x == 0) {
        const uint32_t tot = s_w[0] + s_w[1] + s_w[2] + s_w[3];
        s_base = tot ? atomicAdd(nadds, tot) : 0u;
    }
    __syncthreads();
    uint32_t pos = s_base + x - c;
    for (uint32_t w = 0; w < wave; ++w) pos += s_w[w];
    while (bits) {
        adds[pos++] = (uint32_t)(t0 + (uint32_t)(__ffsll((unsigned long long)bits) - 1));
        bits &= bits - 1;
    }
}

template <int KLEN, int KMAX>
__global__ __launch_bounds__(256) void k_stream_probe(KeysDev keys, uint64_t base, const uint32_t *__restrict__ adds,
                                                      const uint32_t *__restrict__ nadds,
                                                      const FilterDesc *__restrict__ filt,
                                                      const uint32_t *__restrict__ kf, HTEntry *__restrict__ T,
                                                      uint32_t log2cap, uint32_t epoch, uint32_t *__restrict__ zmask,
                                                      uint32_t *__restrict__ prefilter, uint32_t pshift) {
    const uint32_t na = *nadds;
    const uint32_t stride = gridDim.x * blockDim.x;
    for (uint32_t a = blockIdx.x * blockDim.x + threadIdx.x; a < na; a += stride) {
        const uint32_t t = adds[a];
        const uint64_t i = base + t;
        uint32_t zm = 0;
        const FilterDesc f = filt[kf[i]];
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
#pragma unroll
        for (int j = 0; j < KMAX; ++j) {
            if ((uint32_t)j < f.k && (word[j] & bit_in_word(idxs[j])) == 0u) {
                zm |= 1u << j;
                ht_insert(T, log2cap, epoch, ((uint64_t)f.fid << 32) | idxs[j], t);
                if (prefilter) {
                    const uint32_t pb = prefilter_bit(f.fid, idxs[j], pshift);
                    atomicOr(&prefilter[pb >> 5], 1u << (pb & 31));
                }
            }
        }
        raise_redis_len(f.redis_len, (unsigned long long)(maxidx >> 3) + 1ULL);
        zmask[a] = zm;
    }
}

template <int KLEN, int KMAX>
__global__ __launch_bounds__(256) void k_stream_contains(KeysDev keys, uint64_t base, uint64_t nchunk,
                                                         const FilterDesc *__restrict__ filt,
                                                         const uint32_t *__restrict__ kf,
                                                         const uint8_t *__restrict__ op,
                                                         const HTEntry *__restrict__ T, uint32_t log2cap,
                                                         uint32_t epoch, const uint32_t *__restrict__ prefilter,
                                                         uint32_t pshift,
                                                         uint8_t *__restrict__ out,
                                                         unsigned long long *__restrict__ counts,
                                                         const unsigned long long *__restrict__ T8, uint32_t bb,
                                                         uint32_t pb, uint32_t kmax, const uint32_t *__restrict__ nadds) {
    uint64_t present = 0;
    const uint32_t lg8 = T8 ? t8_log2(*nadds, kmax) : 0;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; t < nchunk; t += stride) {
        const uint64_t i = base + t;
        if (op[i]) continue;
        const FilterDesc f = filt[kf[i]];
        uint64_t h1, h2;
        hash_key<KLEN>(keys, i, h1, h2);
        // doubling stages 1, 2, 4, ...: all loads of a stage in flight, stop at a clear bit
        bool all = true;
        uint64_t h = h1;
        uint32_t j = 0;
        for (uint32_t width = 1; j < f.k && all; width <<= 1) {
            uint32_t word[KMAX], idxs[KMAX];
            const uint32_t e = min(f.k, j + width);
#pragma unroll
            for (int u = 0; u < KMAX; ++u) {
                if (j + u < e) {
                    const uint32_t idx = mod63(h & 0x7fffffffffffffffULL, f.mp);
                    idxs[u] = idx;
                    word[u] = f.bm[idx >> 5];
                    h += ((j + u) & 1) ? h1 : h2;
                }
            }
#pragma unroll
            for (int u = 0; u < KMAX; ++u) {
                if (j + u < e && all && (word[u] & bit_in_word(idxs[u])) == 0u) {
                    // set by an earlier add of this chunk?  Only possible if the filter says so.
                    if (maybe_claimed(prefilter, pshift, f.fid, idxs[u], ((uint64_t)f.fid << bb) | idxs[u], lg8)) {
                        const uint32_t owner = T8 ? t8_find(T8, lg8, pb, ((uint64_t)f.fid << bb) | idxs[u])
                                                  : ht_find(T, log2cap, epoch, ((uint64_t)f.fid << 32) | idxs[u]);
                        all = owner < (uint32_t)t;
                    } else {
                        all = false;
                    }
                }
            }
            j = e;
        }
        if (out) out[i] = all;
        present += all;
    }
    if (counts) block_add_u64(present, counts);
}

// The same answers with the per-lane slot schedule of k_bloom_contains_q (§3.1b): one bit per
// key per round trip, P keys in flight per lane.  A wave's queue holds only the chunk's contains
// commands (ballot-compacted while the wave hashes a 64*Q-command range), so add commands cost
// no lane time, and a clear bit consults the prefilter / first-setter table exactly as above.
template <int KLEN, int P, int Q>
__global__ __launch_bounds__(256) void k_stream_contains_q(KeysDev keys, uint64_t base, uint64_t nchunk,
                                                           const ProbeDesc *__restrict__ pdesc,
                                                           const uint32_t *__restrict__ kf,
                                                           const uint8_t *__restrict__ op,
                                                           const HTEntry *__restrict__ T, uint32_t log2cap,
                                                           uint32_t epoch, const uint32_t *__restrict__ prefilter,
                                                           uint32_t pshift,
                                                           uint8_t *__restrict__ out,
                                                           unsigned long long *__restrict__ counts,
                                                           const unsigned long long *__restrict__ T8, uint32_t bb,
                                                           uint32_t pb, uint32_t kmax,
                                                           const uint32_t *__restrict__ nadds, uint32_t diag = 0,
                                                           uint32_t lookup_rounds = 0) {
    constexpr uint32_t RANGE = 64 * Q, WAVES = 4;
    const uint32_t lg8 = T8 ? t8_log2(*nadds, kmax) : 0;
    // r05: with the 8-byte table and no prefilter, a clear bit's first-setter lookup is a round of
    // its own: the slot's next load is the table entry instead of a bitmap word, in flight with
    // the other slots' gathers (inline, each lookup chain stalled the lane's whole round)
    const bool rounds = lookup_rounds && T8 && !prefilter && !(diag & 1);
    const uint32_t tmask = (uint32_t)((1ULL << lg8) - 1);
    const uint64_t pmask = (1ULL << pb) - 1;
    struct alignas(16) QEnt {
        uint64_t h1, h2;
        uint32_t t, fi, idx0, pad;  // chunk-local command index, filter index, first bit
    };
    __shared__ QEnt s_q[WAVES][2][RANGE];
    const uint32_t wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const uint64_t lt = (1ULL << lane) - 1;
    QEnt *qb = &s_q[wave][0][0];
    const uint64_t nranges = (nchunk + RANGE - 1) / RANGE;
    const uint64_t nw = (uint64_t)gridDim.x * WAVES;
    uint64_t rnext = (uint64_t)blockIdx.x * WAVES + wave;
    uint32_t qlen[2] = {0, 0};
    auto fill = [&](uint32_t b) {  // wave-uniform: the contains of the next non-empty range
        qlen[b] = 0;
        while (qlen[b] == 0 && rnext < nranges) {
            const uint64_t rb = rnext * RANGE;
#pragma unroll
            for (uint32_t q = 0; q < Q; ++q) {
                const uint64_t t = rb + q * 64 + lane;
                const bool c = t < nchunk && op[base + t] == 0;
                const uint64_t mask = __ballot(c);
                if (c) {
                    QEnt e;
                    hash_key<KLEN>(keys, base + t, e.h1, e.h2);
                    e.t = (uint32_t)t;
                    e.fi = kf[base + t];
                    e.idx0 = mod63c(e.h1 & 0x7fffffffffffffffULL, pdesc[e.fi].mc);
                    qb[b * RANGE + qlen[b] + (uint32_t)__popcll(mask & lt)] = e;
                }
                qlen[b] += (uint32_t)__popcll(mask);
            }
            rnext += nw;
        }
        __builtin_amdgcn_wave_barrier();
    };
    bool act[P], sph[P];  // sph: the slot's next load is a first-setter table entry (lookup round)
    uint64_t sh1[P], sh2[P], sh[P];
    uint32_t st[P], sjk[P], sidx[P], sfid[P], tsl[P];  // command index, j | k << 16, bit index, table id, table slot
    const uint32_t *sbm[P];
    ModC smp[P];
#pragma unroll
    for (int s = 0; s < P; ++s) act[s] = sph[s] = false;
    uint32_t cur = 0, qpos = 0;
    int stale = -1;
    fill(0);
    fill(1);
    uint64_t present = 0;
    for (;;) {
#pragma unroll
        for (int s = 0; s < P; ++s) {
            bool need = !act[s];
            for (;;) {
                const uint64_t nm = __ballot(need);
                if (!nm) break;
                if (qpos >= qlen[cur]) {
                    if (stale == (int)(cur ^ 1)) {
                        fill(cur ^ 1);
                        stale = -1;
                    }
                    if (qlen[cur ^ 1] == 0) break;
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
                    const ProbeDesc f = pdesc[e.fi];
                    act[s] = true;
                    need = false;
                    sh1[s] = e.h1;
                    sh2[s] = e.h2;
                    sh[s] = e.h1 + e.h2;
                    st[s] = e.t;
                    sidx[s] = e.idx0;
                    sbm[s] = f.bm;
                    smp[s] = f.mc;
                    sjk[s] = f.k << 16;
                    sfid[s] = f.fid;
                }
                qpos += min<uint32_t>((uint32_t)__popcll(nm), avail);
            }
        }
        bool any = false;
#pragma unroll
        for (int s = 0; s < P; ++s) any |= act[s];
        if (!__ballot(any)) break;
        unsigned long long e8[P];  // a table entry (lookup round) or, in its low half, a bitmap word
#pragma unroll
        for (int s = 0; s < P; ++s) {
            if (act[s] && sph[s]) e8[s] = T8[tsl[s]];
            else if (act[s]) e8[s] = sbm[s][sidx[s] >> 5];
        }
        if (stale >= 0) {
            fill((uint32_t)stale);
            stale = -1;
        }
#pragma unroll
        for (int s = 0; s < P; ++s) {
            bool fin_p = false;
            if (act[s]) {
                bool clear;
                if (sph[s]) {  // lookup round: EMPTY ends the probe (not claimed), another key probes on
                    const uint64_t key = ((uint64_t)sfid[s] << bb) | sidx[s];
                    const unsigned long long e = e8[s];
                    if (e != ~0ULL && (e >> pb) != key) {
                        tsl[s] = (tsl[s] + 1) & tmask;
                        continue;
                    }
                    sph[s] = false;
                    clear = e == ~0ULL || !((uint32_t)(e & pmask) < st[s]);
                } else {
                    clear = ((uint32_t)e8[s] & bit_in_word(sidx[s])) == 0u;
                    if (clear && rounds) {
                        sph[s] = true;
                        tsl[s] = (uint32_t)t8_slot(((uint64_t)sfid[s] << bb) | sidx[s], lg8);
                        continue;
                    }
                    if (clear && !(diag & 1)) {  // set by an earlier add of this chunk?  Only if the filter says so.
                        if (maybe_claimed(prefilter, pshift, sfid[s], sidx[s], ((uint64_t)sfid[s] << bb) | sidx[s], lg8))
                            clear = !((T8 ? t8_find(T8, lg8, pb, ((uint64_t)sfid[s] << bb) | sidx[s])
                                          : ht_find(T, log2cap, epoch, ((uint64_t)sfid[s] << 32) | sidx[s])) < st[s]);
                    }
                }
                bool fin = clear;
                if (!clear && ((++sjk[s]) & 0xffffu) >= (sjk[s] >> 16)) {
                    fin = fin_p = true;
                } else if (!clear) {
                    sidx[s] = mod63c(sh[s] & 0x7fffffffffffffffULL, smp[s]);
                    sh[s] += (sjk[s] & 1) ? sh1[s] : sh2[s];
                }
                if (fin) {
                    act[s] = false;
                    if (out) out[base + st[s]] = fin_p;
                }
            }
            present += fin_p;
        }
    }
    if (counts) block_add_u64(present, counts);
}

template <int KLEN, int KMAX>
__global__ __launch_bounds__(256) void k_stream_commit(KeysDev keys, uint64_t base, const uint32_t *__restrict__ adds,
                                                       const uint32_t *__restrict__ nadds,
                                                       const FilterDesc *__restrict__ filt,
                                                       const uint32_t *__restrict__ kf, const HTEntry *__restrict__ T,
                                                       uint32_t log2cap, uint32_t epoch,
                                                       const uint32_t *__restrict__ zmask, uint8_t *__restrict__ out,
                                                       unsigned long long *__restrict__ counts) {
    uint64_t added = 0;
    const uint32_t na = *nadds;
    const uint32_t stride = gridDim.x * blockDim.x;
    for (uint32_t a = blockIdx.x * blockDim.x + threadIdx.x; a < na; a += stride) {
        const uint32_t t = adds[a];
        const uint64_t i = base + t;
        const uint32_t zm = zmask[a];
        bool isnew = false;
        if (zm) {
            const FilterDesc f = filt[kf[i]];
            uint64_t h1, h2;
            hash_key<KLEN>(keys, i, h1, h2);
            uint64_t h = h1;
#pragma unroll
            for (int j = 0; j < KMAX; ++j) {
                if ((zm >> j) & 1u) {
                    const uint32_t idx = mod63(h & 0x7fffffffffffffffULL, f.mp);
                    if (ht_owner(T, log2cap, epoch, ((uint64_t)f.fid << 32) | idx) == t) {
                        isnew = true;
                        atomicOr(&f.bm[idx >> 5], bit_in_word(idx));
                    }
                }
                h += (j & 1) ? h1 : h2;
            }
        }
        if (out) out[i] = isnew;
        added += isnew;
    }
    if (counts) block_add_u64(added, counts + 1);
}

// ---- ordered stream, r04: 8-byte first-setter entries, committed by a table walk -------------
// The r03 probe spent ~15 memory requests per add: per zero bit a tag load, a CAS and
// an atomicMin on a 16-byte entry of a 2 GiB epoch-tagged table, plus the commit's re-hash, zmask
// read and owner lookup per zero bit.  Here an entry is ONE word, (fid << bb | bit) << pb | position:
// a zero bit is claimed by one CAS on an empty slot (a slot already holding the bit takes an
// atomicMin -- same high bits, so the minimum is the first setter), the table is sized to the
// chunk's adds (2^t8_log2 entries, e.g. 16M = 128 MiB for a C5 chunk's 838K adds), and the commit is a
// streaming walk over it: every entry is an owned bit (its minimum position is the first add that
// meets it at 0), so the walk ORs the bit into its bitmap, flags its owner and empties the slot.
// A final pass over the add list turns the flags into replies and the new-add count.
template <int KLEN, int KMAX>
__global__ __launch_bounds__(256) void k_stream_probe8(KeysDev keys, uint64_t base, const uint32_t *__restrict__ adds,
                                                       const uint32_t *__restrict__ nadds,
                                                       const FilterDesc *__restrict__ filt,
                                                       const uint32_t *__restrict__ kf, unsigned long long *__restrict__ T,
                                                       uint32_t bb, uint32_t pb, uint32_t kmax,
                                                       uint32_t *__restrict__ prefilter, uint32_t pshift,
                                                       uint32_t batch, uint32_t *__restrict__ zmask,
                                                       uint32_t *__restrict__ fslot) {
    const uint32_t na = *nadds;
    const uint32_t lg = t8_log2(na, kmax);
    const uint32_t stride = gridDim.x * blockDim.x;
    for (uint32_t a = blockIdx.x * blockDim.x + threadIdx.x; a < na; a += stride) {
        const uint32_t t = adds[a];
        const uint64_t i = base + t;
        const FilterDesc f = filt[kf[i]];
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
        for (int j = 0; j < KMAX; ++j)
            if ((uint32_t)j < f.k && (word[j] & bit_in_word(idxs[j])) == 0u) zm |= 1u << j;
        if (batch == 2) zm = 0;  // DIAGNOSTIC: no claims
        // the slot of the first zero bit's entry: k_stream_final8 decides the reply from it
        const uint32_t fs = t8_claim<KMAX>(T, lg, bb, pb, f.fid, idxs, zm, t, batch);
        if (zmask) {
            zmask[a] = zm;
            fslot[a] = fs;
        }
        if (prefilter && pshift) {  // pshift 0: occupancy bitmap, built by k_stream_occ
#pragma unroll
            for (int j = 0; j < KMAX; ++j) {
                if (zm & (1u << j)) {
                    const uint32_t pb2 = prefilter_bit(f.fid, idxs[j], pshift);
                    atomicOr(&prefilter[pb2 >> 5], 1u << (pb2 & 31));
                }
            }
        }
        raise_redis_len(f.redis_len, (unsigned long long)(maxidx >> 3) + 1ULL);
    }
}

// the occupancy bitmap of the table's 2^lg slots (bit s = slot s holds an entry), one ballot per 64
// slots: streamed after the probe, no atomics (the r03 prefilter cost a memory-side atomicOr per
// zero bit).  lg >= 12, so every wave's 64 slots exist.
__global__ __launch_bounds__(256) void k_stream_occ(const unsigned long long *__restrict__ T,
                                                    const uint32_t *__restrict__ nadds, uint32_t kmax,
                                                    uint32_t *__restrict__ occ) {
    const uint64_t nslots = 1ULL << t8_log2(*nadds, kmax);
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t s = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; s - (threadIdx.x & 63) < nslots; s += stride) {
        const uint64_t m = __ballot(T[s] != ~0ULL);
        if ((threadIdx.x & 63) == 0) ((unsigned long long *)occ)[s >> 6] = m;
    }
}

// every entry: OR its bit into its bitmap, flag its owner, empty the slot (two entries per lane)
__global__ __launch_bounds__(256) void k_stream_walk(unsigned long long *__restrict__ T, const uint32_t *__restrict__ nadds,
                                                     uint32_t kmax, uint32_t bb, uint32_t pb,
                                                     uint32_t *const *__restrict__ fid_bm, uint8_t *__restrict__ flag,
                                                     uint32_t diag = 0, uint32_t reset_all = 0) {
    // reset_all: every pair is rewritten EMPTY with whole-line streaming stores (at the ~30% loads
    // the tables run at almost every line holds an entry, and one scattered 16-byte store per
    // occupied pair cost a partial-line write request each); 0: only occupied pairs are rewritten
    const uint32_t lg = nadds ? t8_log2(*nadds, kmax) : kmax;  // no count: kmax carries lg itself
    const uint64_t n2 = (1ULL << lg) / 2;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    const uint64_t pmask = (1ULL << pb) - 1, bmask = (1ULL << bb) - 1;
    using u64x2 = unsigned long long __attribute__((ext_vector_type(2)));
    for (uint64_t q = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; q < n2; q += stride) {
        u64x2 e = ((const u64x2 *)T)[q];
        if ((e.x & e.y) == ~0ULL) {  // both empty
            if (reset_all) __builtin_nontemporal_store(u64x2{~0ULL, ~0ULL}, (u64x2 *)T + q);
            continue;
        }
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const unsigned long long v = h ? e.y : e.x;
            if (v == ~0ULL) continue;
            const uint64_t key = v >> pb;
            const uint32_t bit = (uint32_t)(key & bmask);
            if (diag & 2) fid_bm[key >> bb][bit >> 5] |= bit_in_word(bit);  // DIAGNOSTIC (racy)
            else atomicOr(&fid_bm[key >> bb][bit >> 5], bit_in_word(bit));
            if (flag && !(diag & 4)) flag[v & pmask] = 1;
        }
        if (reset_all) __builtin_nontemporal_store(u64x2{~0ULL, ~0ULL}, (u64x2 *)T + q);
        else ((u64x2 *)T)[q] = u64x2{~0ULL, ~0ULL};
    }
}

// replies and the new-add count from the owner flags; the flags are cleared for the next chunk
__global__ __launch_bounds__(256) void k_stream_final(uint64_t base, const uint32_t *__restrict__ adds,
                                                      const uint32_t *__restrict__ nadds, uint8_t *__restrict__ flag,
                                                      uint8_t *__restrict__ out, unsigned long long *__restrict__ counts) {
    uint64_t added = 0;
    const uint32_t na = *nadds;
    const uint32_t stride = gridDim.x * blockDim.x;
    for (uint32_t a = blockIdx.x * blockDim.x + threadIdx.x; a < na; a += stride) {
        const uint32_t t = adds[a];
        const uint8_t v = flag[t];
        if (v) flag[t] = 0;
        if (out) out[base + t] = v;
        added += v;
    }
    if (counts) block_add_u64(added, counts + 1);
}

// r05: replies and the new-add count without owner flags, BEFORE the walk empties the table.  An
// add is new iff it is the first setter of one of its zero bits; the entry of its FIRST zero bit
// (slot recorded by the probe) decides almost every add at one load: position == t -> new.  Only when
// an earlier add of the chunk claimed that bit too (a shared bit: the same key added twice, or two
// keys colliding on a bit) are the remaining zero bits looked up, the indexes recomputed from the key.
// (The r04 walk stored a flag byte per owned bit -- ~4.3 per add, scattered -- and a final pass read
// them back.)
template <int KLEN, int KMAX>
__global__ __launch_bounds__(256) void k_stream_final8(KeysDev keys, uint64_t base, const uint32_t *__restrict__ adds,
                                                       const uint32_t *__restrict__ nadds,
                                                       const FilterDesc *__restrict__ filt,
                                                       const uint32_t *__restrict__ kf,
                                                       const unsigned long long *__restrict__ T, uint32_t bb,
                                                       uint32_t pb, uint32_t kmax, const uint32_t *__restrict__ zmask,
                                                       const uint32_t *__restrict__ fslot, uint8_t *__restrict__ out,
                                                       unsigned long long *__restrict__ counts) {
    uint64_t added = 0;
    const uint32_t na = *nadds;
    const uint32_t lg = t8_log2(na, kmax);
    const uint64_t pmask = (1ULL << pb) - 1;
    const uint32_t stride = gridDim.x * blockDim.x;
    for (uint32_t a = blockIdx.x * blockDim.x + threadIdx.x; a < na; a += stride) {
        const uint32_t t = adds[a];
        const uint32_t zm = zmask[a];
        bool isnew = false;
        if (zm) {
            isnew = (T[fslot[a]] & pmask) == t;
            const uint32_t rest = zm & (zm - 1);
            if (!isnew && rest) {  // the first zero bit is shared with an earlier add: the others
                const uint64_t i = base + t;
                const FilterDesc f = filt[kf[i]];
                uint64_t h1, h2;
                hash_key<KLEN>(keys, i, h1, h2);
                uint64_t h = h1;
#pragma unroll
                for (int j = 0; j < KMAX; ++j) {
                    if (((rest >> j) & 1u) && !isnew) {
                        const uint32_t idx = mod63(h & 0x7fffffffffffffffULL, f.mp);
                        isnew = t8_find(T, lg, pb, ((uint64_t)f.fid << bb) | idx) == t;
                    }
                    h += (j & 1) ? h1 : h2;
                }
            }
        }
        if (out) out[base + t] = isnew;
        added += isnew;
    }
    if (counts) block_add_u64(added, counts + 1);
}

// ---- multi-tenant add (r05): the stream's 8-byte first-setter table for add(Collection) batches -
// A multi-tenant add batch (segment s = keys [seg_off[s], seg_off[s+1]) added to filters[s], the
// segments in order) is the ordered stream with every command an add: key t of a chunk claims its
// zero bits with entries ((fid << bb | bit) << pb) | t (one CAS each, t8_claim), the reply comes from
// the entry of its first zero bit (k_madd_final8), and k_stream_walk ORs every owned bit and empties
// the table.  The r03 path kept 16-byte epoch-tagged entries (a CAS and an atomicMin per zero bit), a
// commit that re-hashed every key to look its zero bits up again, and one atomicAdd per new key into
// its segment's count; here the counts are one atomic per (wave, segment).
template <int KLEN, int KMAX>
__global__ __launch_bounds__(256) void k_madd_probe8(KeysDev keys, uint64_t base, uint64_t nchunk,
                                                     const FilterDesc *__restrict__ filt,
                                                     const uint64_t *__restrict__ seg_off, uint32_t nseg,
                                                     const uint32_t *__restrict__ tile_seg0,
                                                     unsigned long long *__restrict__ T, uint32_t lg, uint32_t bb,
                                                     uint32_t pb, uint32_t batch, uint32_t *__restrict__ zmask,
                                                     uint32_t *__restrict__ fslot) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; t < nchunk; t += stride) {
        const uint64_t i = base + t;
        const FilterDesc f = filt[seg_from(seg_off, nseg, tile_seg0[i >> 8], i)];
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
        for (int j = 0; j < KMAX; ++j)
            if ((uint32_t)j < f.k && (word[j] & bit_in_word(idxs[j])) == 0u) zm |= 1u << j;
        const uint32_t fs = t8_claim<KMAX>(T, lg, bb, pb, f.fid, idxs, zm, (uint32_t)t, batch);
        zmask[t] = zm;
        fslot[t] = fs;
        raise_redis_len(f.redis_len, (unsigned long long)(maxidx >> 3) + 1ULL);
    }
}

template <int KLEN, int KMAX>
__global__ __launch_bounds__(256) void k_madd_final8(KeysDev keys, uint64_t base, uint64_t nchunk,
                                                     const FilterDesc *__restrict__ filt,
                                                     const uint64_t *__restrict__ seg_off, uint32_t nseg,
                                                     const uint32_t *__restrict__ tile_seg0,
                                                     const unsigned long long *__restrict__ T, uint32_t lg, uint32_t bb,
                                                     uint32_t pb, const uint32_t *__restrict__ zmask,
                                                     const uint32_t *__restrict__ fslot, uint8_t *__restrict__ out_new,
                                                     unsigned long long *__restrict__ seg_counts) {
    const uint64_t pmask = (1ULL << pb) - 1;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    // every lane of a wave runs the same number of iterations (wave_seg_add is a wave operation)
    const uint64_t n_up = (nchunk + 63) & ~63ULL;
    for (uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; t < n_up; t += stride) {
        const bool in = t < nchunk;
        const uint64_t i = base + t;
        uint32_t seg = 0;
        bool isnew = false;
        if (in) {
            seg = seg_from(seg_off, nseg, tile_seg0[i >> 8], i);
            const uint32_t zm = zmask[t];
            if (zm) {
                isnew = (T[fslot[t]] & pmask) == t;
                const uint32_t rest = zm & (zm - 1);
                if (!isnew && rest) {  // the first zero bit is shared with an earlier key: the others
                    const FilterDesc f = filt[seg];
                    uint64_t h1, h2;
                    hash_key<KLEN>(keys, i, h1, h2);
                    uint64_t h = h1;
#pragma unroll
                    for (int j = 0; j < KMAX; ++j) {
                        if (((rest >> j) & 1u) && !isnew) {
                            const uint32_t idx = mod63(h & 0x7fffffffffffffffULL, f.mp);
                            isnew = t8_find(T, lg, pb, ((uint64_t)f.fid << bb) | idx) == (uint32_t)t;
                        }
                        h += (j & 1) ? h1 : h2;
                    }
                }
            }
            if (out_new) out_new[i] = isnew;
        }
        if (seg_counts) wave_seg_add(in, seg, isnew ? 1u : 0u, seg_counts);
    }
}

// ---- multi-tenant add, r05 default: optimistic SETBITs with conflict repair ---------------------
// The first-setter table costs a CAS per zero bit and the walk an atomicOr per owned bit: 11 memory-side
// atomics per C3 key, which bound the call (profiles/r05: 1.1G atomics per 100M-key add_multi).  But a
// zero bit matters for the in-order replies only when two keys of the chunk share it.  So:
//   K1 k_maddx_gather: the k bits of every key are read BEFORE any is set (zmask = zero bits);
//   K2 k_maddx_set:    every zero bit is set with a returning atomicOr; a key that finds its zero bit
//                      already set (another key of the chunk set it first, in execution order) records
//                      the bit in a small conflict table C (entry (fid << bb | bit) << pb | position,
//                      atomicMin: the smallest position among the losers);
//   K3 k_maddx_claim:  only when C is not empty: every key registers its zero bits that are in C
//                      (atomicMin), so C holds each shared bit's first setter in key order;
//   K4 k_maddx_reply:  key t is new iff one of its zero bits is not in C (t is its only setter) or is
//                      in C with first setter t.
// Bits: the same SETBITs land (every zero bit of every key), so bitmap bytes are identical.  Replies:
// exact (M/RedissonBloomFilter.java:104-137 with M/command/CommandBatchService.java:115-134's order).
// C overflows (more than half full, or a probe run past 64 slots: adversarial batches of repeated keys)
// -> K3 registers every zero bit of every key in the full 8-byte first-setter table T instead, K4
// answers from T, and K5 empties T again.  Atomics per C3 key: ~5 (the SETBITs) instead of ~11.
template <int KMAX>
__device__ __forceinline__ void madd_indexes(uint64_t h1, uint64_t h2, const ModParams &mp, uint32_t zm,
                                             uint32_t (&idxs)[KMAX]) {
    uint64_t h = h1;
#pragma unroll
    for (int j = 0; j < KMAX; ++j) {
        if ((zm >> j) & 1u) idxs[j] = mod63(h & 0x7fffffffffffffffULL, mp);
        h += (j & 1) ? h1 : h2;
    }
}

// slot of key8 in C, or -1 (linear probing; C is never more than half full when consulted)
__device__ __forceinline__ int64_t c_find(const unsigned long long *__restrict__ C, uint32_t lgC, uint32_t pb,
                                          uint64_t key8, unsigned long long *e_out) {
    const uint64_t mask = (1ULL << lgC) - 1;
    uint64_t slot = t8_slot(key8, lgC);
    for (uint32_t probes = 0; probes < 64; ++probes) {
        const unsigned long long e = C[slot];
        if (e == ~0ULL) return -1;
        if ((e >> pb) == key8) {
            *e_out = e;
            return (int64_t)slot;
        }
        slot = (slot + 1) & mask;
    }
    return -1;  // unreachable while the overflow rule holds (an insert past 64 probes overflows)
}

template <int KLEN, int KMAX>
__global__ __launch_bounds__(256) void k_maddx_gather(KeysDev keys, uint64_t base, uint64_t nchunk,
                                                      const FilterDesc *__restrict__ filt,
                                                      const uint64_t *__restrict__ seg_off, uint32_t nseg,
                                                      const uint32_t *__restrict__ tile_seg0,
                                                      uint32_t *__restrict__ zmask, unsigned long long *__restrict__ C,
                                                      uint32_t lgC, MaddxState *__restrict__ cst,
                                                      const uint32_t *__restrict__ big, uint64_t segmax) {
    if (big && !*big) return;  // k_madd_seg took every segment (uniform; K2..K5 check the same word)
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    const uint64_t tid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    for (uint64_t s = tid; s < (1ULL << lgC); s += stride) C[s] = ~0ULL;  // the previous chunk's C
    if (tid == 0) *cst = MaddxState{0, 0};
    for (uint64_t t = tid; t < nchunk; t += stride) {
        const uint64_t i = base + t;
        const uint32_t sg = seg_from(seg_off, nseg, tile_seg0[i >> 8], i);
        if (big && seg_off[sg + 1] - seg_off[sg] <= segmax) {  // k_madd_seg's segment: not here
            zmask[t] = 0;
            continue;
        }
        const FilterDesc f = filt[sg];
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
        for (int j = 0; j < KMAX; ++j)
            if ((uint32_t)j < f.k && (word[j] & bit_in_word(idxs[j])) == 0u) zm |= 1u << j;
        zmask[t] = zm;
        raise_redis_len(f.redis_len, (unsigned long long)(maxidx >> 3) + 1ULL);
    }
}

template <int KLEN, int KMAX>
__global__ __launch_bounds__(256) void k_maddx_set(KeysDev keys, uint64_t base, uint64_t nchunk,
                                                   const FilterDesc *__restrict__ filt,
                                                   const uint64_t *__restrict__ seg_off, uint32_t nseg,
                                                   const uint32_t *__restrict__ tile_seg0,
                                                   const uint32_t *__restrict__ zmask,
                                                   unsigned long long *__restrict__ C, uint32_t lgC, uint32_t bb,
                                                   uint32_t pb, MaddxState *__restrict__ cst,
                                                   const uint32_t *__restrict__ big) {
    if (big && !*big) return;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    const uint64_t cmask = (1ULL << lgC) - 1;
    for (uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; t < nchunk; t += stride) {
        const uint32_t zm = zmask[t];
        if (!zm) continue;
        const uint64_t i = base + t;
        const FilterDesc f = filt[seg_from(seg_off, nseg, tile_seg0[i >> 8], i)];
        uint64_t h1, h2;
        hash_key<KLEN>(keys, i, h1, h2);
        uint32_t idxs[KMAX], old[KMAX];
        madd_indexes<KMAX>(h1, h2, f.mp, zm, idxs);
#pragma unroll
        for (int j = 0; j < KMAX; ++j)  // every SETBIT in flight at once
            if ((zm >> j) & 1u) old[j] = atomicOr(&f.bm[idxs[j] >> 5], bit_in_word(idxs[j]));
#pragma unroll
        for (int j = 0; j < KMAX; ++j) {
            if (!((zm >> j) & 1u) || !(old[j] & bit_in_word(idxs[j]))) continue;
            // lost the race for a zero bit: another key of the chunk shares it
            const uint64_t key8 = ((uint64_t)f.fid << bb) | idxs[j];
            const unsigned long long mine = ((unsigned long long)key8 << pb) | t;
            uint64_t slot = t8_slot(key8, lgC);
            bool done = false;
            for (uint32_t probes = 0; probes < 64 && !done; ++probes) {
                const unsigned long long o = atomicCAS(&C[slot], ~0ULL, mine);
                if (o == ~0ULL) {
                    if (atomicAdd(&cst->count, 1u) + 1 > (uint32_t)(cmask >> 1)) atomicOr(&cst->overflow, 1u);
                    done = true;
                } else if ((o >> pb) == key8) {
                    if (o > mine) atomicMin(&C[slot], mine);
                    done = true;
                } else {
                    slot = (slot + 1) & cmask;
                }
            }
            if (!done) atomicOr(&cst->overflow, 1u);
        }
    }
}

template <int KLEN, int KMAX>
__global__ __launch_bounds__(256) void k_maddx_claim(KeysDev keys, uint64_t base, uint64_t nchunk,
                                                     const FilterDesc *__restrict__ filt,
                                                     const uint64_t *__restrict__ seg_off, uint32_t nseg,
                                                     const uint32_t *__restrict__ tile_seg0,
                                                     const uint32_t *__restrict__ zmask,
                                                     unsigned long long *__restrict__ C, uint32_t lgC,
                                                     unsigned long long *__restrict__ T, uint32_t lgT, uint32_t bb,
                                                     uint32_t pb, const MaddxState *__restrict__ cst, uint32_t batch,
                                                     const uint32_t *__restrict__ big) {
    if (big && !*big) return;
    const MaddxState cs = *cst;
    if (cs.count == 0 && !cs.overflow) return;  // no shared zero bit: every key with one is new
    const uint64_t pmask = (1ULL << pb) - 1;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; t < nchunk; t += stride) {
        const uint32_t zm = zmask[t];
        if (!zm) continue;
        const uint64_t i = base + t;
        const FilterDesc f = filt[seg_from(seg_off, nseg, tile_seg0[i >> 8], i)];
        uint64_t h1, h2;
        hash_key<KLEN>(keys, i, h1, h2);
        uint32_t idxs[KMAX];
        madd_indexes<KMAX>(h1, h2, f.mp, zm, idxs);
        if (cs.overflow) {  // every zero bit into the full first-setter table
            (void)t8_claim<KMAX>(T, lgT, bb, pb, f.fid, idxs, zm, (uint32_t)t, batch);
            continue;
        }
#pragma unroll
        for (int j = 0; j < KMAX; ++j) {
            if (!((zm >> j) & 1u)) continue;
            const uint64_t key8 = ((uint64_t)f.fid << bb) | idxs[j];
            unsigned long long e;
            const int64_t slot = c_find(C, lgC, pb, key8, &e);
            if (slot >= 0 && (e & pmask) > t) atomicMin(&C[slot], ((unsigned long long)key8 << pb) | t);
        }
    }
}

template <int KLEN, int KMAX>
__global__ __launch_bounds__(256) void k_maddx_reply(KeysDev keys, uint64_t base, uint64_t nchunk,
                                                     const FilterDesc *__restrict__ filt,
                                                     const uint64_t *__restrict__ seg_off, uint32_t nseg,
                                                     const uint32_t *__restrict__ tile_seg0,
                                                     const uint32_t *__restrict__ zmask,
                                                     const unsigned long long *__restrict__ C, uint32_t lgC,
                                                     const unsigned long long *__restrict__ T, uint32_t lgT,
                                                     uint32_t bb, uint32_t pb, const MaddxState *__restrict__ cst,
                                                     uint8_t *__restrict__ out_new,
                                                     unsigned long long *__restrict__ seg_counts,
                                                     const uint32_t *__restrict__ big, uint64_t segmax) {
    if (big && !*big) return;
    const MaddxState cs = *cst;
    const uint64_t pmask = (1ULL << pb) - 1;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    const uint64_t n_up = (nchunk + 63) & ~63ULL;  // whole waves (wave_seg_add)
    for (uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; t < n_up; t += stride) {
        const uint64_t i = base + t;
        uint32_t seg = 0;
        bool in = t < nchunk;
        if (in) {
            seg = seg_from(seg_off, nseg, tile_seg0[i >> 8], i);
            in = !(big && seg_off[seg + 1] - seg_off[seg] <= segmax);  // k_madd_seg answered it
        }
        bool isnew = false;
        if (in) {
            const uint32_t zm = zmask[t];
            if (zm && cs.count == 0 && !cs.overflow) {
                isnew = true;
            } else if (zm) {
                const FilterDesc f = filt[seg];
                uint64_t h1, h2;
                hash_key<KLEN>(keys, i, h1, h2);
                uint32_t idxs[KMAX];
                madd_indexes<KMAX>(h1, h2, f.mp, zm, idxs);
#pragma unroll
                for (int j = 0; j < KMAX; ++j) {
                    if (!((zm >> j) & 1u) || isnew) continue;
                    const uint64_t key8 = ((uint64_t)f.fid << bb) | idxs[j];
                    if (cs.overflow) {
                        isnew = t8_find(T, lgT, pb, key8) == (uint32_t)t;
                    } else {
                        unsigned long long e;
                        isnew = c_find(C, lgC, pb, key8, &e) < 0 || (e & pmask) == t;
                    }
                }
            }
            if (out_new) out_new[i] = isnew;
        }
        if (seg_counts) wave_seg_add(in, seg, isnew ? 1u : 0u, seg_counts);
    }
}

// after an overflowed chunk: T back to EMPTY (its bits were set by k_maddx_set already)
__global__ __launch_bounds__(256) void k_maddx_reset(unsigned long long *__restrict__ T, uint32_t lgT,
                                                     const MaddxState *__restrict__ cst, const uint32_t *__restrict__ big) {
    if (big && !*big) return;
    if (!cst->overflow) return;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t s = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; s < (1ULL << lgT); s += stride)
        if (T[s] != ~0ULL) T[s] = ~0ULL;
}

// ---- multi-tenant add, r05: one workgroup per segment ------------------------------------------
// When every filter of an add batch appears in one segment only, the segments touch disjoint bitmaps,
// so a workgroup that owns a segment owns its bitmap for the whole call: no other workgroup reads or
// writes it, and no memory-side atomic is needed.  The workgroup walks its segment in tiles of TILE
// keys (one per thread): (1) every key's k words are read -- `sc1` loads, served by this XCD's L2,
// which holds the previous tile's stores (the vector L1 is not refreshed by stores); (2) its zero bits
// go into two LDS hash tables: bit -> smallest position of a key meeting it at 0 (CAS + min), word ->
// the OR of the zero bits and the word as read (every key reads the same value: no store of this tile
// has happened yet); (3) every word is written back once with a plain store, old | bits; (4) key t is
// new iff one of its zero bits has t as smallest position.  Tiles run one after another (each sees the
// previous one's bits), so a key is new iff one of its bits was 0 before the batch and no earlier key
// of the batch touches it: M/RedissonBloomFilter.java:104-137 in CommandBatchService order.  Segments
// longer than segmax keys are left to the k_maddx_* chunks (flag `big`).
template <int KLEN, int KMAX>
__global__ __launch_bounds__(256) void k_madd_seg(KeysDev keys, const FilterDesc *__restrict__ filt,
                                                  const uint64_t *__restrict__ seg_off, uint32_t nseg, uint32_t lgs,
                                                  uint32_t tile, uint64_t segmax, uint8_t *__restrict__ out_new,
                                                  unsigned long long *__restrict__ seg_counts,
                                                  uint32_t *__restrict__ big) {
    extern __shared__ unsigned long long s_dyn[];
    const uint32_t S = 1u << lgs, smask = S - 1u;
    unsigned long long *BT = s_dyn;              // bit << 32 | smallest position in the segment; ~0 empty
    uint32_t *WK = (uint32_t *)(BT + S);         // word index; ~0 empty
    uint32_t *WV = WK + S;                       // old word | zero bits
    __shared__ uint32_t s_red[8];
    const uint32_t tid = threadIdx.x, lane = tid & 63u, wave = tid >> 6;
    for (uint32_t sg = blockIdx.x; sg < nseg; sg += gridDim.x) {
        const uint64_t a = seg_off[sg], b = seg_off[sg + 1];
        if (b - a > segmax) {  // uniform: left to the chunked path
            if (tid == 0) atomicOr(big, 1u);
            continue;
        }
        if (b == a) continue;
        const FilterDesc f = filt[sg];
        uint32_t maxidx = 0, nnew = 0;
        for (uint64_t base = a; base < b; base += tile) {
            for (uint32_t q = tid; q < S; q += blockDim.x) {
                BT[q] = ~0ULL;
                WK[q] = ~0u;
                WV[q] = 0u;
            }
            __syncthreads();
            const uint64_t i = base + tid;
            const bool act = tid < tile && i < b;
            const uint32_t pos = (uint32_t)(i - a);
            uint32_t idxs[KMAX], word[KMAX], zm = 0;
            if (act) {
                uint64_t h1, h2;
                hash_key<KLEN>(keys, i, h1, h2);
                uint64_t h = h1;
#pragma unroll
                for (int j = 0; j < KMAX; ++j) {
                    if ((uint32_t)j < f.k) {
                        const uint32_t idx = mod63(h & 0x7fffffffffffffffULL, f.mp);
                        idxs[j] = idx;
                        word[j] = __hip_atomic_load(&f.bm[idx >> 5], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        maxidx = idx > maxidx ? idx : maxidx;
                    }
                    h += (j & 1) ? h1 : h2;
                }
#pragma unroll
                for (int j = 0; j < KMAX; ++j)
                    if ((uint32_t)j < f.k && (word[j] & bit_in_word(idxs[j])) == 0u) zm |= 1u << j;
#pragma unroll
                for (int j = 0; j < KMAX; ++j) {
                    if (!((zm >> j) & 1u)) continue;
                    const unsigned long long mine = ((unsigned long long)idxs[j] << 32) | pos;
                    for (uint32_t q = (idxs[j] * 0x9E3779B1u) >> (32 - lgs);; q = (q + 1u) & smask) {
                        const unsigned long long o = atomicCAS(&BT[q], ~0ULL, mine);
                        if (o == ~0ULL) break;
                        if ((uint32_t)(o >> 32) == idxs[j]) {
                            if (o > mine) atomicMin(&BT[q], mine);
                            break;
                        }
                    }
                    const uint32_t w = idxs[j] >> 5;
                    for (uint32_t q = (w * 0x9E3779B1u) >> (32 - lgs);; q = (q + 1u) & smask) {
                        const uint32_t o = atomicCAS(&WK[q], ~0u, w);
                        if (o == ~0u || o == w) {
                            atomicOr(&WV[q], word[j] | bit_in_word(idxs[j]));
                            break;
                        }
                    }
                }
            }
            __syncthreads();
            for (uint32_t q = tid; q < S; q += blockDim.x) {  // every touched word once, plain stores
                const uint32_t w = WK[q];
                if (w != ~0u) f.bm[w] = WV[q];
            }
            bool isnew = false;
            if (act) {
#pragma unroll
                for (int j = 0; j < KMAX; ++j) {
                    if (!((zm >> j) & 1u) || isnew) continue;
                    for (uint32_t q = (idxs[j] * 0x9E3779B1u) >> (32 - lgs);; q = (q + 1u) & smask) {
                        const unsigned long long o = BT[q];
                        if ((uint32_t)(o >> 32) == idxs[j]) {
                            isnew = (uint32_t)o == pos;
                            break;
                        }
                    }
                }
                if (out_new) out_new[i] = isnew;
            }
            nnew += isnew;
            // this tile's stores reach L2 before the next tile's sc1 loads, and the tables are reused
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();
        }
        // the segment's count and the Redis string length (every SETBIT grows it to idx / 8 + 1)
        uint32_t c = nnew, mx = maxidx;
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) {
            c += __shfl_down(c, off, 64);
            mx = max(mx, (uint32_t)__shfl_down(mx, off, 64));
        }
        if (lane == 0) {
            s_red[wave] = c;
            s_red[4 + wave] = mx;
        }
        __syncthreads();
        if (tid == 0) {
            uint32_t tc = 0, tm = 0;
            for (uint32_t w = 0; w < blockDim.x / 64u; ++w) {
                tc += s_red[w];
                tm = max(tm, s_red[4 + w]);
            }
            if (tc && seg_counts) atomicAdd(&seg_counts[sg], (unsigned long long)tc);
            raise_redis_len(f.redis_len, (unsigned long long)(tm >> 3) + 1ULL);
        }
        __syncthreads();  // s_red reuse
    }
}

template <int KLEN>
static void launch_madd_seg_len(const MaddSegArgs &a, hipStream_t st) {
    const size_t lds = (size_t)(8 + 4 + 4) << a.lgs;
    const dim3 grid(std::min<uint32_t>(a.nseg, 4096));
    if (a.kmax <= 8)
        hipLaunchKernelGGL((k_madd_seg<KLEN, 8>), grid, dim3(256), lds, st, a.keys, a.filt, a.seg_off, a.nseg, a.lgs,
                           a.tile, a.segmax, a.out_new, a.seg_counts, a.big);
    else
        hipLaunchKernelGGL((k_madd_seg<KLEN, 16>), grid, dim3(256), lds, st, a.keys, a.filt, a.seg_off, a.nseg, a.lgs,
                           a.tile, a.segmax, a.out_new, a.seg_counts, a.big);
}

void launch_madd_seg(const MaddSegArgs &a, int klen_fast, hipStream_t st) {
    switch (klen_fast) {
    case 16: launch_madd_seg_len<16>(a, st); break;
    case 32: launch_madd_seg_len<32>(a, st); break;
    case 64: launch_madd_seg_len<64>(a, st); break;
    default: launch_madd_seg_len<0>(a, st); break;
    }
}

static int g_stream_slots = 1;  // rbx_tune("stream_contains_slots"): 0 staged kernel, 1 slot kernel (default)
void set_stream_slots(int v) { g_stream_slots = v; }
// The slot stream kernel at P = 2, Q = 2 (120 VGPRs, four blocks per CU) on 1024 blocks, one
// resident round: C5 9.91 (2048) -> 9.67 ms; shapes 32 / 42 / 24: 10.8 / 11.2 / 11.2 ms
// (profiles/r03/r03u_c5sweep_qshape_qgrid.jsonl).
static unsigned g_stream_qgrid = 1024;
void set_stream_qgrid(int v) { g_stream_qgrid = (unsigned)v; }
// k_stream_contains runs best at four 256-thread blocks per CU (4 waves/SIMD): the Zipf-hot
// tenants' bitmaps live in L2, and more resident waves interleave more tenants.  Its registers
// (93 VGPRs since the r02 hash) would admit five, so the launch reserves 33,000 bytes of dynamic
// LDS per block (four fit in 160 KiB).  C5, same box: 11.28 -> 10.99 ms per 1e8 commands; three
// blocks per CU: 0.66 ms per chunk vs 0.545 (profiles/r02/r02ze_c5_occupancy.txt).
// rbx_tune("stream_contains_lds") overrides the bytes (0: registers decide).
static int g_stream_lds = 33000;
void set_stream_contains_lds(int v) { g_stream_lds = v; }
// k_stream_probe8: 1 (default) every zero bit's home-slot CAS issued before any is waited on, 0 one
// claim after another (rbx_tune "stream_probe_batch")
static uint32_t g_probe8_batch = 1;
void set_stream_probe_batch(int v) { g_probe8_batch = (uint32_t)v; }
// DIAGNOSTICS ONLY (timing; answers become wrong): 1 = the stream contains skip the first-setter
// lookups, 2 = the walk ORs bits with plain read-modify-writes, 4 = the walk writes no owner flags,
// 8 = the probe makes no claims
static uint32_t g_stream_diag = 0;
void set_stream_diag(int v) { g_stream_diag = (uint32_t)v; }
// r05 (rbx_tune "stream_owner"): 1 (default) replies from the first claims' slots (k_stream_final8),
// 0 the r04 owner flags written by the walk (k_stream_final)
static int g_stream_owner = 1;
void set_stream_owner(int v) { g_stream_owner = v; }
// r05 (rbx_tune "stream_lookup_rounds"): 1 (default) the slot contains kernel issues a first-setter
// lookup as one more round of its slot (in flight with the other slots' gathers), 0 inline
static uint32_t g_stream_lookup_rounds = 1;
void set_stream_lookup_rounds(int v) { g_stream_lookup_rounds = (uint32_t)v; }
// rbx_tune "walk_reset_all": bit 0 = the stream's walk rewrites every pair (whole lines), bit 1 =
// the multi-tenant add's walk does
static uint32_t g_walk_reset_all = 0;
void set_walk_reset_all(int v) { g_walk_reset_all = (uint32_t)v; }
// rbx_tune "stream_final_grid": k_stream_final8's blocks.  Each block adds its new-add count to ONE counter,
// and same-address atomics serialise: 2048 / 512 / 256 blocks 39.3 / 28.3 / 35.6 us per C5 chunk (r05as).
static unsigned g_final8_grid = 512;
void set_stream_final_grid(int v) { g_final8_grid = (unsigned)v; }

template <int KLEN, int KMAX>
static void launch_stream_chunk_k(const StreamChunkArgs &a, hipStream_t st) {
    const unsigned grid = grid_for(a.nchunk, kMaxGrid);
    const unsigned cgrid = (unsigned)((a.nchunk + kCompactBlock - 1) / kCompactBlock);
    hipLaunchKernelGGL(k_stream_compact, dim3(cgrid ? cgrid : 1), dim3(256), 0, st, a.op, a.base, a.nchunk, a.adds,
                       a.nadds);
    const bool own8 = a.t8 && g_stream_owner == 1;  // r05: replies from the first claims, no flags
    if (a.t8)
        hipLaunchKernelGGL((k_stream_probe8<KLEN, KMAX>), dim3(grid), dim3(256), 0, st, a.keys, a.base, a.adds, a.nadds,
                           a.filt, a.kf, a.t8, a.bb, a.pb, a.tkmax, a.prefilter, a.pshift,
                           (g_stream_diag & 8) ? 2u : g_probe8_batch, own8 ? a.zmask : nullptr,
                           own8 ? a.fslot : nullptr);
    else
        hipLaunchKernelGGL((k_stream_probe<KLEN, KMAX>), dim3(grid), dim3(256), 0, st, a.keys, a.base, a.adds, a.nadds,
                           a.filt, a.kf, a.table, a.log2cap, a.epoch, a.zmask, a.prefilter, a.pshift);
    if (a.t8 && a.prefilter && a.pshift == 0)  // occupancy filter of the 8-byte table
        hipLaunchKernelGGL(k_stream_occ, dim3(kMaxGrid), dim3(256), 0, st, a.t8, a.nadds, a.tkmax, a.prefilter);
    if (g_stream_slots)
        hipLaunchKernelGGL((k_stream_contains_q<KLEN, 2, 2>), dim3(std::min(grid, g_stream_qgrid)), dim3(256), 0, st,
                           a.keys, a.base, a.nchunk, a.pdesc, a.kf, a.op, a.table, a.log2cap, a.epoch, a.prefilter,
                           a.pshift, a.out, a.counts, a.t8, a.bb, a.pb, a.tkmax, a.nadds, g_stream_diag,
                           g_stream_lookup_rounds);
    else
        hipLaunchKernelGGL((k_stream_contains<KLEN, KMAX>), dim3(grid), dim3(256), g_stream_lds, st, a.keys, a.base, a.nchunk,
                           a.filt, a.kf, a.op, a.table, a.log2cap, a.epoch, a.prefilter, a.pshift, a.out, a.counts,
                           a.t8, a.bb, a.pb, a.tkmax, a.nadds);
    if (own8) {
        hipLaunchKernelGGL((k_stream_final8<KLEN, KMAX>), dim3(std::min(grid, g_final8_grid)), dim3(256), 0, st, a.keys,
                           a.base, a.adds, a.nadds,
                           a.filt, a.kf, a.t8, a.bb, a.pb, a.tkmax, a.zmask, a.fslot, a.out, a.counts);
        hipLaunchKernelGGL(k_stream_walk, dim3(kMaxGrid), dim3(256), 0, st, a.t8, a.nadds, a.tkmax, a.bb, a.pb, a.fid_bm,
                           (uint8_t *)nullptr, g_stream_diag, g_walk_reset_all & 1u);
    } else if (a.t8) {
        hipLaunchKernelGGL(k_stream_walk, dim3(kMaxGrid), dim3(256), 0, st, a.t8, a.nadds, a.tkmax, a.bb, a.pb, a.fid_bm,
                           a.flag, g_stream_diag, g_walk_reset_all & 1u);
        hipLaunchKernelGGL(k_stream_final, dim3(grid), dim3(256), 0, st, a.base, a.adds, a.nadds, a.flag, a.out, a.counts);
    } else {
        hipLaunchKernelGGL((k_stream_commit<KLEN, KMAX>), dim3(grid), dim3(256), 0, st, a.keys, a.base, a.adds, a.nadds,
                           a.filt, a.kf, a.table, a.log2cap, a.epoch, a.zmask, a.out, a.counts);
    }
}

template <int KLEN>
static void launch_stream_chunk_len(const StreamChunkArgs &a, hipStream_t st) {
    if (a.kmax <= 8) launch_stream_chunk_k<KLEN, 8>(a, st);
    else if (a.kmax <= 16) launch_stream_chunk_k<KLEN, 16>(a, st);
    else launch_stream_chunk_k<KLEN, 32>(a, st);
}

template <int KLEN, int KMAX>
static void launch_madd8_chunk_k(const MaddChunkArgs &a, hipStream_t st) {
    const unsigned grid = grid_for(a.nchunk, kMaxGrid);
    hipLaunchKernelGGL((k_madd_probe8<KLEN, KMAX>), dim3(grid), dim3(256), 0, st, a.keys, a.base, a.nchunk, a.filt,
                       a.seg_off, a.nseg, a.tile_seg0, a.t8, a.lg, a.bb, a.pb, g_probe8_batch, a.zmask, a.fslot);
    hipLaunchKernelGGL((k_madd_final8<KLEN, KMAX>), dim3(grid), dim3(256), 0, st, a.keys, a.base, a.nchunk, a.filt,
                       a.seg_off, a.nseg, a.tile_seg0, a.t8, a.lg, a.bb, a.pb, a.zmask, a.fslot, a.out_new,
                       a.seg_counts);
    hipLaunchKernelGGL(k_stream_walk, dim3(kMaxGrid), dim3(256), 0, st, a.t8, (const uint32_t *)nullptr, a.lg, a.bb,
                       a.pb, a.fid_bm, (uint8_t *)nullptr, 0u, (g_walk_reset_all >> 1) & 1u);
}

template <int KLEN, int KMAX>
static void launch_maddx_chunk_k(const MaddChunkArgs &a, hipStream_t st) {
    const unsigned grid = grid_for(std::max<uint64_t>(a.nchunk, 1ULL << a.lgC), kMaxGrid);
    hipLaunchKernelGGL((k_maddx_gather<KLEN, KMAX>), dim3(grid), dim3(256), 0, st, a.keys, a.base, a.nchunk, a.filt,
                       a.seg_off, a.nseg, a.tile_seg0, a.zmask, a.c8, a.lgC, a.cst, a.big, a.segmax);
    hipLaunchKernelGGL((k_maddx_set<KLEN, KMAX>), dim3(grid), dim3(256), 0, st, a.keys, a.base, a.nchunk, a.filt,
                       a.seg_off, a.nseg, a.tile_seg0, a.zmask, a.c8, a.lgC, a.bb, a.pb, a.cst, a.big);
    hipLaunchKernelGGL((k_maddx_claim<KLEN, KMAX>), dim3(grid), dim3(256), 0, st, a.keys, a.base, a.nchunk, a.filt,
                       a.seg_off, a.nseg, a.tile_seg0, a.zmask, a.c8, a.lgC, a.t8, a.lg, a.bb, a.pb, a.cst,
                       g_probe8_batch, a.big);
    hipLaunchKernelGGL((k_maddx_reply<KLEN, KMAX>), dim3(grid), dim3(256), 0, st, a.keys, a.base, a.nchunk, a.filt,
                       a.seg_off, a.nseg, a.tile_seg0, a.zmask, a.c8, a.lgC, a.t8, a.lg, a.bb, a.pb, a.cst, a.out_new,
                       a.seg_counts, a.big, a.segmax);
    hipLaunchKernelGGL(k_maddx_reset, dim3(kMaxGrid), dim3(256), 0, st, a.t8, a.lg, a.cst, a.big);
}

template <int KLEN>
static void launch_madd8_chunk_len(const MaddChunkArgs &a, hipStream_t st) {
    if (a.c8) {
        if (a.kmax <= 8) launch_maddx_chunk_k<KLEN, 8>(a, st);
        else if (a.kmax <= 16) launch_maddx_chunk_k<KLEN, 16>(a, st);
        else launch_maddx_chunk_k<KLEN, 32>(a, st);
        return;
    }
    if (a.kmax <= 8) launch_madd8_chunk_k<KLEN, 8>(a, st);
    else if (a.kmax <= 16) launch_madd8_chunk_k<KLEN, 16>(a, st);
    else launch_madd8_chunk_k<KLEN, 32>(a, st);
}

void launch_madd8_chunk(const MaddChunkArgs &a, int klen_fast, hipStream_t st) {
    switch (klen_fast) {
    case 16: launch_madd8_chunk_len<16>(a, st); break;
    case 32: launch_madd8_chunk_len<32>(a, st); break;
    case 64: launch_madd8_chunk_len<64>(a, st); break;
    default: launch_madd8_chunk_len<0>(a, st); break;
    }
}

void launch_stream_chunk(const StreamChunkArgs &a, int klen_fast, hipStream_t st) {
    switch (klen_fast) {
    case 16: launch_stream_chunk_len<16>(a, st); break;
    case 32: launch_stream_chunk_len<32>(a, st); break;
    case 64: launch_stream_chunk_len<64>(a, st); break;
    default: launch_stream_chunk_len<0>(a, st); break;
    }
}

}  // namespace rbx
