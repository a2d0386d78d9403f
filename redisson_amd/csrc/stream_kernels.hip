// stream_kernels.hip -- the ordered mixed contains/add stream (C5, rbx_bloom_stream[_dev]) and the
// multi-tenant add (rbx_bloom_add_multi[_dev]) on gfx950; split from bloom_kernels.hip in r05 so
// the two compile in parallel.  Semantics: M/RedissonBloomFilter.java:99-137,198-201 with
// M/command/CommandBatchService.java:115-134's in-order execution.
// M/ = /root/reference/redisson/src/main/java/org/redisson/
#include "bloom_common.h"

#include <atomic>

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
// (first-setter table of add positions per initially-zero bit), then the contains -- a zero bit counts
// as set iff an add at an earlier position of the chunk claimed it -- then commit the adds.  Earlier
// chunks are committed before later ones probe, so chunking keeps the order.  The add list is
// unordered: owners are resolved by atomicMin.  (r03-r05 also carried a (fid, bit) prefilter and a
// table-occupancy bitmap in front of the lookups; both measured slower on the fresh stream and were
// removed in r06: profiles/r04/r04g_c5_fresh_prefilter.jsonl, r04o_c5_occupancy_rejected.jsonl.)

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
                                                      uint32_t log2cap, uint32_t epoch, uint32_t *__restrict__ zmask) {
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
            }
        }
        raise_redis_len(f.redis_len, (unsigned long long)(maxidx >> 3) + 1ULL);
        zmask[a] = zm;
    }
}

// The chunk's contains with the per-lane slot schedule of k_bloom_contains_q (§3.1b): one bit per
// key per round trip, P keys in flight per lane.  A wave's queue holds only the chunk's contains
// commands (ballot-compacted while the wave hashes a 64*Q-command range), so add commands cost
// no lane time.  (The r02 staged kernel, k_stream_contains, was removed in r06.)
template <int KLEN, int P, int Q>
__global__ __launch_bounds__(256) void k_stream_contains_q(KeysDev keys, uint64_t base, uint64_t nchunk,
                                                           const ProbeDesc *__restrict__ pdesc,
                                                           const uint32_t *__restrict__ kf,
                                                           const uint8_t *__restrict__ op,
                                                           const HTEntry *__restrict__ T, uint32_t log2cap,
                                                           uint32_t epoch, uint8_t *__restrict__ out,
                                                           unsigned long long *__restrict__ counts,
                                                           const unsigned long long *__restrict__ T8, uint32_t bb,
                                                           uint32_t pb, uint32_t kmax,
                                                           const uint32_t *__restrict__ nadds, uint32_t diag) {
    if (!kDiag) diag = 0;  // wrong-answer diagnostics exist in the profiling build only (rbx_kernels.h)
    constexpr uint32_t RANGE = 64 * Q, WAVES = 4;
    const uint32_t lg8 = T8 ? t8_log2(*nadds, kmax) : 0;
    // r05: with the 8-byte table a clear bit's first-setter lookup is a round of its own: the slot's
    // next load is the table entry instead of a bitmap word, in flight with the other slots' gathers
    // (inline, each lookup chain stalled the lane's whole round).  DIAG bit 1: no lookups.
    const bool rounds = T8 && !(diag & 1);
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
                    if (clear && !T8 && !(diag & 1))  // set by an earlier add of this chunk (16-byte table)?
                        clear = !(ht_find(T, log2cap, epoch, ((uint64_t)sfid[s] << 32) | sidx[s]) < st[s]);
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
                                                       uint32_t bb, uint32_t pb, uint32_t kmax, uint32_t batch,
                                                       uint32_t *__restrict__ zmask, uint32_t *__restrict__ fslot) {
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
        if (kDiag && batch == 2) zm = 0;  // DIAGNOSTIC: no claims
        // the slot of the first zero bit's entry: k_stream_final8 decides the reply from it
        const uint32_t fs = t8_claim<KMAX>(T, lg, bb, pb, f.fid, idxs, zm, t, batch);
        zmask[a] = zm;
        fslot[a] = fs;
        raise_redis_len(f.redis_len, (unsigned long long)(maxidx >> 3) + 1ULL);
    }
}

// every entry: OR its bit into its bitmap and empty the slot (two entries per lane).  (r04 also wrote an
// owner flag per entry for a final pass, and had a whole-line reset variant; both removed in r06.)
__global__ __launch_bounds__(256) void k_stream_walk(unsigned long long *__restrict__ T, const uint32_t *__restrict__ nadds,
                                                     uint32_t kmax, uint32_t bb, uint32_t pb,
                                                     uint32_t *const *__restrict__ fid_bm) {
    const uint32_t lg = nadds ? t8_log2(*nadds, kmax) : kmax;  // no count: kmax carries lg itself
    const uint64_t n2 = (1ULL << lg) / 2;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    const uint64_t bmask = (1ULL << bb) - 1;
    using u64x2 = unsigned long long __attribute__((ext_vector_type(2)));
    for (uint64_t q = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; q < n2; q += stride) {
        u64x2 e = ((const u64x2 *)T)[q];
        if ((e.x & e.y) == ~0ULL) continue;  // both empty
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const unsigned long long v = h ? e.y : e.x;
            if (v == ~0ULL) continue;
            const uint64_t key = v >> pb;
            const uint32_t bit = (uint32_t)(key & bmask);
            atomicOr(&fid_bm[key >> bb][bit >> 5], bit_in_word(bit));
        }
        ((u64x2 *)T)[q] = u64x2{~0ULL, ~0ULL};
    }
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

// The slot stream kernel at P = 2, Q = 2 (120 VGPRs, four blocks per CU) on 1024 blocks, one
// resident round: C5 9.91 (2048) -> 9.67 ms; shapes 32 / 42 / 24: 10.8 / 11.2 / 11.2 ms
// (profiles/r03/r03u_c5sweep_qshape_qgrid.jsonl).  rbx_tune "stream_qgrid".
static std::atomic<unsigned> g_stream_qgrid{1024};
void set_stream_qgrid(int v) { g_stream_qgrid = (unsigned)v; }
// DIAGNOSTICS ONLY, profiling build (kDiag; answers become wrong): 1 = the stream contains skip the
// first-setter lookups, 8 = the probe makes no claims
static std::atomic<uint32_t> g_stream_diag{0};
void set_stream_diag(int v) { g_stream_diag = (uint32_t)v; }
// rbx_tune "stream_final_grid": k_stream_final8's blocks.  Each block adds its new-add count to ONE counter,
// and same-address atomics serialise: 2048 / 512 / 256 blocks 39.3 / 28.3 / 35.6 us per C5 chunk (r05as).
static std::atomic<unsigned> g_final8_grid{512};
void set_stream_final_grid(int v) { g_final8_grid = (unsigned)v; }

// One chunk: compact -> probe (8-byte claims, or the 16-byte table when (fid, bit) does not fit 41 bits)
// -> slot contains -> replies from the first claims (k_stream_final8) + walk, or the 16-byte commit.
template <int KLEN, int KMAX>
static void launch_stream_chunk_k(const StreamChunkArgs &a, hipStream_t st) {
    const unsigned grid = grid_for(a.nchunk, kMaxGrid);
    const unsigned cgrid = (unsigned)((a.nchunk + kCompactBlock - 1) / kCompactBlock);
    const uint32_t diag = kDiag ? g_stream_diag.load() : 0u;
    hipLaunchKernelGGL(k_stream_compact, dim3(cgrid ? cgrid : 1), dim3(256), 0, st, a.op, a.base, a.nchunk, a.adds,
                       a.nadds);
    if (a.t8)
        hipLaunchKernelGGL((k_stream_probe8<KLEN, KMAX>), dim3(grid), dim3(256), 0, st, a.keys, a.base, a.adds, a.nadds,
                           a.filt, a.kf, a.t8, a.bb, a.pb, a.tkmax, (diag & 8) ? 2u : 1u, a.zmask, a.fslot);
    else
        hipLaunchKernelGGL((k_stream_probe<KLEN, KMAX>), dim3(grid), dim3(256), 0, st, a.keys, a.base, a.adds, a.nadds,
                           a.filt, a.kf, a.table, a.log2cap, a.epoch, a.zmask);
    hipLaunchKernelGGL((k_stream_contains_q<KLEN, 2, 2>), dim3(std::min(grid, g_stream_qgrid.load())), dim3(256), 0, st,
                       a.keys, a.base, a.nchunk, a.pdesc, a.kf, a.op, a.table, a.log2cap, a.epoch, a.out, a.counts,
                       a.t8, a.bb, a.pb, a.tkmax, a.nadds, diag);
    if (a.t8) {
        hipLaunchKernelGGL((k_stream_final8<KLEN, KMAX>), dim3(std::min(grid, g_final8_grid.load())), dim3(256), 0, st,
                           a.keys, a.base, a.adds, a.nadds, a.filt, a.kf, a.t8, a.bb, a.pb, a.tkmax, a.zmask, a.fslot,
                           a.out, a.counts);
        hipLaunchKernelGGL(k_stream_walk, dim3(kMaxGrid), dim3(256), 0, st, a.t8, a.nadds, a.tkmax, a.bb, a.pb, a.fid_bm);
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
static void launch_maddx_chunk_k(const MaddChunkArgs &a, hipStream_t st) {
    const unsigned grid = grid_for(std::max<uint64_t>(a.nchunk, 1ULL << a.lgC), kMaxGrid);
    hipLaunchKernelGGL((k_maddx_gather<KLEN, KMAX>), dim3(grid), dim3(256), 0, st, a.keys, a.base, a.nchunk, a.filt,
                       a.seg_off, a.nseg, a.tile_seg0, a.zmask, a.c8, a.lgC, a.cst, a.big, a.segmax);
    hipLaunchKernelGGL((k_maddx_set<KLEN, KMAX>), dim3(grid), dim3(256), 0, st, a.keys, a.base, a.nchunk, a.filt,
                       a.seg_off, a.nseg, a.tile_seg0, a.zmask, a.c8, a.lgC, a.bb, a.pb, a.cst, a.big);
    hipLaunchKernelGGL((k_maddx_claim<KLEN, KMAX>), dim3(grid), dim3(256), 0, st, a.keys, a.base, a.nchunk, a.filt,
                       a.seg_off, a.nseg, a.tile_seg0, a.zmask, a.c8, a.lgC, a.t8, a.lg, a.bb, a.pb, a.cst, 1u,
                       a.big);
    hipLaunchKernelGGL((k_maddx_reply<KLEN, KMAX>), dim3(grid), dim3(256), 0, st, a.keys, a.base, a.nchunk, a.filt,
                       a.seg_off, a.nseg, a.tile_seg0, a.zmask, a.c8, a.lgC, a.t8, a.lg, a.bb, a.pb, a.cst, a.out_new,
                       a.seg_counts, a.big, a.segmax);
    hipLaunchKernelGGL(k_maddx_reset, dim3(kMaxGrid), dim3(256), 0, st, a.t8, a.lg, a.cst, a.big);
}

template <int KLEN>
static void launch_madd8_chunk_len(const MaddChunkArgs &a, hipStream_t st) {
    if (a.kmax <= 8) launch_maddx_chunk_k<KLEN, 8>(a, st);
    else if (a.kmax <= 16) launch_maddx_chunk_k<KLEN, 16>(a, st);
    else launch_maddx_chunk_k<KLEN, 32>(a, st);
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
