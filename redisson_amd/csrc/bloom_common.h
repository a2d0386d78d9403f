// bloom_common.h -- device helpers shared by bloom_kernels.hip (contains, single-filter add, wide
// filters) and stream_kernels.hip (the ordered stream and the multi-tenant adds): key hashing,
// block / wave reductions, segment search, the 16-byte first-setter table, the launch grid.
#pragma once
#include "rbx_kernels.h"

namespace rbx {

// ---------------------------------------------------------------------------------
// key hashing dispatch
// ---------------------------------------------------------------------------------
template <int KLEN>
__device__ __forceinline__ void hash_key(const KeysDev &keys, uint64_t i, uint64_t &h1, uint64_t &h2) {
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

__device__ __forceinline__ void block_add_u64(uint64_t v, unsigned long long *dst) {
    // wave reduce, then one atomic per wave-leader through LDS
    __shared__ unsigned long long s_part[8];
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_down(v, off, 64);
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    if (lane == 0) s_part[wid] = v;
    __syncthreads();
    if (threadIdx.x == 0) {
        unsigned long long t = 0;
        const int nw = (blockDim.x + 63) >> 6;
        for (int w = 0; w < nw; ++w) t += s_part[w];
        if (t) atomicAdd(dst, t);
    }
}

// the block's total stored (plain store, thread 0) at *dst -- a per-block partial that one small kernel
// adds up afterwards (k_add_partials): same-address atomics from every block of a short kernel serialise
// at its end (~140 per us measured on the stream's final kernel, r05as)
__device__ __forceinline__ void block_store_u64(uint64_t v, unsigned long long *dst) {
    __shared__ unsigned long long s_part[8];
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_down(v, off, 64);
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    if (lane == 0) s_part[wid] = v;
    __syncthreads();
    if (threadIdx.x == 0) {
        unsigned long long t = 0;
        const int nw = (blockDim.x + 63) >> 6;
        for (int w = 0; w < nw; ++w) t += s_part[w];
        *dst = t;
    }
}

__device__ __forceinline__ uint64_t wave_max_u64(uint64_t v) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        const uint64_t o = __shfl_down(v, off, 64);
        v = o > v ? o : v;
    }
    return v;
}

// The Redis string length only grows; a relaxed read first keeps the atomic off the
// hot path once the length has saturated (a stale read only costs an extra atomic).
__device__ __forceinline__ void raise_redis_len(unsigned long long *len, unsigned long long v) {
    if (v > __hip_atomic_load(len, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) atomicMax(len, v);
}

// Adds val into counts[seg] with one atomic per distinct segment of the wave.
__device__ __forceinline__ void wave_seg_add(bool active, uint32_t seg, uint32_t val,
                                             unsigned long long *counts) {
    uint64_t pending = __ballot(active);
    while (pending) {
        const int leader = __ffsll((unsigned long long)pending) - 1;
        const uint32_t s = __shfl(seg, leader, 64);
        const bool mine = active && seg == s;
        const uint64_t grp = __ballot(mine);
        const uint64_t hits = __ballot(mine && val);
        if ((threadIdx.x & 63) == (unsigned)leader && hits) atomicAdd(&counts[s], (unsigned long long)__popcll(hits));
        pending &= ~grp;
    }
}

// Multi-tenant: segment s = keys [seg_off[s], seg_off[s+1]) against filters[s].
// A block handles 256 consecutive keys; their segments are found by one global
// binary search (lane 0) plus an LDS search over the <= 257 segment starts.
__device__ __forceinline__ uint32_t upper_seg(const uint64_t *off, uint32_t nseg, uint64_t key) {
    // largest s in [0, nseg) with off[s] <= key   (off[0] = 0 <= key)
    uint32_t lo = 0, hi = nseg;  // invariant off[lo] <= key < off[hi]
    while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (off[mid] <= key) lo = mid;
        else hi = mid;
    }
    return lo;
}

// segment of key i, scanning forward from a lower bound s (off[s] <= i)
__device__ __forceinline__ uint32_t seg_from(const uint64_t *__restrict__ off, uint32_t nseg, uint32_t s,
                                             uint64_t i) {
    while (s + 1 < nseg && off[s + 1] <= i) ++s;
    return s;
}

// ---------------------------------------------------------------------------------
// add: first-setter table
// ---------------------------------------------------------------------------------
__device__ __forceinline__ uint64_t ht_slot(uint64_t keypart, uint32_t log2cap) {
    return (keypart * 0x9E3779B97F4A7C15ULL) >> (64 - log2cap);
}

// Inserts (keypart, id); the entry's idw ends as min over ids of this epoch.
__device__ __forceinline__ void ht_insert(HTEntry *__restrict__ T, uint32_t log2cap, uint32_t epoch,
                                          uint64_t keypart, uint32_t id) {
    const uint64_t mask = (1ULL << log2cap) - 1;
    const uint64_t mytag = ((uint64_t)epoch << 56) | keypart;
    const unsigned long long myidw = ((unsigned long long)(254u - epoch) << 32) | id;
    uint64_t slot = ht_slot(keypart, log2cap);
    for (uint64_t probes = 0; probes <= mask; ++probes) {
        unsigned long long cur = __hip_atomic_load((unsigned long long *)&T[slot].tag, __ATOMIC_RELAXED,
                                                   __HIP_MEMORY_SCOPE_AGENT);
        for (;;) {
            if (cur == mytag) {
                atomicMin((unsigned long long *)&T[slot].idw, myidw);
                return;
            }
            if ((uint32_t)(cur >> 56) == epoch) break;  // occupied by another key this epoch
            const unsigned long long prev = atomicCAS((unsigned long long *)&T[slot].tag, cur, mytag);
            if (prev == cur) {
                atomicMin((unsigned long long *)&T[slot].idw, myidw);
                return;
            }
            cur = prev;  // re-examine this slot
        }
        slot = (slot + 1) & mask;
    }
}

// Returns the min id recorded for keypart (the entry must exist).
__device__ __forceinline__ uint32_t ht_owner(const HTEntry *__restrict__ T, uint32_t log2cap, uint32_t epoch,
                                             uint64_t keypart) {
    const uint64_t mask = (1ULL << log2cap) - 1;
    const uint64_t mytag = ((uint64_t)epoch << 56) | keypart;
    uint64_t slot = ht_slot(keypart, log2cap);
    for (uint64_t probes = 0; probes <= mask; ++probes) {
        const HTEntry e = T[slot];
        if (e.tag == mytag) return (uint32_t)e.idw;
        slot = (slot + 1) & mask;
    }
    return 0xffffffffu;
}

static inline unsigned grid_for(uint64_t n, unsigned cap) {
    uint64_t g = (n + 255) / 256;
    if (g == 0) g = 1;
    return (unsigned)(g < cap ? g : cap);
}

}  // namespace rbx
