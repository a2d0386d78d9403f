// bucket_common.h -- helpers shared by the region-partitioned Bloom pipelines
// (contains_partitioned.hip, add_partitioned.hip): key hashing dispatch and the LDS bucket scan.
#pragma once

#include "rbx_kernels.h"

namespace rbx {

// Stores of the partition passes' runs.  Experiment builds (-DRBX_RUN_STORES_PLAIN, tools/_ab/)
// use plain stores instead, which keep the line in the XCD's L2 where partial lines written by
// different workgroups can merge before write-back.
template <class T> __device__ __forceinline__ void run_store(T v, T *p) {
#ifdef RBX_RUN_STORES_PLAIN
    *p = v;
#else
    __builtin_nontemporal_store(v, p);
#endif
}

// HighwayHash128 of key i (Hash.hash128, M/misc/Hash.java:53-74): 16/32/64-byte fast path or
// the generic any-length path
template <int KLEN>
__device__ __forceinline__ void bk_hash(const KeysDev &keys, uint64_t i, uint64_t &h1, uint64_t &h2) {
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

// exclusive scan of cnt[0..nb) (nb <= 128) by wave 0 into start[] and pos[]
__device__ __forceinline__ void bk_scan128(const uint32_t *cnt, uint32_t nb, uint32_t *start, uint32_t *pos,
                                           uint32_t lane = threadIdx.x) {
    const uint32_t a = 2 * lane < nb ? cnt[2 * lane] : 0u;
    const uint32_t b = 2 * lane + 1 < nb ? cnt[2 * lane + 1] : 0u;
    uint32_t x = a + b;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const uint32_t y = __shfl_up(x, off, 64);
        if ((int)lane >= off) x += y;
    }
    const uint32_t ex = x - a - b;
    if (2 * lane < nb) start[2 * lane] = pos[2 * lane] = ex;
    if (2 * lane + 1 < nb) start[2 * lane + 1] = pos[2 * lane + 1] = ex + a;
}

// exclusive scan of cnt[j] + car[j] (j < nb <= 128) by wave 0: start[j] = the bucket's image
// offset (its carried entries first), pos[j] = start[j] + car[j] (where its new entries go)
__device__ __forceinline__ void bk_scan128c(const uint32_t *cnt, const uint32_t *car, uint32_t nb, uint32_t *start,
                                            uint32_t *pos) {
    const uint32_t lane = threadIdx.x;
    const uint32_t ca = 2 * lane < nb ? car[2 * lane] : 0u, cb = 2 * lane + 1 < nb ? car[2 * lane + 1] : 0u;
    const uint32_t a = (2 * lane < nb ? cnt[2 * lane] : 0u) + ca;
    const uint32_t b = (2 * lane + 1 < nb ? cnt[2 * lane + 1] : 0u) + cb;
    uint32_t x = a + b;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const uint32_t y = __shfl_up(x, off, 64);
        if ((int)lane >= off) x += y;
    }
    const uint32_t ex = x - a - b;
    if (2 * lane < nb) {
        start[2 * lane] = ex;
        pos[2 * lane] = ex + ca;
    }
    if (2 * lane + 1 < nb) {
        start[2 * lane + 1] = ex + a;
        pos[2 * lane + 1] = ex + a + cb;
    }
}

// bk_scan128c with every bucket's extent rounded up to a multiple of `al` slots (a power of two):
// bucket starts are then aligned to whole output lines, so the 64-slot windows of a slot-linear
// store never split a line between two store instructions
__device__ __forceinline__ void bk_scan128c_al(const uint32_t *cnt, const uint32_t *car, uint32_t nb, uint32_t al,
                                               uint32_t *start, uint32_t *pos) {
    const uint32_t lane = threadIdx.x;
    const uint32_t ca = 2 * lane < nb ? car[2 * lane] : 0u, cb = 2 * lane + 1 < nb ? car[2 * lane + 1] : 0u;
    const uint32_t a = ((2 * lane < nb ? cnt[2 * lane] : 0u) + ca + al - 1) & ~(al - 1);
    const uint32_t b = ((2 * lane + 1 < nb ? cnt[2 * lane + 1] : 0u) + cb + al - 1) & ~(al - 1);
    uint32_t x = a + b;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const uint32_t y = __shfl_up(x, off, 64);
        if ((int)lane >= off) x += y;
    }
    const uint32_t ex = x - a - b;
    if (2 * lane < nb) {
        start[2 * lane] = ex;
        pos[2 * lane] = ex + ca;
    }
    if (2 * lane + 1 < nb) {
        start[2 * lane + 1] = ex + a;
        pos[2 * lane + 1] = ex + a + cb;
    }
}

// the same for nb <= 256 (four buckets per lane)
__device__ __forceinline__ void bk_scan256(const uint32_t *cnt, uint32_t nb, uint32_t *start, uint32_t *pos) {
    const uint32_t lane = threadIdx.x;
    uint32_t v[4], s = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        v[j] = 4 * lane + j < nb ? cnt[4 * lane + j] : 0u;
        s += v[j];
    }
    uint32_t x = s;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const uint32_t y = __shfl_up(x, off, 64);
        if ((int)lane >= off) x += y;
    }
    uint32_t ex = x - s;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        if (4 * lane + j < nb) start[4 * lane + j] = pos[4 * lane + j] = ex;
        ex += v[j];
    }
}

// Phase timer for A/B diagnostics (template-gated: the production instantiation carries none of
// it): s_memtime deltas of the block's wave 0 summed per phase, added by thread 0 to dst[0..N).
template <bool ON, int N = 8> struct PhaseStamps {
    uint64_t t = 0, acc[N] = {};
    __device__ __forceinline__ void start() {
        if constexpr (ON) t = __builtin_amdgcn_s_memtime();
    }
    __device__ __forceinline__ void mark(int i) {
        if constexpr (ON) {
            const uint64_t n = __builtin_amdgcn_s_memtime();
            acc[i] += n - t;
            t = n;
        }
    }
    __device__ __forceinline__ void flush(unsigned long long *dst) {
        if constexpr (ON) {
            if (threadIdx.x == 0)
                for (int i = 0; i < N; ++i) atomicAdd(dst + i, (unsigned long long)acc[i]);
        }
    }
};

}  // namespace rbx
