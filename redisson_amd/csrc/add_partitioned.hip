// add_partitioned.hip -- RBloomFilter.add(Collection) for one large filter
// (M/RedissonBloomFilter.java:104-137) with first-setter resolution in LDS.
//
// The reference executes n*k SETBITs in submission order (CommandBatchService.java:115-134,
// :335, :600-602) and counts a key as new iff one of its replies was 0.  So key i is new iff
// some bit b of key i was 0 before the batch and i is the smallest key id touching b.  The
// table path (bloom_kernels.hip) resolves that with ~28 random memory requests per key (gathers,
// CAS into a first-setter table, lookups, atomicOr).  Here every (bit, key) pair is routed
// through two streaming radix passes to its 2^16-bit region, and one workgroup per region resolves
// the first setters in LDS:
//   A  k_ba_stage1  : hash, all k pairs per key -> <= 256 level-1 buckets (kBaSub sub-partitions each)
//   B  k_ba_rebucket: level 1 -> regions (idx >> 16), fan-out <= 256
//   C  k_ba_region  : region bitmap + met-once / met-again bitsets + a collision table in LDS;
//                     owners set their bits; the bitmap is written back
//   D  k_ba_keys_rec: owner records -> new_bits
//   E  k_ba_final   : out_new bytes and the count (non-owner counters decoded here, r05)
// Reporting new keys: a key is new iff at least one of its k pairs owns its bit.  k_ba_mode
// samples the bitmap's fill per chunk and picks (rbx_tune "add_records" can force one):
//   - below a fill of 3/32 each NON-OWNER pair bumps its key's byte counter with one
//     fire-and-forget atomic (C2 into an empty filter: only the ~4% in-batch collisions do) and
//     E turns counters into replies (count < k);
//   - otherwise the region kernel writes the OWNER pairs' key ids as runs bucketed by 2^20-key
//     range (one reservation per range per region) and D' sets their bits in LDS images of the
//     ranges' new_bits words -- streaming instead of one scattered atomic per report, so the
//     add costs 5.0-5.9 ms for 50M keys at every fill (owner bits by direct atomics: 9.8 ms at
//     fill 1/2, 15.8 ms at 0).
// Chunks run strictly one after another (each chunk's regions are updated before the next
// chunk's pairs are examined), so the in-order semantics hold across chunks.  Capacities are
// sized for uniform bits; a batch that overflows one (adversarial repeats) sets `overflow`, the
// region/keys/final kernels then do nothing, and the host reruns the chunk on the table path --
// the bitmap is untouched until C, and C checks the flag before writing, so the result is exact
// either way.
#include "bucket_common.h"

#include <atomic>

namespace rbx {

constexpr uint32_t kBaRegionWords = 1u << (kBaRegionBits - 5);  // 2048

// Runs are written slot by slot: after the LDS placement every thread takes the image slots
// i = tid, tid + NT, ... and stores slot i to its bucket's reservation (the bucket id of each slot
// is kept in a byte array), so all lanes store, consecutive lanes to consecutive addresses.  At
// fan-out 256 the runs average 3-4 lines; one wave per bucket left most lanes idle.  (Whole-line
// runs with LDS carries, as in contains_partitioned.hip, measured slower here: stage A 2.09 ->
// 2.61 ms, the rebucket 2.10 -> 2.42 ms, 50M C2 keys.)

// Runs of the two radix passes are written with plain (L2 write-back) stores, not the
// nontemporal ones the contains pipeline uses: these runs are not whole lines, and the partial
// line at the end of one block's run and the start of the next reservation's (a block of the
// same sub-partition, blockIdx % 16, so the same XCD's L2 under round-robin dispatch) merge in
// L2 before write-back.  Measured (50M C2 keys): stage-1 write requests 72.6M -> 56.9M, rebucket
// 52.7M -> 49.8M, add 5.01 -> 4.83 ms; the contains pipeline, whose runs are whole lines, was
// 4.64 -> 4.84 ms slower with plain stores (profiles/r02/r02z_plain_stores.txt).
template <class T> __device__ __forceinline__ void ba_run_store(T v, T *p) { *p = v; }

// A ------------------------------------------------------------------------------------
template <int KMAX> constexpr int ba_per() { return KMAX <= 8 ? 2 : 1; }

constexpr int kBaS1Threads = 512;  // 1024 keys per tile (KMAX 8): 64 KiB image, two blocks per CU
// (2048-key tiles, one block per CU: 1.76 -> 1.89 ms)

// PF (fixed-length keys): the next tile's key bytes are loaded into registers right after this
// tile's hash, so they arrive during its count / reserve / place / store phases.
template <int KLEN, int KMAX, bool PF>
__global__ __launch_bounds__(kBaS1Threads) void k_ba_stage1(KeysDev keys, uint64_t base, uint64_t nchunk, FilterDesc f,
                                                   uint32_t s1, uint32_t ncoarse, uint64_t cap1,
                                                   unsigned long long *__restrict__ p1, uint32_t *__restrict__ cnt1,
                                                   uint32_t *__restrict__ overflow) {
    constexpr int NT = kBaS1Threads, PER = ba_per<KMAX>(), TILE = NT * PER;
    __shared__ __attribute__((aligned(16))) unsigned long long s_img[TILE * KMAX];
    __shared__ uint8_t s_bkt[TILE * KMAX];
    __shared__ uint32_t s_cnt[256], s_start[256], s_pos[256], s_gb[256];
    const uint64_t ntiles = (nchunk + TILE - 1) / TILE;
    const uint32_t sub = blockIdx.x % kBaSub;
    const uint32_t lane = threadIdx.x & 63;
    uint32_t maxidx = 0;
    constexpr bool KP = PF && KLEN > 0;
    constexpr int NV = KLEN > 0 ? KLEN / 16 : 1;
    uint4 kx[PER][NV];
    auto load_keys = [&](uint64_t tl) {
#pragma unroll
        for (int q = 0; q < PER; ++q) {
            const uint64_t t = tl * TILE + threadIdx.x + q * NT;
            if (t < nchunk) {
                const uint4 *v = (const uint4 *)(keys.bytes + (base + t) * (uint64_t)(KLEN > 0 ? KLEN : 16));
#pragma unroll
                for (int j = 0; j < NV; ++j) kx[q][j] = ld_nt16(v + j);
            }
        }
    };
    if constexpr (KP) {
        if ((uint64_t)blockIdx.x < ntiles) load_keys(blockIdx.x);
    }
    for (uint64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
        if (threadIdx.x < 256) s_cnt[threadIdx.x] = 0;
        const uint64_t t0 = tile * TILE + threadIdx.x;
        uint32_t idx[PER][KMAX];
#pragma unroll
        for (int q = 0; q < PER; ++q) {
            const uint64_t t = t0 + q * NT;
            uint64_t h1 = 0, h2 = 0;
            if constexpr (KP) {
                if (t < nchunk) hh128_regs<(KLEN > 0 ? KLEN : 16)>(kx[q], h1, h2);
            } else {
                if (t < nchunk) bk_hash<KLEN>(keys, base + t, h1, h2);
            }
            uint64_t h = h1;
#pragma unroll
            for (int j = 0; j < KMAX; ++j) {
                if ((uint32_t)j < f.k) idx[q][j] = mod63(h & 0x7fffffffffffffffULL, f.mp);
                h += (j & 1) ? h1 : h2;
            }
        }
        if constexpr (KP) {
            if (tile + gridDim.x < ntiles) load_keys(tile + gridDim.x);
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
        uint32_t gb = 0;
        if (threadIdx.x < 64) bk_scan256(s_cnt, ncoarse, s_start, s_pos);
        else if (threadIdx.x >= 256 && threadIdx.x - 256 < ncoarse) {
            const uint32_t b = threadIdx.x - 256;
            if (s_cnt[b]) gb = atomicAdd(&cnt1[b * kBaSub + sub], s_cnt[b]);
        }
        __syncthreads();
#pragma unroll
        for (int q = 0; q < PER; ++q) {
            const uint64_t t = t0 + q * NT;
            if (t < nchunk) {
#pragma unroll
                for (int j = 0; j < KMAX; ++j) {
                    if ((uint32_t)j < f.k) {
                        const uint32_t b = idx[q][j] >> s1;
                        const uint32_t slot = atomicAdd(&s_pos[b], 1u);
                        s_img[slot] = ((unsigned long long)idx[q][j] << 32) | (uint32_t)t;
                        s_bkt[slot] = (uint8_t)b;
                    }
                }
            }
        }
        // reservation results stored after the placement, which overlapped their round trip
        if (threadIdx.x >= 256 && threadIdx.x - 256 < ncoarse) s_gb[threadIdx.x - 256] = gb;
        __syncthreads();
        const uint32_t total = (uint32_t)min<uint64_t>(TILE, nchunk - tile * TILE) * f.k;
        for (uint32_t i = threadIdx.x; i < total; i += NT) {
            const uint32_t b = s_bkt[i];
            const uint64_t gp = (uint64_t)s_gb[b] + (i - s_start[b]);
            if (gp < cap1) ba_run_store(s_img[i], p1 + (uint64_t)(b * kBaSub + sub) * cap1 + gp);
            else *overflow = 1u;
        }
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
// Input partitions part = parent * sub_div + s; a pair's output partition =
// (parent << fo) + ((idx >> shift_out) & (2^fo - 1)).  Work items (partition, tile) are numbered
// so that the blocks running at one time read different parents.
constexpr uint32_t kBaRbThreads = 1024, kBaRbTile = 16 * kBaRbThreads;  // 128 KiB image: one block per CU

// Region pairs are 6 bytes when P6 (the default): lo = region offset (16 bits) << 16 | key bits
// 0-15, hi (u16) = key bits 16-25 (chunks hold <= 2^26 keys), two arrays of cap_out entries per
// region.  Against 8-byte pairs: a quarter fewer bytes written here and read by the region pass,
// and 12 registers per thread for a region block's 8 pairs instead of 16.
template <bool P6>
__device__ __forceinline__ void ba_put_region(unsigned long long e, uint64_t reg, uint64_t slot,
                                              unsigned long long *pout, uint64_t cap_out) {
    if constexpr (P6) {
        // region reg's bytes: [cap_out lo words][cap_out hi halves] (cap_out is a multiple of 64, so
        // both rows start 128-byte aligned)
        uint32_t *lo = (uint32_t *)pout + reg * (cap_out * 3 / 2);
        uint16_t *hi = (uint16_t *)(lo + cap_out);
        const uint32_t idx = (uint32_t)(e >> 32), key = (uint32_t)e;
        ba_run_store((idx << 16) | (key & 0xffffu), lo + slot);
        ba_run_store((uint16_t)(key >> 16), hi + slot);
    } else {
        ba_run_store(e, pout + reg * cap_out + slot);
    }
}

// 16K-pair tiles, one 1024-thread block per CU (8K-pair tiles at two blocks per CU, each
// overlapping the other's loads, measured 1.65 -> 1.78 ms).  A slot's bucket is read back from its
// pair (no bucket byte array).
template <bool P6, bool STAMP, bool PF>
__global__ __launch_bounds__(kBaRbThreads) void k_ba_rebucket(const unsigned long long *__restrict__ pin,
                                                     const uint32_t *__restrict__ cnt_in, uint64_t cap_in,
                                                     uint32_t nparents, uint32_t sub_div, uint32_t items_per_part,
                                                     uint32_t shift_out, uint32_t fo, uint32_t nparts_out,
                                                     unsigned long long *__restrict__ pout,
                                                     uint32_t *__restrict__ cnt_out, uint64_t cap_out,
                                                     uint32_t *__restrict__ overflow,
                                                     unsigned long long *__restrict__ stamps) {
    constexpr int NT = kBaRbThreads, PER = 8, TILE = kBaRbTile;  // PER uint4 = two pairs each
    PhaseStamps<STAMP, 4> ps;
    ps.start();
    __shared__ __attribute__((aligned(16))) unsigned long long s_img[TILE];
    __shared__ uint32_t s_cnt[256], s_start[256], s_pos[256], s_gb[256];
    const uint32_t nf = 1u << fo, fmask = nf - 1;
    const uint32_t nparts = nparents * sub_div;
    const uint32_t nitems = nparts * items_per_part;
    struct Item {
        uint32_t parent, part, m;
        uint64_t start;
    };
    // uniform: the next item with pairs.  64 candidate items per round, one per lane, so a small
    // batch (C1: 7M pairs in items sized for the worst case) does not walk its empty items one
    // dependent count load after another (C1's rebucket ~96 us per 1M-key add)
    auto find_item = [&](uint32_t from, Item &ii) -> uint32_t {
        const uint32_t lane = threadIdx.x & 63;
        for (uint32_t base = from; base < nitems; base += 64 * gridDim.x) {
            const uint32_t cand = base + lane * gridDim.x;
            bool has = false;
            if (cand < nitems) {
                const uint32_t it = cand / nparts, ix = cand - it * nparts;
                const uint32_t part = (ix % nparents) * sub_div + ix / nparents;
                has = (uint64_t)it * TILE < min<uint64_t>(cnt_in[part], cap_in);
            }
            const uint64_t hit = __ballot(has);
            if (hit) {
                const uint32_t item = base + (uint32_t)__builtin_ctzll(hit) * gridDim.x;
                const uint32_t it = item / nparts, ix = item - it * nparts;
                ii.parent = ix % nparents;
                ii.part = ii.parent * sub_div + ix / nparents;
                const uint64_t nc = min<uint64_t>(cnt_in[ii.part], cap_in);
                ii.start = (uint64_t)it * TILE;
                ii.m = (uint32_t)min<uint64_t>(TILE, nc - ii.start);
                return item;
            }
        }
        return nitems;
    };
    unsigned long long e[2 * PER];
    auto load_tile = [&](const Item &ii) {
        // cap_in is a multiple of TILE: the tile is 16-byte aligned
        const u32x4 *src = (const u32x4 *)(pin + (uint64_t)ii.part * cap_in + ii.start);
#pragma unroll
        for (int p = 0; p < PER; ++p) {
            const uint32_t q = 2 * (p * NT + threadIdx.x);
            u32x4 v = {0u, 0u, 0u, 0u};
            if (q < ii.m) v = __builtin_nontemporal_load(src + p * NT + threadIdx.x);
            e[2 * p] = w2(v.x, v.y);
            e[2 * p + 1] = w2(v.z, v.w);
        }
    };
    Item cur{};
    uint32_t item = find_item(blockIdx.x, cur);
    if (PF && item < nitems) load_tile(cur);
    while (item < nitems) {
        const uint32_t parent = cur.parent, m = cur.m;
        if (threadIdx.x < 256) s_cnt[threadIdx.x] = 0;
        __syncthreads();
        if (!PF) load_tile(cur);
#pragma unroll
        for (int p = 0; p < 2 * PER; ++p) {
            const uint32_t q = 2 * ((p >> 1) * NT + threadIdx.x) + (p & 1);
            if (q < m) atomicAdd(&s_cnt[(uint32_t)(e[p] >> (32 + shift_out)) & fmask], 1u);
        }
        __syncthreads();
        ps.mark(0);
        uint32_t gb = 0;
        if (threadIdx.x < 64) bk_scan256(s_cnt, nf, s_start, s_pos);
        else if (threadIdx.x >= 256 && threadIdx.x - 256 < nf) {
            const uint32_t f = threadIdx.x - 256;
            const uint32_t r = (parent << fo) + f;
            if (s_cnt[f] && r < nparts_out) gb = atomicAdd(&cnt_out[r], s_cnt[f]);
        }
        __syncthreads();
        ps.mark(1);
#pragma unroll
        for (int p = 0; p < 2 * PER; ++p) {
            const uint32_t q = 2 * ((p >> 1) * NT + threadIdx.x) + (p & 1);
            if (q < m) {
                const uint32_t f = (uint32_t)(e[p] >> (32 + shift_out)) & fmask;
                const uint32_t slot = atomicAdd(&s_pos[f], 1u);
                s_img[slot] = e[p];
            }
        }
        // PF: the next item's tile is loaded into the pair registers (free after the placement),
        // so the load flies during this tile's stores instead of stalling the next tile's count
        Item nxt{};
        const uint32_t nitem = find_item(item + gridDim.x, nxt);
        if (PF && nitem < nitems) load_tile(nxt);
        // the reservation results reach LDS only now: the placement above overlapped their round trip
        if (threadIdx.x >= 256 && threadIdx.x - 256 < nf) s_gb[threadIdx.x - 256] = gb;
        __syncthreads();
        ps.mark(2);
        for (uint32_t i = threadIdx.x; i < m; i += NT) {
            const unsigned long long e1 = s_img[i];
            const uint32_t f = (uint32_t)(e1 >> (32 + shift_out)) & fmask;
            const uint64_t gp = (uint64_t)s_gb[f] + (i - s_start[f]);
            if (gp < cap_out) ba_put_region<P6>(e1, (parent << fo) + f, gp, pout, cap_out);
            else *overflow = 1u;
        }
        __syncthreads();
        ps.mark(3);
        item = nitem;
        cur = nxt;
    }
    ps.flush(stamps);
}

// The r05 whole-line rebucket (k_ba_emit2), which padded a partition's last runs with kBaPadHi pairs, was
// removed in r06; the region pass still skips such pairs, which nothing emits now.
constexpr uint16_t kBaPadHi = 0xffffu;  // hi half of a padding pair: real keys are < 2^26 (hi < 1024)
static_assert(kBaMaxRegionPairs <= 65536, "region pair counts fit the LDS counters");

// (k_ba_emit2, the whole-line rebucket, measured 0.03 ms slower at C2 and was removed in r06:
// profiles/r05/; the padding constants above stay for the region pass.)

// mode -----------------------------------------------------------------------------------
// Sampled fill of the bitmap -> how C reports new keys (see the header): 1 = non-owner counters,
// 2 = owner records, 0 = owner bits.
// r05: every block also zeroes the chunk's counters (zero_a: cnt1 .. overflow, not the mode word)
// and new_bits (zero_b) -- two hipMemsetAsync fills (~5 us each on the C1 add) folded into this
// launch.
__global__ __launch_bounds__(1024) void k_ba_mode(const uint32_t *__restrict__ bm, uint64_t nwords4, uint32_t policy,
                                                  uint32_t *__restrict__ mode, uint32_t *__restrict__ zero_a,
                                                  uint64_t na, uint32_t *__restrict__ zero_b, uint64_t nb) {
    __shared__ uint32_t s_sum[16];
    {
        const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
        for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < na; i += stride) zero_a[i] = 0u;
        for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nb / 4; i += stride)
            ((u32x4 *)zero_b)[i] = u32x4{0u, 0u, 0u, 0u};
        if (blockIdx.x == 0 && threadIdx.x < (nb & 3)) zero_b[(nb & ~3ULL) + threadIdx.x] = 0u;
    }
    if (blockIdx.x != 0) return;  // uniform: the mode is block 0's
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
            // sampled fill f = t / (4096 * 32): non-owner counters below 3/32, owner records
            // above (owner bits never measured faster: profiles/r02/r02j_addfill_modes.jsonl)
            m = t < 4096u * 3u ? 1u : 2u;
        }
        *mode = m;
    }
}

// C ------------------------------------------------------------------------------------
// One 1024-thread block per 2^16-bit region at a time, two blocks per CU (32 KiB of LDS each;
// the 64-VGPR budget of 8 waves/SIMD holds the region's <= 8192 pairs in registers).
// A bit's first setter is the smallest key id among the pairs that meet it at 0.  Most such bits
// are met by one pair only (~5.3K pairs on 65K bits at C2: ~0.3% of bits are met twice), so
// instead of an owner word per bit the block keeps two bitsets -- met once, met again -- and
// resolves only the bits met again, in a small LDS table {bit, min key id} (atomicCAS claim +
// atomicMin).  A table that fills up (adversarial batches) is cleared and the bits still pending
// take another round; every round resolves at least one bit, so the loop ends.
constexpr uint32_t kBaRegionThreads = 1024;
constexpr uint32_t kBaPer = kBaMaxRegionPairs / kBaRegionThreads;  // pairs per thread
constexpr uint32_t kBaTableBits = 10;                               // 1024 collision slots
static_assert(kBaPer <= 32, "pair masks are 32-bit");

__device__ __forceinline__ uint32_t ba_slot(uint32_t off, uint32_t t) {
    return ((off * 2654435761u) >> (32 - kBaTableBits)) + t & ((1u << kBaTableBits) - 1);
}


// C (6-byte pairs, pipelined) -----------------------------------------------------------
// The region pass (the resolution of the r02 k_ba_region, removed in r06), with the next region's inputs in flight while the current
// one is resolved.  The r02 kernel waited, per region, for its pair count, then for the region's pairs
// and bitmap (two dependent memory round trips before any work), and took 60 B/lane of spills.
// Here, right after a region's pairs are copied from LDS into registers, the block issues the next
// region's pairs straight into that LDS buffer (global_load_lds: no registers held for them) and
// its bitmap into 4 registers, so both land during the current region's passes.
// An LDS-DMA is a pending LDS write on the VM counter, and a __syncthreads() fence waits for every
// VM operation, which would drain the prefetch at the first barrier; so the barriers in the body
// are raw s_barrier with an LDS-counter wait only (ba_bar), the block-wide ORs go through LDS flag
// words (ba_bar_or), and the one drain is an explicit vmcnt(0) at the top of the next region.
// LDS (77 KiB: two blocks per CU): the pair buffer (32 KiB lo + 16 KiB hi), the region's bitmap,
// the met-once / met-again bitsets (8 KiB each), a 512-slot collision table; the owner records
// reuse the bitmap/bitset/table space (7168 slots) once the bitmap has been written back, and a
// region with more owners than that (only adversarial batches in records mode) reports them by
// direct atomics instead.
__device__ __forceinline__ void ba_bar() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }
// Makes the pair registers opaque at a phase boundary, so the compiler recomputes each pair's word
// offset, bit and key (a few VALU ops) instead of keeping them live across the phases: at 64 VGPRs
// that CSE spilled, and a scratch reload waits on the VM counter, which drains the prefetch.
// LDS atomics of the region passes as inline asm: hipcc waits for every outstanding LDS-DMA
// (vmcnt(0)) before an LDS atomic it emits itself, even into another LDS object, which drained the
// prefetch at pass 1.  The asm forms are counted on lgkmcnt like the compiler's own (extra younger
// LDS operations only make its counted waits stricter); a returning form waits for its result.
__device__ __forceinline__ uint32_t lds_addr(const void *p) {
    return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void *)p;
}
__device__ __forceinline__ uint32_t lds_or_rtn(uint32_t *p, uint32_t v) {
    uint32_t r;
    asm volatile("ds_or_rtn_b32 %0, %1, %2\n\ts_waitcnt lgkmcnt(0)" : "=v"(r) : "v"(lds_addr(p)), "v"(v) : "memory");
    return r;
}
__device__ __forceinline__ void lds_or(uint32_t *p, uint32_t v) {
    asm volatile("ds_or_b32 %0, %1" ::"v"(lds_addr(p)), "v"(v) : "memory");
}
__device__ __forceinline__ void lds_add(uint32_t *p, uint32_t v) {
    asm volatile("ds_add_u32 %0, %1" ::"v"(lds_addr(p)), "v"(v) : "memory");
}
__device__ __forceinline__ uint32_t lds_add_rtn(uint32_t *p, uint32_t v) {
    uint32_t r;
    asm volatile("ds_add_rtn_u32 %0, %1, %2\n\ts_waitcnt lgkmcnt(0)" : "=v"(r) : "v"(lds_addr(p)), "v"(v) : "memory");
    return r;
}
__device__ __forceinline__ void lds_min(uint32_t *p, uint32_t v) {
    asm volatile("ds_min_u32 %0, %1" ::"v"(lds_addr(p)), "v"(v) : "memory");
}
template <int N> __device__ __forceinline__ void ba_opaque(uint32_t (&v)[N]) {
#pragma unroll
    for (int i = 0; i < N; ++i) asm volatile("" : "+v"(v[i]));
}

// Bits met again get compact slots instead of a hashed table: after pass 1 every word of the
// met-again bitset gets the rank base of its bits (one LDS counter add per nonzero word), so a bit's
// slot is base[word] + the popcount of the met-again bits below it in its word, and its first
// setter is one atomicMin there -- no claim, no probing.  kBa6Slots slots per round; a region with
// more bits met again (C2: ~200) takes further rounds.
constexpr uint32_t kBa6Slots = 1024;
constexpr uint32_t kBa6Main = 3 * kBaRegionWords + kBa6Slots;  // 7168 words
static_assert(kBa6Main >= 7168, "record space");

template <bool STAMP>
__global__ __launch_bounds__(kBaRegionThreads) __attribute__((amdgpu_waves_per_eu(8))) void k_ba_region6(
    const uint32_t *__restrict__ p3, const uint32_t *__restrict__ cnt3, uint64_t cap3, uint32_t nregions,
    uint32_t *__restrict__ bm, uint64_t nwords4, uint32_t *__restrict__ new_bits, uint32_t *__restrict__ ctr,
    uint32_t *__restrict__ recs, uint32_t *__restrict__ rec_cnt, uint64_t cap_rec, uint32_t nranges,
    const uint32_t *__restrict__ overflow, const uint32_t *__restrict__ mode, uint32_t rec_limit, uint32_t diag,
    unsigned long long *__restrict__ stamps) {
    if (!kDiag) diag = 0;  // wrong-answer diagnostics exist in the profiling build only (rbx_kernels.h)
    constexpr uint32_t NT = kBaRegionThreads, PER = kBaPer, C = kBa6Slots;
    PhaseStamps<STAMP> ps;
    constexpr uint32_t NV = kBaRegionWords / 4;  // 16-byte vectors of the region's bitmap
    static_assert(PER == 8 && NV <= NT, "8 pair slots and at most one 16-byte bitmap vector per thread");
    // The DMA target is an LDS object of its own, so the compiler can tell that the passes' LDS
    // accesses (the other object) do not alias it and need not wait for the DMA.
    __shared__ __attribute__((aligned(16))) uint32_t lds_pairs[kBaMaxRegionPairs * 3 / 2];
    __shared__ __attribute__((aligned(16))) uint32_t lds[kBa6Main + 4 * 64 + 8];
    uint32_t *s_plo = lds_pairs;                                    // [8192] pair lo words
    uint16_t *s_phi = (uint16_t *)(lds_pairs + kBaMaxRegionPairs);  // [8192] pair hi halves
    uint32_t *s_main = lds;
    uint32_t *s_bm = s_main, *s_seen = s_bm + kBaRegionWords, *s_multi = s_seen + kBaRegionWords;
    uint32_t *s_tmin = s_multi + kBaRegionWords;                    // [C] first setter per slot
    uint16_t *s_base = (uint16_t *)s_seen;                          // [2048] slot bases, after pass 1
    uint32_t *s_rec = s_main;                                       // [kBa6Main] after the write-back
    uint32_t *s_rc = s_main + kBa6Main, *s_rst = s_rc + 64, *s_rpos = s_rst + 64, *s_rgb = s_rpos + 64;
    uint32_t *s_flag = s_rgb + 64;  // [6] owner total, [7] bits met again
    if (*overflow) return;
    const uint32_t md = *mode;
    const bool counters = md == 1, records = md == 2, bits = md == 0;
    const uint32_t rlim = min(rec_limit, kBa6Main);
    // The block's regions are blockIdx.x + i * gridDim.x; lane l of every wave holds the pair count
    // of region i = ibase + l (one vector load per 64 regions instead of a dependent scalar load per
    // region).  Returns the first region at or after index i with pairs (uniform), or nregions.
    uint32_t ibase = 0, cvec = 0;
    auto load_counts = [&](uint32_t ib) {
        ibase = ib;
        const uint32_t rr = blockIdx.x + (ib + (threadIdx.x & 63)) * gridDim.x;
        cvec = rr < nregions ? (uint32_t)min<uint64_t>(cnt3[rr], cap3) : 0u;
    };
    auto next_region = [&](uint32_t i, uint32_t &cnt) -> uint32_t {
        for (;;) {
            if (blockIdx.x + ibase * gridDim.x >= nregions) return nregions;
            if (i >= ibase + 64) {
                load_counts(i & ~63u);
                continue;
            }
            const uint64_t m = __ballot(cvec != 0u && (threadIdx.x & 63) >= i - ibase);
            if (m) {
                const uint32_t l = (uint32_t)__builtin_ctzll(m);
                cnt = (uint32_t)__builtin_amdgcn_readlane((int)cvec, (int)l);
                return blockIdx.x + (ibase + l) * gridDim.x;
            }
            i = ibase + 64;
        }
    };
    // the region's pairs -> the LDS buffer (16 B per lane, lane-linear per wave), its bitmap -> registers
    auto prefetch = [&](uint32_t tid, uint32_t r, uint32_t cnt, u32x4 &bw) {
        const uint32_t wave = tid >> 6;
        const uint32_t *lo = p3 + (uint64_t)r * (cap3 * 3 / 2);
        const uint32_t nlo = (cnt + 3) / 4, nhi = (cnt + 7) / 8;
#pragma unroll
        for (uint32_t i = 0; i < 2; ++i) {
            const uint32_t j = i * NT + tid;
            if (j < nlo)
                __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void *)((const u32x4 *)lo + j),
                                                 (__attribute__((address_space(3))) void *)((u32x4 *)s_plo + i * NT + wave * 64),
                                                 16, 0, 0);
        }
        if (tid < nhi)
            __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void *)((const u32x4 *)(lo + cap3) + tid),
                                             (__attribute__((address_space(3))) void *)((u32x4 *)s_phi + wave * 64),
                                             16, 0, 0);
        const uint64_t w0 = (uint64_t)r * kBaRegionWords;
        bw = u32x4{0u, 0u, 0u, 0u};
        if (tid < NV && w0 + 4 * tid < nwords4) bw = ((const u32x4 *)(bm + w0))[tid];
    };
    uint32_t n = 0;
    load_counts(0);
    uint32_t r = next_region(0, n);
    u32x4 bw;
    if (r < nregions) prefetch(threadIdx.x, r, n, bw);
    ps.start();
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the first region's pairs and bitmap
    ba_bar();
    while (r < nregions) {
        ps.mark(0);
        // the thread index made opaque per region: values derived from it (LDS addresses, lane
        // predicates) are recomputed instead of hoisted out of the loop and kept live (spilled)
        uint32_t tid = threadIdx.x;
        asm volatile("" : "+v"(tid));
        // re-derived at each phase, so no copy of it lives (and spills) across the phases
        auto fresh_tid = [&]() {
            tid = threadIdx.x;
            asm volatile("" : "+v"(tid));
        };
        // my pairs: q = p * NT + tid (strided, so every thread holds ceil(n / NT) or one fewer: with
        // 8 consecutive pairs per thread a 5.3K-pair region left a third of the block idle and the
        // rest on an 8-deep serial chain of LDS round trips)
        uint32_t lo[PER], hw[PER / 2];
#pragma unroll
        for (uint32_t p = 0; p < PER; ++p) lo[p] = s_plo[p * NT + tid];
#pragma unroll
        for (uint32_t p = 0; p < PER; p += 2)
            hw[p / 2] = (uint32_t)s_phi[p * NT + tid] | (uint32_t)s_phi[(p + 1) * NT + tid] << 16;
        // (k_ba_emit2 pads a partition's last runs with kBaPadHi pairs: not pairs of any key)
        auto valid = [&](uint32_t p) {
            return p * NT + tid < n && ((hw[p >> 1] >> (16 * (p & 1))) & 0xffffu) != kBaPadHi;
        };
        const uint64_t w0 = (uint64_t)r * kBaRegionWords;
        const bool has_words = tid < NV && w0 + 4 * tid < nwords4;
        if (tid < NV) {
            ((u32x4 *)s_bm)[tid] = bw;
            ((u32x4 *)s_seen)[tid] = u32x4{0u, 0u, 0u, 0u};
            ((u32x4 *)s_multi)[tid] = u32x4{0u, 0u, 0u, 0u};
        }
        for (uint32_t i = tid; i < C; i += NT) s_tmin[i] = ~0u;
        if (tid < 64) s_rc[tid] = 0;
        if (tid == 0) {  // owner total and slot counter (the previous region's reads ended at its last barrier)
            s_flag[6] = 0u;
            s_flag[7] = 0u;
        }
        ba_bar();  // the pair buffer has been read by every thread: refill it for the next region
        ps.mark(1);
        uint32_t nn = 0;
        const uint32_t rn = next_region((r - blockIdx.x) / gridDim.x + 1, nn);
        if (rn < nregions && !(diag & 8)) prefetch(tid, rn, nn, bw);
        ps.mark(2);
        auto key_of = [&](uint32_t p) { return ((hw[p >> 1] >> (16 * (p & 1))) & 0xffffu) << 16 | (lo[p] & 0xffffu); };
        // pass 1: which pairs meet a 0 bit, and which of those bits are met more than once
        uint32_t zm = 0;
#pragma unroll
        for (uint32_t p = 0; p < PER; ++p) {
            const uint32_t off = lo[p] >> 16, w = off >> 5, b = bit_in_word(off);
            if (valid(p) && (s_bm[w] & b) == 0u) {
                zm |= 1u << p;
                if (lds_or_rtn(&s_seen[w], b) & b) lds_or(&s_multi[w], b);
            }
        }
        ba_bar();
        ps.mark(3);
        ba_opaque(lo);
        fresh_tid();
        // pass 2: a bit met once is owned by its pair; bits met again get slots (see kBa6Slots)
        uint32_t own = 0, pend = 0;
#pragma unroll
        for (uint32_t p = 0; p < PER; ++p) {
            if (zm & (1u << p)) {
                const uint32_t off = lo[p] >> 16;
                if (s_multi[off >> 5] & bit_in_word(off)) pend |= 1u << p;
                else own |= 1u << p;
            }
        }
        {  // slot bases of my two met-again words (s_seen, now s_base, is dead after pass 1)
            const uint32_t m0 = s_multi[2 * tid], m1 = s_multi[2 * tid + 1];
            const uint32_t c = __popc(m0) + __popc(m1);
            if (c) {
                const uint32_t b0 = lds_add_rtn(&s_flag[7], c);
                s_base[2 * tid] = (uint16_t)b0;
                s_base[2 * tid + 1] = (uint16_t)(b0 + __popc(m0));
            }
        }
        ba_bar();
        ps.mark(4);
        const uint32_t nmulti = s_flag[7];  // uniform
        ba_opaque(lo);
        fresh_tid();
        auto slot_of = [&](uint32_t p) {
            const uint32_t off = lo[p] >> 16, w = off >> 5, b = bit_in_word(off);
            return (uint32_t)s_base[w] + (uint32_t)__popc(s_multi[w] & (b - 1u));
        };
        for (uint32_t r0 = 0; r0 < nmulti; r0 += C) {  // uniform; one round at C2
            ba_opaque(lo);
            ba_opaque(hw);
            fresh_tid();
            if (r0) {
                ba_bar();  // the previous round's reads of s_tmin
                for (uint32_t i = tid; i < C; i += NT) s_tmin[i] = ~0u;
                ba_bar();
            }
#pragma unroll
            for (uint32_t p = 0; p < PER; ++p) {
                if (pend & (1u << p)) {
                    const uint32_t sl = slot_of(p) - r0;
                    if (sl < C) lds_min(&s_tmin[sl], key_of(p));
                }
            }
            ba_bar();
            ba_opaque(lo);
            ba_opaque(hw);
            fresh_tid();
#pragma unroll
            for (uint32_t p = 0; p < PER; ++p) {
                if (pend & (1u << p)) {
                    const uint32_t sl = slot_of(p) - r0;
                    if (sl < C && s_tmin[sl] == key_of(p)) own |= 1u << p;
                }
            }
        }
        ps.mark(5);
        // owners set their bits; the other kind is reported to the key pass
        ba_opaque(lo);
        ba_opaque(hw);
        fresh_tid();
#pragma unroll
        for (uint32_t p = 0; p < PER; ++p) {
            const uint32_t off = lo[p] >> 16;
            if (own & (1u << p)) {
                lds_or(&s_bm[off >> 5], bit_in_word(off));
                if (diag & 4) continue;
                const uint32_t key = key_of(p);
                if (bits) atomicOr(&new_bits[key >> 5], 1u << (key & 31));
                else if (records) lds_add(&s_rc[key >> kBaKeyRangeBits], 1u);
            } else if (counters && !(diag & 4) && valid(p)) {
                const uint32_t key = key_of(p);
                atomicAdd(&ctr[key >> 2], 1u << (8 * (key & 3)));  // no return: not waited on here
            }
        }
        fresh_tid();
        const uint32_t lane = tid & 63, wave = tid >> 6;
        if (records) {  // owner total of the block (one LDS atomic per wave)
            uint32_t c = __popc(own);
#pragma unroll
            for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o, 64);
            if (lane == 0 && c) lds_add(&s_flag[6], c);
        }
        // the region's words go back whether or not a bit changed (they are this block's alone)
        ba_bar();
        ps.mark(6);
        {
            if (has_words) ((u32x4 *)(bm + w0))[tid] = ((const u32x4 *)s_bm)[tid];
            if (records && !(diag & 4)) {
                const uint32_t tot = s_flag[6];
                if (tot > rlim) {  // uniform: too many records for LDS, report them directly
#pragma unroll
                    for (uint32_t p = 0; p < PER; ++p) {
                        if (own & (1u << p)) {
                            const uint32_t key = key_of(p);
                            atomicOr(&new_bits[key >> 5], 1u << (key & 31));
                        }
                    }
                } else {  // owner key ids as runs per 2^20-key range
                    uint32_t gb = 0;
                    const uint32_t q = tid - 128;
                    const bool reserver = tid >= 128 && q < nranges;
                    if (tid < 64) bk_scan128(s_rc, nranges, s_rst, s_rpos, lane);
                    else if (reserver && s_rc[q]) gb = atomicAdd(&rec_cnt[q], s_rc[q]);
                    ba_bar();  // the scan, and the write-back's reads of s_bm, before s_rec is written
#pragma unroll
                    for (uint32_t p = 0; p < PER; ++p) {
                        if (own & (1u << p)) {
                            const uint32_t key = key_of(p);
                            s_rec[atomicAdd(&s_rpos[key >> kBaKeyRangeBits], 1u)] = key;
                        }
                    }
                    if (reserver) s_rgb[q] = gb;
                    ba_bar();
                    // records per range <= 2^20 keys x k = cap_rec: no overflow
                    for (uint32_t rq = wave; rq < nranges; rq += NT / 64) {
                        const uint32_t rn2 = s_rc[rq], st = s_rst[rq];
                        uint32_t *dst = recs + (uint64_t)rq * cap_rec + s_rgb[rq];
                        for (uint32_t t = lane; t < rn2; t += 64) run_store(s_rec[st + t], dst + t);
                    }
                }
            }
        }
        // one barrier ends this region and starts the next: the next region's pairs and bitmap (and
        // this region's stores) are complete, and s_bm / s_rec / s_rc / s_flag[6] may be reused
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        ba_bar();
        ps.mark(7);
        r = rn;
        n = nn;
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    ps.flush(stamps);
}

// D ------------------------------------------------------------------------------------
// Owner records -> new_bits: item = (key range q, slice s of 2^20 records): the slice's key ids
// set bits of a 128 KiB LDS image of the range's new_bits words, whose nonzero words are OR-ed in.
constexpr uint32_t kBaRangeWords = 1u << (kBaKeyRangeBits - 5);  // 32768

__global__ __launch_bounds__(1024) void k_ba_keys_rec(const uint32_t *__restrict__ recs,
                                                      const uint32_t *__restrict__ rec_cnt, uint64_t cap_rec,
                                                      uint32_t nranges, uint32_t nslices,
                                                      uint32_t *__restrict__ new_bits,
                                                      const uint32_t *__restrict__ overflow,
                                                      const uint32_t *__restrict__ mode) {
    constexpr uint32_t NT = 1024;
    __shared__ uint32_t s_bits[kBaRangeWords];  // 128 KiB
    if (*overflow || *mode != 2) return;
    const uint32_t nitems = nranges * nslices;
    for (uint32_t item = blockIdx.x; item < nitems; item += gridDim.x) {
        const uint32_t q = item % nranges, sl = item / nranges;
        const uint64_t nrec = min<uint64_t>(rec_cnt[q], cap_rec);
        const uint64_t start = (uint64_t)sl << kBaKeyRangeBits;
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
// Replies and the count, one thread per 32 keys.  Non-owner counters (mode 1) are read here
// directly -- key t is new iff fewer than k of its pairs were non-owners -- and zeroed for the next
// call (r05: the separate k_ba_keys pass and its launch are gone); owner bits / records (modes 0,
// 2) arrive as new_bits.
__global__ __launch_bounds__(256) void k_ba_final(const uint32_t *__restrict__ new_bits, uint32_t *__restrict__ ctr,
                                                  uint32_t k, uint64_t nchunk, uint64_t base,
                                                  uint8_t *__restrict__ out_new,
                                                  unsigned long long *__restrict__ count,
                                                  const uint32_t *__restrict__ overflow,
                                                  const uint32_t *__restrict__ mode) {
    __shared__ unsigned long long s_part[4];
    if (*overflow) return;
    const bool counters = *mode == 1u;
    unsigned long long c = 0;
    const uint64_t nwords = (nchunk + 31) >> 5;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; g < nwords; g += stride) {
        uint32_t v = 0;
        if (counters) {
            u32x4 *src = (u32x4 *)(ctr + 8 * g);
            const u32x4 a = src[0], b = src[1];
            const uint32_t c8[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
#pragma unroll
            for (uint32_t j = 0; j < 8; ++j)
#pragma unroll
                for (uint32_t t = 0; t < 4; ++t) v |= (((c8[j] >> (8 * t)) & 0xffu) < k ? 1u : 0u) << (4 * j + t);
            if (a.x | a.y | a.z | a.w) src[0] = u32x4{0u, 0u, 0u, 0u};
            if (b.x | b.y | b.z | b.w) src[1] = u32x4{0u, 0u, 0u, 0u};
        } else {
            v = new_bits[g];
        }
        const uint64_t rem = nchunk - (g << 5);
        if (rem < 32) v &= (1u << rem) - 1u;
        c += __popc(v);
        if (out_new) {
            uint8_t *o = out_new + base + (g << 5);
            if (rem >= 32 && ((uintptr_t)o & 3) == 0) {
#pragma unroll
                for (uint32_t q = 0; q < 8; ++q) {
                    const uint32_t nib = (v >> (4 * q)) & 0xfu;
                    ((uint32_t *)o)[q] = (nib & 1u) | ((nib & 2u) << 7) | ((nib & 4u) << 14) | ((nib & 8u) << 21);
                }
            } else {
                const uint32_t m = rem < 32 ? (uint32_t)rem : 32u;
                for (uint32_t q = 0; q < m; ++q) o[q] = (uint8_t)((v >> q) & 1u);
            }
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

// launcher ---------------------------------------------------------------------------------
// rbx_tune "add_region_grid": k_ba_region6 blocks; each walks regions r, r + grid, ...
static std::atomic<uint32_t> g_region_grid{2048};
void set_add_region_grid(int v) { g_region_grid = (uint32_t)v; }
// rbx_tune "add_rec_lds_limit" (tests): owner records a k_ba_region6 block stages in LDS before it
// reports a region's owners by direct atomics instead (default and maximum kBa6Main)
static std::atomic<uint32_t> g_rec_limit{kBa6Main};
void set_add_rec_lds_limit(int v) { g_rec_limit = (uint32_t)v; }
// (r02-r05 A/B switches removed in r06 with the variants they selected: add_region_kernel (8-byte
// pairs + k_ba_region), add_rebucket_lines (k_ba_emit2), add_rebucket_prefetch 0, add_stage1_prefetch 0.)

template <int KLEN, int KMAX>
static void ba_chunk(const BaArgs &a, hipStream_t st) {
    constexpr int TILE = kBaS1Threads * ba_per<KMAX>();
    const uint64_t ntiles = (a.nchunk + TILE - 1) / TILE;
    // (the mode word is the last counter word: zeroed by nobody, written by block 0)
    const uint64_t na = (uint64_t)(a.mode - a.cnt1), nb = (uint64_t)a.nranges << (kBaKeyRangeBits - 5);
    const unsigned zgrid = (unsigned)std::min<uint64_t>(1024, std::max<uint64_t>(na, nb / 4) / 1024 + 1);
    hipLaunchKernelGGL(k_ba_mode, dim3(zgrid), dim3(1024), 0, st, (const uint32_t *)a.f.bm, a.nwords4, a.record_policy,
                       a.mode, a.cnt1, na, a.new_bits, nb);
    hipLaunchKernelGGL((k_ba_stage1<KLEN, KMAX, true>), dim3((unsigned)std::min<uint64_t>(ntiles, 4096)),
                       dim3(kBaS1Threads), 0, st, a.keys, a.base, a.nchunk, a.f, a.s1, a.ncoarse, a.cap1, a.p1, a.cnt1,
                       a.overflow);
    const uint32_t it1 = (uint32_t)((a.cap1 + kBaRbTile - 1) / kBaRbTile);
    const dim3 rgrid(std::min<uint32_t>(a.nregions, g_region_grid.load()));
    // phase stamps (rbx_bench_add_stamps) only in the profiling build
    const bool stamps = kDiag && a.stamps;
    unsigned long long *rst = stamps ? a.stamps + 8 : nullptr;
#define BA_REBUCKET(ST)                                                                                                  \
    hipLaunchKernelGGL((k_ba_rebucket<true, ST, true>), dim3(2048), dim3(kBaRbThreads), 0, st, a.p1, a.cnt1, a.cap1,      \
                       a.ncoarse, kBaSub, it1, a.s3, a.f3, a.nregions, a.p3, a.cnt3, a.cap3, a.overflow, rst)
#define BA_REGION6(ST)                                                                                                    \
    hipLaunchKernelGGL((k_ba_region6<ST>), rgrid, dim3(kBaRegionThreads), 0, st, (const uint32_t *)a.p3, a.cnt3, a.cap3,   \
                       a.nregions, a.f.bm, a.nwords4, a.new_bits, a.ctr, a.recs, a.rec_cnt, a.cap_rec, a.nranges,          \
                       a.overflow, a.mode, g_rec_limit.load(), a.diag, stamps ? a.stamps : nullptr)
    if constexpr (kDiag) {
        if (stamps) {
            BA_REBUCKET(true);
            BA_REGION6(true);
        } else {
            BA_REBUCKET(false);
            BA_REGION6(false);
        }
    } else {
        BA_REBUCKET(false);
        BA_REGION6(false);
    }
#undef BA_REBUCKET
#undef BA_REGION6
    hipLaunchKernelGGL(k_ba_keys_rec, dim3(std::min<uint32_t>(a.nranges * a.f.k, 2048)), dim3(1024), 0, st, a.recs,
                       a.rec_cnt, a.cap_rec, a.nranges, a.f.k, a.new_bits, a.overflow, a.mode);
    // one thread per 32 keys (a per-thread chain over a smaller grid was the C1 add's third-largest cost);
    // at most 512 blocks: each adds its count to ONE counter, and those atomics serialise (r05)
    hipLaunchKernelGGL(k_ba_final, dim3((unsigned)std::min<uint64_t>(512, ((a.nchunk + 31) / 32 + 255) / 256)),
                       dim3(256), 0, st, a.new_bits, a.ctr, a.f.k, a.nchunk, a.base, a.out_new, a.count, a.overflow,
                       a.mode);
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
