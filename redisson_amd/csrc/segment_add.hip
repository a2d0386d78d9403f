// segment_add.hip -- the per-segment multi-tenant add (rbx_bloom_add_multi[_dev] when every filter of
// the batch is distinct: C3's add half) on gfx950.  Split from stream_kernels.hip in r06.
// Semantics: M/RedissonBloomFilter.java:104-137 in M/command/CommandBatchService.java:115-134 order
// (DESIGN.md §3.9).  M/ = /root/reference/redisson/src/main/java/org/redisson/
#include "bloom_common.h"

namespace rbx {

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
//
// r06 (profiles/r06/): tiles of min(256, 0.625 * 2^lgs / k) keys (256 at k = 10, where r05
// took 192 of its 256 lanes); each tile's gathers are issued before its tables are cleared (the clear
// and the barrier run under the gathers' latency) and the next tile's hash is computed while this
// tile's stores drain; 8192 workgroups grid-stride over the segments (4096: +2%, 512: +15%, one per
// segment: +13%).  Two other designs were built and measured slower at C3 (1,000 keys per segment): the
// whole segment's SETBITs held in LDS until the segment ends (8,192-slot tables, 512 threads, one
// workgroup per CU: 35.1 ms; 4,096 slots, 256 threads: 47.1 ms; vs 28.5 ms for these tiles).
template <int KLEN, int KMAX>
__global__ __launch_bounds__(256) void k_madd_seg(KeysDev keys, const FilterDesc *__restrict__ filt,
                                                    const uint64_t *__restrict__ seg_off, uint32_t nseg, uint32_t lgs,
                                                    uint32_t tile, uint64_t segmax, uint8_t *__restrict__ out_new,
                                                    unsigned long long *__restrict__ seg_counts,
                                                    uint32_t *__restrict__ big, FilterDesc single) {
    extern __shared__ unsigned long long s_dyn[];
    const uint32_t S = 1u << lgs, smask = S - 1u;
    unsigned long long *BT = s_dyn;              // bit << 32 | smallest position in the segment; ~0 empty
    uint32_t *WK = (uint32_t *)(BT + S);         // word index; ~0 empty
    uint32_t *WV = WK + S;                       // old word | zero bits
    __shared__ uint32_t s_red[8];
    const uint32_t tid = threadIdx.x, lane = tid & 63u, wave = tid >> 6;
    for (uint32_t sg = blockIdx.x; sg < nseg; sg += gridDim.x) {
        const uint64_t a = filt ? seg_off[sg] : 0, b = filt ? seg_off[sg + 1] : keys.n;
        if (b - a > segmax) {  // uniform: left to the chunked path
            if (tid == 0 && big) atomicOr(big, 1u);
            continue;
        }
        if (b == a) continue;
        const FilterDesc f = filt ? filt[sg] : single;
        uint32_t maxidx = 0, nnew = 0;
        uint64_t h1 = 0, h2 = 0;  // the key's hash, computed before the previous tile's store wait
        if (tid < tile && a + tid < b) hash_key<KLEN>(keys, a + tid, h1, h2);
        for (uint64_t base = a; base < b; base += tile) {
            const uint64_t i = base + tid;
            const bool act = tid < tile && i < b;
            const uint32_t pos = (uint32_t)(i - a);
            uint32_t idxs[KMAX], word[KMAX], zm = 0;
            // the gathers go out first and the tables are cleared under their latency (the barrier then
            // waits for both; r05 cleared, synchronised, then gathered)
            if (act) {
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
            }
            for (uint32_t q = tid; q < S; q += blockDim.x) {
                BT[q] = ~0ULL;
                WK[q] = ~0u;
                WV[q] = 0u;
            }
            __syncthreads();
            if (act) {
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
            // the next tile's hash while this tile's stores drain
            if (tid < tile && base + tile + tid < b) hash_key<KLEN>(keys, base + tile + tid, h1, h2);
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

template <int KLEN, int KMAX>
static void launch_madd_seg_km(const MaddSegArgs &a, hipStream_t st) {
    const uint32_t lgs = 12;  // 2^12 slots per table, 16 B each: 64 KiB of LDS, two workgroups per CU
    const uint32_t tile = std::min<uint32_t>(256, (5u << (lgs - 3)) / std::max<uint32_t>(a.kmax, 1));  // <= 0.625 load
    hipLaunchKernelGGL((k_madd_seg<KLEN, KMAX>), dim3(a.filt ? std::min<uint32_t>(a.nseg, a.grid) : 1u), dim3(256), (size_t)16 << lgs, st,
                       a.keys, a.filt, a.seg_off, a.filt ? a.nseg : 1u, lgs, tile, a.segmax, a.out_new, a.seg_counts, a.big,
                       a.single);
}

template <int KLEN>
static void launch_madd_seg_len(const MaddSegArgs &a, hipStream_t st) {
    if (a.kmax <= 8) launch_madd_seg_km<KLEN, 8>(a, st);
    else launch_madd_seg_km<KLEN, 16>(a, st);
}

void launch_madd_seg(const MaddSegArgs &a, int klen_fast, hipStream_t st) {
    switch (klen_fast) {
    case 16: launch_madd_seg_len<16>(a, st); break;
    case 32: launch_madd_seg_len<32>(a, st); break;
    case 64: launch_madd_seg_len<64>(a, st); break;
    default: launch_madd_seg_len<0>(a, st); break;
    }
}

}  // namespace rbx
