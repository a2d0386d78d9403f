// rbx_kernels.h -- shared device structs and kernel launchers (host <-> .hip files).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "rbx_device.h"

namespace rbx {

constexpr unsigned kMaxGrid = 2048;  // grid-stride cap: 256 CUs x 8 blocks of 256 threads

// Diagnostic switches that make answers wrong (timing A/Bs: rbx_tune "stream_diag",
// "contains_partition_flags", "add_partition_diag") exist only in the profiling build
// librbx_diag.so (`make diag`: -DRBX_DIAG=1, used by tools/ through RBX_LIB_PATH).  In librbx.so
// kDiag is false: every kernel zeroes its diag argument on entry, so those branches are compiled
// out, and rbx_tune rejects the keys.
#ifndef RBX_DIAG
#define RBX_DIAG 0
#endif
constexpr bool kDiag = RBX_DIAG != 0;  // grid-stride cap: 256 CUs x 8 blocks of 256 threads

struct KeysDev {
    const uint8_t *bytes;
    const uint64_t *offsets;  // nullable: fixed stride
    uint64_t stride;
    uint64_t n;
    uint64_t off_base;        // subtracted from offsets[] (a slice of a larger arena)
};

// One Bloom filter as the kernels see it (device-resident table for multi-tenant calls).
struct FilterDesc {
    uint32_t *bm;                   // bitmap words (Redis string bytes, MSB-first)
    unsigned long long *redis_len;  // device word: Redis string length in bytes
    ModParams mp;
    uint32_t k;
    uint32_t fid;  // identity in the first-setter table (unique per filter within a call)
};

// The per-filter fields a probing kernel reads, in one 32-byte line-aligned record (FilterDesc is 56
// bytes with the 64-bit modulus and the Redis-length pointer): the ordered stream's contains reads
// one per command of a random (Zipf) tenant.
struct alignas(32) ProbeDesc {
    const uint32_t *bm;
    ModC mc;
    uint32_t k;
    uint32_t fid;
};
static_assert(sizeof(ProbeDesc) == 32, "one half line");

struct alignas(16) HTEntry {
    unsigned long long tag;  // [63:56] epoch, [55:32] fid, [31:0] bit index
    unsigned long long idw;  // [63:32] 254 - epoch, [31:0] min key id
};

struct AddChunkArgs {
    KeysDev keys;
    uint64_t base, nchunk;
    const FilterDesc *filt;  // nullable: single filter
    const uint64_t *seg_off;
    uint32_t nseg;
    const uint32_t *tile_seg0;
    FilterDesc single;
    HTEntry *table;
    uint32_t log2cap, epoch;
    uint32_t *zmask;  // nchunk words (k <= 32) or nchunk*k bytes
    uint32_t kmax;
    uint8_t *out_new;
    unsigned long long *count;
    unsigned long long *seg_counts;
    bool narrow;  // single filter, k <= 32: 8-byte entries, table cleared per chunk
};

// partitioned contains (contains_partitioned.hip): one chunk of keys against one filter
constexpr int kBkRegionBits = 19;  // 2^19 bits = 64 KiB bitmap region = one LDS image
#ifndef RBX_BK_SUB
#define RBX_BK_SUB 16
#endif
constexpr uint32_t kBkSub = RBX_BK_SUB;  // sub-partitions (own counters) per coarse bucket
#ifndef RBX_BA_SUB
#define RBX_BA_SUB 8
#endif
constexpr uint32_t kBaSub = RBX_BA_SUB;  // the partitioned add's stage-1 sub-partitions per level-1 bucket
constexpr int kBkMissRangeBits = 19;  // probe misses are bucketed by 2^19-key range (64 KiB LDS bitmap)
struct PcArgs {
    KeysDev keys;
    uint64_t base, nchunk;
    const uint32_t *bm;
    ModParams mp;
    uint32_t k;
    uint32_t nregions;      // ceil(size / 2^kBkRegionBits)
    uint32_t fb;            // regions per coarse bucket = 2^fb
    uint32_t cshift;        // kBkRegionBits + fb
    uint32_t ncoarse;       // <= 64
    uint64_t cap1, cap2;    // pair capacity per coarse sub-partition / per region
    uint64_t nwords4;       // bitmap words rounded up to a multiple of 4
    uint32_t *cnt1;         // ncoarse * kBkSub, zeroed
    uint32_t *cnt2;         // nregions, zeroed
    unsigned long long *alive;  // ceil(nchunk/64)
    unsigned long long *miss;   // ceil(nchunk/64), zeroed
    uint32_t *mrec;         // nmranges * capm: key ids of the probe's clear bits, by 2^19-key range
    uint32_t *mcnt;         // nmranges, zeroed
    uint64_t capm;
    uint32_t nmranges;      // ceil(nchunk / 2^kBkMissRangeBits) <= 256
    unsigned long long *pairs1; // ncoarse * kBkSub * cap1
    uint32_t *p2lo;         // nregions * cap2: region offset << 13 | key bits 0-12
    uint16_t *p2hi;         // nregions * cap2: key bits 13-26
    uint8_t *out;
    unsigned long long *count;
    uint32_t flags;  // diagnostics only (rbx_tune "contains_partition_flags"); 0 in normal operation
    unsigned long long *stamps;  // flags & 64: emit2 / probe phase times (rbx_bench_add_stamps), else null
};
// k_bk_final's blocks: each adds its count to ONE counter, and same-address atomics serialise at the
// kernel's end, so 512 blocks (grid-stride) rather than 2048 (r05, cf. k_stream_final8)
inline unsigned grid_for_pc(uint64_t n) {
    uint64_t g = ((n + 63) / 64 + 255) / 256;
    return (unsigned)(g < 1 ? 1 : (g > 512 ? 512 : g));
}
void launch_contains_partitioned_chunk(const PcArgs &a, int klen_fast, hipStream_t st);
void set_add_region_grid(int v);  // 256..65536 (default 2048)
void set_add_rec_lds_limit(int v);  // 0..7168 (tests)

// partitioned single-filter add (add_partitioned.hip): one chunk of keys
// Partitioned add: 2^16-bit regions (8 KiB bitmap + two bitsets + a collision table = 32 KiB
// of LDS, two blocks per CU); at most 8 pairs per thread of the 1024-thread region block.
constexpr int kBaRegionBits = 16;
constexpr uint32_t kBaMaxRegionPairs = 8192;  // cap3 <= this
constexpr int kBaKeyRangeBits = 20;           // owner records are bucketed by 2^20-key range
struct BaArgs {
    KeysDev keys;
    uint64_t base, nchunk;
    FilterDesc f;                 // bm, redis_len, mp, k
    uint32_t ncoarse;             // level-1 buckets (<= 256, each kBkSub sub-partitions)
    uint32_t s1, s3;              // level-1 bucket = idx >> s1, region = idx >> s3 (s3 = kBaRegionBits)
    uint32_t f3;                  // fan-out bits of the rebucket (level 1 -> regions), <= 8
    uint32_t nregions;
    uint64_t cap1, cap3;
    unsigned long long *p1, *p3;  // level-1 and region pair arrays
    uint32_t *cnt1, *cnt3;        // zeroed per chunk
    uint32_t *new_bits;           // ceil(nchunk / 32) words, zeroed per chunk
    uint32_t *ctr;                // byte counter per key (nchunk rounded up to 32), all zero between calls
    uint32_t *recs, *rec_cnt;     // owner records: nranges x cap_rec key ids, counts (zeroed per chunk)
    uint64_t cap_rec;             // k x 2^20: a range's records never exceed it
    uint32_t nranges;             // 2^20-key ranges of the chunk
    uint32_t *overflow;           // zeroed; set when a pair does not fit (the chunk then reruns on the table path)
    uint32_t *mode;               // written by k_ba_mode: 1 non-owner counters, 2 owner records, 0 owner bits
    uint32_t record_policy;       // rbx_tune "add_records": 0 owner bits, 1 counters, 3 owner records, 2 from the sampled fill
    uint64_t nwords4;             // bitmap words rounded up to a multiple of 4
    uint8_t *out_new;
    unsigned long long *count;
    uint32_t diag;                // diagnostics only (rbx_tune "add_partition_diag"); 0 in normal operation
    unsigned long long *stamps;   // diagnostics only (add_partition_diag & 64): region-pass phase times, else null
};
void launch_add_partitioned_chunk(const BaArgs &a, int klen_fast, hipStream_t st);

// ordered mixed contains/add stream (one chunk of keys)
struct StreamChunkArgs {
    KeysDev keys;
    uint64_t base, nchunk;
    const FilterDesc *filt;
    const ProbeDesc *pdesc;  // the same filters' probe fields (stream contains)
    const uint32_t *kf;   // per key: index into filt
    const uint8_t *op;    // per key: 0 contains, 1 add
    HTEntry *table;
    uint32_t log2cap, epoch;
    uint32_t *zmask;      // per add-list entry
    uint32_t kmax;
    uint8_t *out;         // per key: present (contains) / newly added (add)
    unsigned long long *counts;  // [0] present contains, [1] new adds
    uint32_t *adds;       // nchunk: compacted chunk-local positions of the adds
    uint32_t *nadds;      // 1, zeroed per chunk
    // r04 first-setter table of 8-byte entries (null: the 16-byte epoch-tagged `table` above).
    // entry = (fid << bb | bit) << pb | chunk position, EMPTY = ~0; one CAS claims a bit, and an
    // atomicMin keeps the first setter of a shared one.  Capacity 2^t8_log2(*nadds, kmax), from the
    // chunk's add count on the device; k_stream_walk commits it and restores every entry to EMPTY.
    unsigned long long *t8;
    uint32_t bb, pb;              // bits of the largest bitmap's bit index / of a chunk position
    uint32_t tkmax;               // sizes the table: 2^t8_log2(*nadds, tkmax), tkmax = kmax x table scale
    uint32_t *const *fid_bm;      // bitmap words per table id (fid)
    uint32_t *fslot;              // per add-list entry: the table slot of its first zero bit's claim (r05)
};
// state of the optimistic multi-tenant add's conflict table (k_maddx_*), reset per chunk
struct MaddxState {
    uint32_t count;     // entries inserted into C
    uint32_t overflow;  // C too full (or a probe run too long): the full table T decides the chunk
};
// One chunk of a multi-tenant add on the 8-byte first-setter table (r05, bloom_kernels.hip k_madd_*):
// probe (claims) -> final (replies, per-segment counts) -> walk (OR owned bits, empty the table).
struct MaddChunkArgs {
    KeysDev keys;
    uint64_t base, nchunk;
    const FilterDesc *filt;
    const uint64_t *seg_off;
    uint32_t nseg;
    const uint32_t *tile_seg0;
    uint32_t kmax;
    unsigned long long *t8;   // 2^lg entries, EMPTY before and after the chunk
    uint32_t lg, bb, pb;
    uint32_t *const *fid_bm;  // bitmap words per filter id
    uint32_t *zmask, *fslot;  // per key of the chunk
    uint8_t *out_new;
    unsigned long long *seg_counts;
    // r05 optimistic SETBITs with conflict repair (k_maddx_*): non-null = that path, with the small
    // conflict table C of 2^lgC entries and its state word; t8 / lg then serve only an overflowed chunk
    unsigned long long *c8;
    uint32_t lgC;
    MaddxState *cst;
    // r05 per-segment path (k_madd_seg) in front: non-null = every k_maddx_* kernel returns unless *big
    // (a segment past segmax exists), and handles only the keys of such segments
    const uint32_t *big;
    uint64_t segmax;
};
void launch_madd8_chunk(const MaddChunkArgs &a, int klen_fast, hipStream_t st);
// per-segment multi-tenant add (segment_add.hip k_madd_seg): one 256-thread workgroup per segment, every
// filter of the batch in one segment only (disjoint bitmaps), k <= 16; segments past segmax (<= kSegMaxKeys)
// keys set *big and are left to the k_maddx_* chunks
constexpr uint32_t kSegMaxKeys = 16384;
struct MaddSegArgs {
    KeysDev keys;
    const FilterDesc *filt;
    const uint64_t *seg_off;
    uint32_t nseg, kmax;
    uint32_t grid;            // workgroups (grid-stride over the segments)
    uint64_t segmax;
    uint8_t *out_new;
    unsigned long long *seg_counts;
    uint32_t *big;            // zeroed before the launch
    // filt == nullptr: one filter passed by value and one segment, all of `keys` (seg_off unused; the
    // small single-filter adds of run_add and bloom_host_tiny, keys.n <= segmax)
    FilterDesc single;
};
void launch_madd_seg(const MaddSegArgs &a, int klen_fast, hipStream_t st);
// entries of the 8-byte stream table for a chunk of nadds adds (load <= 8/9 even if every bit is 0)
__host__ __device__ inline uint32_t t8_log2(uint32_t nadds, uint32_t kmax) {
    const uint64_t need = (uint64_t)nadds * kmax;
    const uint64_t want = need + need / 8;
    uint32_t lg = 12;
    while ((1ULL << lg) < want) ++lg;
    return lg;
}

// bloom_kernels.hip
void launch_stream_chunk(const StreamChunkArgs &a, int klen_fast, hipStream_t st);
void launch_bloom_contains(const KeysDev &keys, int klen_fast, const uint32_t *bm, const ModParams &mp,
                           uint32_t k, uint8_t *out, unsigned long long *count, hipStream_t st);
// add(T) / contains(T): one key of one filter (k <= 16), one lane; an add needs no first-setter table
// (run_add, keys.n == 1).  done (nullable): seq is stored there last, at system scope (bloom_host_tiny)
void launch_bloom_one(bool add, const KeysDev &keys, int klen_fast, const FilterDesc &f, uint8_t *out,
                      unsigned long long *count, uint32_t *done, uint32_t seq, hipStream_t st);
// one store of seq into done (coherent host memory), after the stream's earlier work
void launch_done_word(uint32_t *done, uint32_t seq, hipStream_t st);
// tile_seg0[t] = segment holding key 256*t (precomputed once per multi-tenant batch)
void launch_tile_seg0(const uint64_t *seg_off, uint32_t nseg, uint64_t nkeys, uint32_t *tile_seg0, hipStream_t st);
void launch_bloom_contains_multi(const KeysDev &keys, int klen_fast, const FilterDesc *filt,
                                 const uint64_t *seg_off, uint32_t nseg, const uint32_t *tile_seg0, uint32_t kmax,
                                 uint8_t *out, unsigned long long *counts, hipStream_t st, bool slots);
void launch_bloom_add_chunk(const AddChunkArgs &a, int klen_fast, hipStream_t st);
// |size| > 2^32 filters (k_wide_*): add = first-setter claim + resolve over a 2^tlog2-entry table
// (all ~0 on entry); *oob = 1 when an index passes the Redis offset limit.  bm may be NULL for
// contains (a missing key).
void launch_bloom_wide(const KeysDev &keys, uint64_t m, uint32_t k, uint32_t *bm, unsigned long long *len,
                       unsigned long long *table, uint32_t tlog2, bool is_add, uint8_t *out,
                       unsigned long long *count, unsigned long long *oob, hipStream_t st);
void launch_bitcount(const uint8_t *bytes, uint64_t nbytes, unsigned long long *out, hipStream_t st);
// order-independent digest of a Redis string's bytes (replica comparison); *out += digest
void launch_digest(const uint8_t *bytes, uint64_t nbytes, unsigned long long *out, hipStream_t st);
// region-local gathers: 6 loads per lane inside XCD-assigned regions (partitioned-probe roofline)
void launch_gather_regions(const uint32_t *tbl, uint64_t nwords, uint64_t region_words, uint64_t total_lanes,
                           uint32_t *sink, hipStream_t st, unsigned grid);
// 4 random 4-byte gathers per key inside the key's segment (keys_per_seg consecutive keys share
// one seg_words slice): the request roofline of multi-tenant batches at their locality
void launch_gather_segments(const uint32_t *tbl, uint64_t nwords, uint64_t seg_words, uint64_t keys_per_seg,
                            uint64_t nkeys, uint32_t *sink, hipStream_t st);
// slice-probe roofline: per bucket b, stream 8-byte entries and test one word of bitmap slice b
void launch_bench_slice_probe(const void *ent, uint64_t per_bucket, uint32_t nbuckets, const uint32_t *bm,
                              uint32_t slice_words_log2, unsigned grid, uint32_t *sink, hipStream_t st);
// streaming 16-byte reads of a whole buffer: the HBM stream-read roofline probe
void launch_stream_read(const void *buf, uint64_t bytes, uint32_t *sink, hipStream_t st);
void launch_stream_write(void *buf, uint64_t bytes, hipStream_t st);
// random 4-byte gathers (k per key, nkeys keys) over an nwords-word table: roofline probe
void launch_gather_probe(const uint32_t *tbl, uint64_t nwords, uint64_t nkeys, uint32_t k, uint32_t *sink,
                         hipStream_t st);

void set_contains_stage1(int v);
void set_contains_qgrid(int v);
void set_stream_diag(int v);           // profiling build only (kDiag): bits 1 | 8, see stream_kernels.hip
void set_stream_final_grid(int v);  // k_stream_final8 blocks (32..2048)
void set_stream_qgrid(int v);  // slot stream-contains kernel grid (blocks)
int get_contains_stage1();

// hll_kernels.hip
struct HllSeg {
    uint8_t *regs;      // 16384 u8 registers
    uint64_t begin;     // element range [begin, end)
    uint64_t end;
    uint32_t seg;       // command index (for the changed flag)
    uint32_t pad;
};
void launch_hll_pfadd(const KeysDev &elems, int elen_fast, const HllSeg *d_tiles, uint32_t ntiles,
                      uint32_t *d_changed, hipStream_t st);
// Per-HLL histogram + Redis estimator; out[i] = count, or ~0 when the hllTau branch
// (a register == 51) must be evaluated on the host with glibc pow.  histo: n*64 ints.
void launch_hll_count(uint8_t *const *d_regs, uint32_t n, int *d_histo, unsigned long long *d_out,
                      hipStream_t st);
// dst = max(dst, src_0..src_{n-1}) over 16384 registers
void launch_hll_merge(uint8_t *dst, uint8_t *const *d_srcs, uint32_t nsrc, hipStream_t st);
// raw registers -> scratch union: out = max over a set of HLLs (multi-key PFCOUNT)
void launch_hll_union(uint8_t *const *d_srcs, uint32_t nsrc, uint8_t *out, hipStream_t st);
// Redis sparse HLL strings kept as redis-server builds them ([redis-7.2] hyperloglog.c
// hllSparseSet, replayed in command order): one u16 per opcode -- ZERO and VAL opcodes are their
// byte, XZERO is (byte0 << 8 | byte1) -- so ZERO < 0x40 <= VAL < 0x100 <= XZERO.
struct HllReplay {
    uint16_t *ops;        // the HLL's opcode list (capacity >= max(its bytes, 3000): opcodes <= bytes)
    uint32_t *state;      // [0] promoted (sticky: the list is stale once set), [1] opcodes (0 = the
                          // createHLLObject string, one XZERO), [2] opcode bytes (after the header)
    const uint8_t *regs;  // merge mode (PFMERGE write-back): the max registers, ascending; else null
    uint64_t begin, end;  // PFADD mode: the command's elements, in order
    const uint8_t *final_regs;  // the registers after the update (PFADD: the key's, merged already)
};
// one block per item; items whose HLL is already promoted return at once
void launch_hll_sparse_replay(const KeysDev &elems, int elen_fast, const HllReplay *items, uint32_t n,
                              uint64_t max_bytes, hipStream_t st);
// zero n pool slots: 16384 register bytes and 4 state words each (kHllStateWords)
void launch_hll_zero(uint8_t *const *d_regs, uint32_t *const *d_state, uint32_t n, hipStream_t st);
// buf[i*16384..] = regs[i] (pack) or regs[i] = max(regs[i], buf[i*16384..]) (unpack_max)
void launch_hll_pack(uint8_t *const *d_regs, uint32_t n, uint8_t *buf, bool unpack_max, hipStream_t st);

}  // namespace rbx
