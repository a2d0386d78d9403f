/*
 * rbx_bench.h -- measurement helpers exported by librbx.so (used by bench.py).
 */
#ifndef RBX_BENCH_H
#define RBX_BENCH_H
#include <stdint.h>
#include "rbx.h"
#ifdef __cplusplus
extern "C" {
#endif
/* Random-gather roofline probe: nkeys x k independent 4-byte loads at pseudo-random
 * offsets of a device table of table_bytes (k = 7 or 10), the contains kernel's access
 * pattern without the hashing.  Enqueued on `stream` (NULL = context stream). */
int rbx_bench_gather(rbx_ctx *ctx, const void *d_table, uint64_t table_bytes, uint64_t nkeys, uint32_t k,
                     void *d_sink, void *stream);
/* Region-local gather probe: nlanes x 6 random 4-byte loads, each workgroup confined to
 * region_bytes-sized regions assigned round-robin by blockIdx % 8 (XCD affinity). */
int rbx_bench_gather_regions(rbx_ctx *ctx, const void *d_table, uint64_t table_bytes, uint64_t region_bytes,
                             uint64_t nlanes, unsigned grid, void *d_sink, void *stream);
/* Slice-probe roofline: nbuckets buckets of per_bucket 8-byte entries {word offset, payload}
 * (device, [bucket][per_bucket]); bucket b's entries each test one word of the bitmap slice
 * b * slice_bytes (a power of two); workgroups take buckets by blockIdx % 8 (XCD affinity). */
int rbx_bench_slice_probe(rbx_ctx *ctx, const void *d_entries, uint64_t per_bucket, uint32_t nbuckets,
                          const void *d_bitmap, uint64_t slice_bytes, unsigned grid, void *d_sink, void *stream);
/* Region-pass phase times of the partitioned add, summed over every block's wave 0 since the
 * last read (s_memtime ticks; collected only in the profiling build librbx_diag.so while
 * rbx_tune("add_partition_diag") has bit 64; all zero in librbx.so):
 * copies n <= 16 counters to host `out` and zeroes them. */
int rbx_bench_add_stamps(rbx_ctx *ctx, unsigned long long *out, uint32_t n);
/* Stream-read roofline probe: reads `bytes` (16-byte aligned buffer) with 16-byte loads. */
int rbx_bench_stream_read(rbx_ctx *ctx, const void *d_buf, uint64_t bytes, void *d_sink, void *stream);
/* Stream-write roofline probe: writes `bytes` (16-byte aligned buffer) with 16-byte nontemporal
 * stores (whole 64-byte write requests). */
int rbx_bench_stream_write(rbx_ctx *ctx, void *d_buf, uint64_t bytes, void *stream);
/* Segment-local gather probe (the locality of a multi-tenant batch): key i belongs to segment
 * i / keys_per_segment, a consecutive segment_bytes slice of the table (wrapping), and does 4
 * random 4-byte loads inside it. */
int rbx_bench_gather_segments(rbx_ctx *ctx, const void *d_table, uint64_t table_bytes, uint64_t segment_bytes,
                              uint64_t keys_per_segment, uint64_t nkeys, void *d_sink, void *stream);
/* The ordered stream's 8-byte first-setter entry layout of the context's last rbx_bloom_stream[_dev]
 * call: out[0] = bb (bitmap-index bits of the call's largest filter), out[1] = fbits (filter-id
 * bits), out[2] = pb = 64 - bb - fbits (chunk-position bits; 0 when the 16-byte table ran),
 * out[3] = commands per chunk.  Tests pin the production packing with it. */
int rbx_bench_stream_geometry(rbx_ctx *ctx, uint64_t *out);
/* Process-wide tuning knobs: the whole whitelist (r06).  No knob of librbx.so changes an answer: each
 * selects between exact paths (the fallbacks the engine takes by itself on other shapes, forced so the
 * tests cover them), or sets a grid, chunk or capacity.  Knobs are atomics; a call reads each once.
 *   "contains_stage1"       early-exit schedule of contains: 0 = all k gathers at once,
 *                           1..3 = that many bits first, 4 = doubling 1,2,4,... (default),
 *                           5 = per-lane key slots (one bit per key per round trip)
 *   "contains_multi_slots"  multi-tenant contains with key slots: 0 never, 1 always,
 *                           2 auto (default: the call's bitmaps exceed 64 MiB)
 *   "contains_qgrid"        slot contains kernel grid, 256..8192 (default 2048)
 *   "contains_partition"    region-bucketed contains for one large filter: 0 never, 1 always
 *                           (k in [2,16]), 2 auto (default: bitmap >= 256 MiB, >= 4M keys)
 *   "add_partition"         region-partitioned add: 0 never, 1 always, 2 auto (default:
 *                           bitmap >= 8 MiB and >= max(2^17, bits / 2^12) keys)
 *   "add_records"           how the partitioned add reports new keys: 0 owner bits, 1 non-owner
 *                           counters, 3 owner records, 2 (default) chosen from the sampled fill
 *   "add_region_grid"       partitioned add, region-pass blocks in [256, 65536] (default 2048)
 *   "add_rec_lds_limit"     owner records a region block stages in LDS, 0..7168 (default 7168;
 *                           tests use small limits to run the direct-report fallback)
 *   "add_multi_table8"      multi-tenant add when (filter id, bit) fits 41 bits and k <= 32: 2 (default)
 *                           optimistic SETBITs (returning atomicOr) with a small conflict table for the
 *                           zero bits two keys share; 0 the 16-byte first-setter table (the fallback)
 *   "add_multi_conflict_log2"  entries (log2, 6..24, default 17) of that conflict table; past half full
 *                           the chunk's replies come from the full first-setter table
 *   "add_multi_segment"     1 (default): a multi-tenant add whose filters are all distinct runs each
 *                           segment of <= add_multi_segmax keys in one workgroup (k_madd_seg: tiles of
 *                           <= 256 keys, LDS first setters, plain word stores), longer ones on the path
 *                           above; 0: off
 *   "add_multi_segmax"      that segment-length limit (keys, 1..16384)
 *   "add_multi_seg_grid"    the per-segment kernel's workgroups, 64..65536 (default 8192), grid-stride
 *                           over the segments
 *   "stream_table8"         ordered stream's first-setter table: 1 (default) 8-byte entries claimed
 *                           by one CAS and committed by a table walk, 0 the 16-byte epoch-tagged table
 *                           (the fallback when (filter id, bit) does not fit 41 bits)
 *   "stream_chunk"          commands per chunk cap (0 = default) of the ordered stream (default: with
 *                           the 8-byte table min(2^pb - 1, 2^27 / k) rounded down to 128, else 2^26 / k)
 *                           and of the chunked multi-tenant add (default min(2^pb - 1, 2^27 / k), not
 *                           rounded)
 *   "stream_qgrid"          ordered-stream slot contains kernel grid, 256..8192 (default 1024)
 *   "stream_final_grid"     ordered stream: k_stream_final8 blocks, 32..2048 (default 512: each block
 *                           adds its count to one counter, and those atomics serialise)
 *   "wide_subchunk"         add / contains on a filter past 2^32 bits: keys per sub-chunk cap (0 =
 *                           default 2^29 / k, which bounds the first-setter table at 2^30 entries)
 *   "host_small_batches"    1 (default): host-arena add/contains batches within host_small_bytes
 *                           take the one-transfer path (pinned copy, one upload, one readback);
 *                           0: every host batch on the pipelined copy-stream path
 *   "host_small_bytes"      that path's limit: key bytes (+ offsets), 4 KiB .. 64 MiB (default
 *                           4 MiB; at most a quarter as many keys)
 *   "host_tiny_keys"        host-arena batches of at most this many keys (0..16384, default 16384)
 *                           and 64 KiB of key bytes run from coherent pinned memory: the kernel reads
 *                           the keys over the host link and writes the flags back, one launch and one
 *                           sync (adds also within add_single_seg_keys); 0: the one-transfer path
 *   "add_single_seg_keys"   single-filter adds of at most this many keys with k <= 16 (0..16384,
 *                           default 256) run the per-segment kernel on one segment (one launch, first
 *                           setters in LDS) instead of the table path; 0: the table path
 *   "add_one_key"           1 (default): a one-key single-filter add with k <= 16 takes
 *                           k_bloom_add_one (one lane, no first-setter table); 0: as above
 *   "host_tiny_spin"        1 (default): a one-key host add/contains (k <= 16) spins on its kernel's
 *                           completion word in the pinned block (2 ms, then a stream sync);
 *                           0: a stream sync
 * Profiling build only (librbx_diag.so, `make diag`; librbx.so rejects them): "stream_diag",
 * "contains_partition_flags", "add_partition_diag" -- timing diagnostics that make answers wrong
 * (rbx_kernels.h kDiag).  Removed in r06 with the variants they selected (measured slower, never
 * default; the A/B records stay in profiles/): contains_qshape, contains_partials, contains_emit2_nt,
 * contains_stage1_per, add_region_kernel, add_rebucket_lines, add_rebucket_prefetch,
 * add_stage1_prefetch, add_multi_seg_lgs, stream_prefilter, stream_occupancy, stream_table_scale,
 * stream_contains_slots, stream_contains_lds, stream_owner, stream_lookup_rounds, stream_probe_batch,
 * walk_reset_all, add_multi_table8 1. */
int rbx_tune(const char *key, int value);
/* Test hook (fault injection): the next n Bloom adds that the node runs on GPU `gpu` (single or
 * multi-tenant, replica or home) fail with RBX_E_DEVICE before they touch the device; n = 0 clears.
 * Exercises the replicated-add failure semantics of rbx_node_bloom_replicate. */
int rbx_node_test_fail_adds(rbx_node *node, int gpu, int n);
#ifdef __cplusplus
}
#endif
#endif
