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
/* Process-wide tuning knobs (results never change):
 *   "contains_stage1"    early-exit schedule of contains: 0 = all k gathers at once,
 *                        1..3 = that many bits first, 4 = doubling 1,2,4,... (default)
 *   "contains_partition" region-bucketed contains for one large filter: 0 never (default),
 *                        1 always (k in [2,16]), 2 auto (bitmap > 16 MiB and >= 1M keys) */
int rbx_tune(const char *key, int value);
#ifdef __cplusplus
}
#endif
#endif
