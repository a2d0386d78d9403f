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
/* Process-wide tuning knobs: "contains_stage1" = early-exit width of contains
 * (0 = all k gathers at once; 1..3 = test that many bits first).  Results never change. */
int rbx_tune(const char *key, int value);
#ifdef __cplusplus
}
#endif
#endif
