/*
 * rbx_selftest.h -- test-only exports of librbx.so: the device primitives compiled
 * for the host, so CPU tests can check them without a GPU (tests/test_selftest.py).
 */
#ifndef RBX_SELFTEST_H
#define RBX_SELFTEST_H
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif
/* mismatches of the divide-free 63-bit modulo against '%' over n random (h, size) pairs x16 */
uint64_t rbx_selftest_mod(uint64_t n, uint64_t seed);
/* HighwayHash128 (Redisson KEY) through the host-compiled device code path */
void rbx_selftest_hash128(const uint8_t *data, uint64_t len, uint64_t out[2]);
/* BigDecimal.valueOf(d).toPlainString() (the stored falseProbability string); returns length */
int rbx_selftest_plain_string(double d, char *out, int cap);
#ifdef __cplusplus
}
#endif
#endif
