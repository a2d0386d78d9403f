/* abi_client.c -- a plain C host of librbx.so (no Python, no torch): the way a
 * cgo/JNI/FFM binding drives the engine.  Replays T/RedissonBloomFilterTest.java
 * testContainsAll/testAddAll/testConfig and T/RedissonHyperLogLogTest.java testMerge
 * through include/rbx.h only.  Exit code 0 = all checks passed. */
#include <stdio.h>
#include <stdint.h>
#include <string.h>
#include "rbx.h"

#define CHECK(c) do { if (!(c)) { fprintf(stderr, "FAIL %s:%d %s (%s)\n", __FILE__, __LINE__, #c, rbx_last_error()); return 1; } } while (0)

static rbx_keys arena(const char **keys, int n, uint8_t *buf, uint64_t *offs) {
    uint64_t o = 0;
    for (int i = 0; i < n; ++i) {
        offs[i] = o;
        memcpy(buf + o, keys[i], strlen(keys[i]));
        o += strlen(keys[i]);
    }
    offs[n] = o;
    rbx_keys k = {buf, offs, 0, (uint64_t)n};
    return k;
}

int main(void) {
    rbx_ctx *ctx;
    CHECK(rbx_init(0, &ctx) == RBX_OK);
    uint8_t buf[256];
    uint64_t offs[16], c = 0;
    int created = 0;

    /* testConfig */
    CHECK(rbx_bloom_try_init(ctx, "filter", 100, 0.03, &created) == RBX_OK && created == 1);
    rbx_bloom_config cfg;
    CHECK(rbx_bloom_read_config(ctx, "filter", &cfg) == RBX_OK);
    CHECK(cfg.size == 729 && cfg.hash_iterations == 5 && cfg.expected_insertions == 100);
    CHECK(strcmp(cfg.false_probability_str, "0.03") == 0);
    CHECK(rbx_bloom_try_init(ctx, "filter", 101, 0.03, &created) == RBX_OK && created == 0);

    /* testContainsAll + testAddAll */
    const char *l123[] = {"1", "2", "3"}, *l15[] = {"1", "5"};
    rbx_keys k123 = arena(l123, 3, buf, offs);
    CHECK(rbx_bloom_contains(ctx, "filter", 729, 5, &k123, NULL, &c) == RBX_OK && c == 0);
    CHECK(rbx_bloom_add(ctx, "filter", 729, 5, &k123, NULL, &c) == RBX_OK && c == 3);
    CHECK(rbx_bloom_add(ctx, "filter", 729, 5, &k123, NULL, &c) == RBX_OK && c == 0);
    CHECK(rbx_bloom_contains(ctx, "filter", 729, 5, &k123, NULL, &c) == RBX_OK && c == 3);
    int64_t cnt = 0;
    CHECK(rbx_bloom_count(ctx, "filter", &cnt) == RBX_OK && cnt == 3);
    rbx_keys k15 = arena(l15, 2, buf, offs);
    CHECK(rbx_bloom_contains(ctx, "filter", 729, 5, &k15, NULL, &c) == RBX_OK && c == 1);
    CHECK(rbx_bloom_add(ctx, "filter", 729, 5, &k15, NULL, &c) == RBX_OK && c == 1);
    CHECK(rbx_bloom_count(ctx, "filter", &cnt) == RBX_OK && cnt == 4);

    /* error classes */
    rbx_keys empty = {buf, offs, 0, 0};
    offs[0] = 0;
    CHECK(rbx_bloom_add(ctx, "filter", 729, 5, &empty, NULL, &c) == RBX_E_ARITHMETIC);
    CHECK(rbx_bloom_add(ctx, "filter", 730, 5, &k15, NULL, &c) == RBX_E_CONFIG_CHANGED);
    CHECK(rbx_bloom_contains(ctx, "nope", 0, 0, &k15, NULL, &c) == RBX_E_ILLEGAL_STATE);
    CHECK(rbx_bloom_try_init(ctx, "bad", 1, 2.0, &created) == RBX_E_ILLEGAL_ARGUMENT);

    /* testMerge */
    const char *h1[] = {"foo", "bar", "zap", "a"}, *h2[] = {"a", "b", "c", "foo", "c"};
    int ch;
    for (int i = 0; i < 4; ++i) {
        rbx_keys e = arena(&h1[i], 1, buf, offs);
        CHECK(rbx_hll_add(ctx, "hll1", &e, &ch) == RBX_OK && ch == 1);
    }
    for (int i = 0; i < 5; ++i) {
        rbx_keys e = arena(&h2[i], 1, buf, offs);
        CHECK(rbx_hll_add(ctx, "hll2", &e, &ch) == RBX_OK && ch == (i < 4));
    }
    const char *srcs[] = {"hll1", "hll2"};
    CHECK(rbx_hll_merge(ctx, "hll3", srcs, 2) == RBX_OK);
    const char *n3[] = {"hll3"};
    uint64_t pc = 0;
    CHECK(rbx_hll_count(ctx, n3, 1, &pc) == RBX_OK && pc == 6);
    CHECK(rbx_hll_count(ctx, srcs, 2, &pc) == RBX_OK && pc == 6);

    int deleted = 0;
    CHECK(rbx_bloom_delete(ctx, "filter", &deleted) == RBX_OK && deleted == 2);
    CHECK(rbx_shutdown(ctx) == RBX_OK);
    printf("abi_client: all checks passed\n");
    return 0;
}
