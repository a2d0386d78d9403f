/* ffm_replay.c -- replays, from plain C, the exact native call sequence and struct layouts of the
 * Java FFM shim written out in INTEGRATION.md §2 (GpuBloomFilter / GpuHyperLogLog / Rbx), so the
 * binding is tested without a JDK.  Every struct offset the Java StructLayouts hard-code is
 * asserted against the C compiler's, then each shim method's downcalls run in the shim's order:
 *
 *   GpuBloomFilter.tryInit      rbx_bloom_try_init_n + readConfig (rbx_bloom_read_config_n)
 *   .add / .contains (batch)    Rbx.keys arena (bytes + offsets[n+1]) -> rbx_bloom_add_n / _contains_n
 *   .count                      rbx_bloom_count_n + readConfig
 *   .getExpectedInsertions ...  rbx_bloom_read_config_n -> CONFIG fields by offset
 *   .sizeInMemoryAsync          rbx_memory_usage_n(name, {name}:config)
 *   .expire / clearExpire       rbx_pexpire_n(name, {name}:config) / rbx_persist
 *   .remainTimeToLive           rbx_pttl
 *   .renamenx / .delete         rbx_bloom_renamenx / rbx_del_n(name, {name}:config)
 *   GpuHyperLogLog.addAllAsync  rbx_hll_add_multi_async + completion upcall(user = ticket, rc)
 *   .countWithAsync             rbx_hll_count_async
 *   .mergeWithAsync             rbx_hll_merge_async
 *   (T/RedissonBloomFilterTest.java testConfig / testContainsAll, T/RedissonHyperLogLogTest.java testMerge)
 * Exit code 0 = all checks passed. */
#include <pthread.h>
#include <stddef.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "rbx.h"

#define CHECK(c)                                                                                   \
    do {                                                                                           \
        if (!(c)) {                                                                                \
            fprintf(stderr, "FAIL %s:%d %s (%s)\n", __FILE__, __LINE__, #c, rbx_last_error());     \
            return 1;                                                                              \
        }                                                                                          \
    } while (0)

/* Rbx.name(): struct rbx_name by value */
static rbx_name nm(const char *s) {
    rbx_name n = {(const uint8_t *)s, strlen(s)};
    return n;
}

/* Rbx.keys(): one off-heap arena (bytes + offsets[n+1]) in a struct rbx_keys */
static rbx_keys arena(const char **keys, int n, uint8_t *buf, uint64_t *offs) {
    uint64_t o = 0;
    for (int i = 0; i < n; ++i) {
        offs[i] = o;
        memcpy(buf + o, keys[i], strlen(keys[i]));
        o += strlen(keys[i]);
    }
    offs[n] = o;
    rbx_keys k;
    memset(&k, 0, sizeof k);
    *(const uint8_t **)((char *)&k + 0) = buf;   /* KEYS: bytes@0   */
    *(const uint64_t **)((char *)&k + 8) = offs; /*       offsets@8 */
    *(uint64_t *)((char *)&k + 16) = 0;          /*       stride@16 */
    *(uint64_t *)((char *)&k + 24) = (uint64_t)n; /*      n@24      */
    return k;
}

/* Rbx.onDone: the completion upcall; `user` is the shim's ticket */
static pthread_mutex_t g_mu = PTHREAD_MUTEX_INITIALIZER;
static int g_done[16], g_rc[16];
static void on_done(void *user, int rc) {
    const intptr_t t = (intptr_t)user;
    pthread_mutex_lock(&g_mu);
    g_done[t] = 1;
    g_rc[t] = rc;
    pthread_mutex_unlock(&g_mu);
}

int main(void) {
    /* ---- the StructLayouts of Rbx ---- */
    CHECK(sizeof(rbx_keys) == 32 && offsetof(rbx_keys, bytes) == 0 && offsetof(rbx_keys, offsets) == 8 &&
          offsetof(rbx_keys, stride) == 16 && offsetof(rbx_keys, n) == 24);
    CHECK(sizeof(rbx_bloom_config) == 96 && offsetof(rbx_bloom_config, size) == 0 &&
          offsetof(rbx_bloom_config, hash_iterations) == 8 && offsetof(rbx_bloom_config, expected_insertions) == 16 &&
          offsetof(rbx_bloom_config, false_probability) == 24 && offsetof(rbx_bloom_config, false_probability_str) == 32);
    CHECK(sizeof(rbx_name) == 16 && offsetof(rbx_name, bytes) == 0 && offsetof(rbx_name, len) == 8);

    rbx_ctx *ctx;
    CHECK(rbx_init(0, &ctx) == RBX_OK);
    uint8_t buf[256];
    uint64_t offs[16];

    /* ---- GpuBloomFilter("ffm-filter").tryInit(100, 0.03) ---- */
    const char *name = "ffm-filter", *cfg_name = "{ffm-filter}:config";
    int created = -1;
    CHECK(rbx_bloom_try_init_n(ctx, nm(name), 100, 0.03, &created) == RBX_OK && created == 1);
    unsigned char cfgmem[96]; /* Rbx.CONFIG segment, read by offset as the Java does */
    CHECK(rbx_bloom_read_config_n(ctx, nm(name), (rbx_bloom_config *)cfgmem) == RBX_OK);
    int64_t size;
    int32_t k;
    memcpy(&size, cfgmem + 0, 8);
    memcpy(&k, cfgmem + 8, 4);
    CHECK(size == 729 && k == 5);
    int64_t expected;
    memcpy(&expected, cfgmem + 16, 8);
    CHECK(expected == 100 && strcmp((const char *)cfgmem + 32, "0.03") == 0);
    CHECK(rbx_bloom_try_init_n(ctx, nm(name), 101, 0.03, &created) == RBX_OK && created == 0);

    /* ---- add / contains (batch) ---- */
    const char *l123[] = {"1", "2", "3"}, *l15[] = {"1", "5"};
    uint64_t count = 0;
    rbx_keys k123 = arena(l123, 3, buf, offs);
    CHECK(rbx_bloom_contains_n(ctx, nm(name), (uint64_t)size, (uint32_t)k, &k123, NULL, &count) == RBX_OK && count == 0);
    CHECK(rbx_bloom_add_n(ctx, nm(name), (uint64_t)size, (uint32_t)k, &k123, NULL, &count) == RBX_OK && count == 3);
    CHECK(rbx_bloom_contains_n(ctx, nm(name), (uint64_t)size, (uint32_t)k, &k123, NULL, &count) == RBX_OK && count == 3);
    rbx_keys k15 = arena(l15, 2, buf, offs);
    CHECK(rbx_bloom_contains_n(ctx, nm(name), (uint64_t)size, (uint32_t)k, &k15, NULL, &count) == RBX_OK && count == 1);
    /* an out-of-date cached config: the Java maps -3 to RedisException */
    CHECK(rbx_bloom_add_n(ctx, nm(name), 730, 5, &k15, NULL, &count) == RBX_E_CONFIG_CHANGED);
    int64_t est = 0;
    CHECK(rbx_bloom_count_n(ctx, nm(name), &est) == RBX_OK && est == 3);

    /* ---- sizeInMemoryAsync / expire / clearExpire / remainTimeToLive ---- */
    rbx_name both[2] = {nm(name), nm(cfg_name)};
    uint64_t mem = 0;
    CHECK(rbx_memory_usage_n(ctx, both, 2, &mem) == RBX_OK && mem > 256);
    int r = 0;
    CHECK(rbx_pexpire_n(ctx, both, 2, 60000, 0, 1 /* NX */, &r) == RBX_OK && r == 1);
    int64_t ttl = 0;
    CHECK(rbx_pttl(ctx, name, &ttl) == RBX_OK && ttl > 0 && ttl <= 60000);
    const char *cnames[2] = {name, cfg_name};
    CHECK(rbx_persist(ctx, cnames, 2, &r) == RBX_OK && r == 1);
    CHECK(rbx_pttl(ctx, name, &ttl) == RBX_OK && ttl == -1);

    /* ---- renamenx / isExists / delete ---- */
    CHECK(rbx_bloom_renamenx(ctx, name, "ffm-filter2", &r) == RBX_OK && r == 1);
    rbx_name both2[2] = {nm("ffm-filter2"), nm("{ffm-filter2}:config")};
    int ex = 0;
    CHECK(rbx_exists_n(ctx, both2, 2, &ex) == RBX_OK && ex == 2);
    CHECK(rbx_del_n(ctx, both2, 2, &r) == RBX_OK && r == 2);

    /* ---- GpuHyperLogLog: addAllAsync x2, mergeWithAsync, countWithAsync (testMerge) ---- */
    const char *h1[] = {"foo", "bar", "zap", "a"}, *h2[] = {"a", "b", "c", "foo", "c"};
    uint8_t b1[64], b2[64];
    uint64_t o1[8], o2[8];
    rbx_keys e1 = arena(h1, 4, b1, o1), e2 = arena(h2, 5, b2, o2);
    const char *n1[] = {"ffm-hll1"}, *n2[] = {"ffm-hll2"};
    uint64_t s1[2] = {0, 4}, s2[2] = {0, 5};
    uint8_t ch1 = 0, ch2 = 0;
    rbx_future *f[4];
    CHECK(rbx_hll_add_multi_async(ctx, n1, 1, s1, &e1, &ch1, on_done, (void *)(intptr_t)1, &f[0]) == RBX_OK);
    CHECK(rbx_hll_add_multi_async(ctx, n2, 1, s2, &e2, &ch2, on_done, (void *)(intptr_t)2, &f[1]) == RBX_OK);
    const char *srcs[] = {"ffm-hll1", "ffm-hll2"};
    CHECK(rbx_hll_merge_async(ctx, "ffm-hll3", srcs, 2, on_done, (void *)(intptr_t)3, &f[2]) == RBX_OK);
    const char *cw[] = {"ffm-hll3"};
    uint64_t pc = 0;
    CHECK(rbx_hll_count_async(ctx, cw, 1, &pc, on_done, (void *)(intptr_t)4, &f[3]) == RBX_OK);
    for (int i = 0; i < 4; ++i) {
        int rc = -99;
        CHECK(rbx_future_wait(f[i], 60000, &rc) == RBX_OK && rc == RBX_OK);
        CHECK(rbx_future_free(f[i]) == RBX_OK);
    }
    pthread_mutex_lock(&g_mu);
    for (int t = 1; t <= 4; ++t) CHECK(g_done[t] == 1 && g_rc[t] == RBX_OK);
    pthread_mutex_unlock(&g_mu);
    CHECK(ch1 == 1 && ch2 == 1 && pc == 6);

    CHECK(rbx_shutdown(ctx) == RBX_OK);
    printf("ffm_replay: all checks passed\n");
    return 0;
}
