/*
 * rbx_oracle_mt.c -- multithreaded form of the CPU restatement (rbx_oracle.c), for bench.py's
 * cpu_baseline leg: "time the build's own multithreaded C++ CPU restatement on all host cores"
 * (BASELINE.md fallback; Redisson + redis-server cannot run in this image).
 *
 * TEST INFRASTRUCTURE ONLY, like rbx_oracle.c: nothing in the product links or calls it.
 *
 * Same results as the single-thread functions, bit for bit:
 *   contains(Collection)  M/RedissonBloomFilter.java:153-186 -- read-only, keys split over
 *                         threads;
 *   add(Collection)       :104-137 with the in-order SETBIT semantics of the reference's batch
 *                         (M/command/CommandBatchService.java:115-134): the bit indexes of a
 *                         chunk are computed in parallel, then every thread applies, in key
 *                         order, the SETBITs that fall in ITS byte range of the bitmap -- each
 *                         bit has one owner thread that sees the keys in submission order, so
 *                         "this SETBIT replied 0" is exactly the sequential answer.
 */
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

void orc_redisson_hash128(const uint8_t *data, size_t len, uint64_t out[2]);
void orc_bloom_indexes(uint64_t hash1, uint64_t hash2, int iterations, int64_t size, int64_t *out);
int64_t orc_bloom_add(uint8_t *bitmap, uint64_t *redis_len, const uint8_t *bytes, const uint64_t *offsets,
                      uint64_t n, int k, int64_t size, uint8_t *out_new);
int64_t orc_bloom_contains(const uint8_t *bitmap, uint64_t redis_len, const uint8_t *bytes,
                           const uint64_t *offsets, uint64_t n, int k, int64_t size, uint8_t *out_present);

/* |size| past 2^32 bits: the single-thread functions (the Redis offset limit, rbx_oracle.c) */
static int wide_size(int64_t size) { return (size < 0 ? 0 - (uint64_t)size : (uint64_t)size) > (1ULL << 32); }

typedef struct {
    const uint8_t *bitmap;
    uint64_t redis_len;
    uint8_t *wbitmap;
    const uint8_t *bytes;
    const uint64_t *offsets;
    uint64_t i0, i1;
    int k;
    int64_t size;
    uint8_t *out;
    int64_t *idx;       /* add: n*k indexes of the chunk */
    uint64_t b0, b1;    /* add: owned byte range [b0, b1) */
    uint64_t len_max;   /* add: highest touched byte + 1 in the owned range */
    int64_t missed;
} orc_job;

static void *contains_worker(void *p) {
    orc_job *j = (orc_job *)p;
    int64_t idx[64];
    int64_t missed = 0;
    for (uint64_t i = j->i0; i < j->i1; i++) {
        uint64_t h[2];
        orc_redisson_hash128(j->bytes + j->offsets[i], (size_t)(j->offsets[i + 1] - j->offsets[i]), h);
        orc_bloom_indexes(h[0], h[1], j->k, j->size, idx);
        int zeros = 0;
        for (int q = 0; q < j->k; q++) {
            const uint64_t b = (uint64_t)idx[q] >> 3;
            if (b >= j->redis_len || !((j->bitmap[b] >> (7 - (idx[q] & 7))) & 1)) {
                zeros = 1;
                break; /* the answer only needs the first 0 bit */
            }
        }
        if (j->out) j->out[i] = zeros == 0;
        missed += zeros;
    }
    j->missed = missed;
    return NULL;
}

/* contains over keys [0, n) with nthreads threads; k <= 64 */
int64_t orc_bloom_contains_mt(const uint8_t *bitmap, uint64_t redis_len, const uint8_t *bytes,
                              const uint64_t *offsets, uint64_t n, int k, int64_t size, uint8_t *out_present,
                              int nthreads) {
    if (n == 0) return -4;
    if (k > 64) return -1;
    if (wide_size(size)) return orc_bloom_contains(bitmap, redis_len, bytes, offsets, n, k, size, out_present);
    if (nthreads < 1) nthreads = 1;
    pthread_t *th = (pthread_t *)calloc((size_t)nthreads, sizeof(pthread_t));
    orc_job *jobs = (orc_job *)calloc((size_t)nthreads, sizeof(orc_job));
    for (int t = 0; t < nthreads; t++) {
        orc_job *j = &jobs[t];
        j->bitmap = bitmap;
        j->redis_len = redis_len;
        j->bytes = bytes;
        j->offsets = offsets;
        j->i0 = n * (uint64_t)t / (uint64_t)nthreads;
        j->i1 = n * (uint64_t)(t + 1) / (uint64_t)nthreads;
        j->k = k;
        j->size = size;
        j->out = out_present;
        pthread_create(&th[t], NULL, contains_worker, j);
    }
    int64_t missed = 0;
    for (int t = 0; t < nthreads; t++) {
        pthread_join(th[t], NULL);
        missed += jobs[t].missed;
    }
    free(th);
    free(jobs);
    return (int64_t)n - missed;
}

static void *hash_worker(void *p) {
    orc_job *j = (orc_job *)p;
    for (uint64_t i = j->i0; i < j->i1; i++) {
        uint64_t h[2];
        orc_redisson_hash128(j->bytes + j->offsets[i], (size_t)(j->offsets[i + 1] - j->offsets[i]), h);
        orc_bloom_indexes(h[0], h[1], j->k, j->size, j->idx + (i - j->i0 + (j->i0 - j->b0)) * (uint64_t)j->k);
    }
    return NULL;
}

static void *setbit_worker(void *p) {
    orc_job *j = (orc_job *)p;
    const uint64_t nk = (j->i1 - j->i0) * (uint64_t)j->k;
    uint64_t len_max = 0;
    for (uint64_t e = 0; e < nk; e++) {
        const uint64_t bit = (uint64_t)j->idx[e], b = bit >> 3;
        if (b < j->b0 || b >= j->b1) continue;
        const uint8_t m = (uint8_t)(0x80u >> (bit & 7));
        if (b + 1 > len_max) len_max = b + 1;
        if (!(j->wbitmap[b] & m)) {
            j->wbitmap[b] |= m;
            __atomic_store_n(&j->out[j->i0 + e / (uint64_t)j->k], (uint8_t)1, __ATOMIC_RELAXED);
        }
    }
    j->len_max = len_max;
    return NULL;
}

/* add over keys [0, n) with nthreads threads; returns the count like orc_bloom_add (the Java
 * `int c` accumulator), out_new (required here) gets the per-key flags. */
int64_t orc_bloom_add_mt(uint8_t *bitmap, uint64_t *redis_len, const uint8_t *bytes, const uint64_t *offsets,
                         uint64_t n, int k, int64_t size, uint8_t *out_new, int nthreads) {
    if (n == 0) return -4;
    if (wide_size(size)) return orc_bloom_add(bitmap, redis_len, bytes, offsets, n, k, size, out_new);
    if (nthreads < 1) nthreads = 1;
    memset(out_new, 0, (size_t)n);
    const uint64_t m = size < 0 ? 0 - (uint64_t)size : (uint64_t)size;
    const uint64_t nbytes = (m + 7) / 8;
    const uint64_t chunk = 1ULL << 22; /* keys per chunk: bounds the index array to 4M x k x 8 B */
    int64_t *idx = (int64_t *)malloc((size_t)(chunk * (uint64_t)k * sizeof(int64_t)));
    pthread_t *th = (pthread_t *)calloc((size_t)nthreads, sizeof(pthread_t));
    orc_job *jobs = (orc_job *)calloc((size_t)nthreads, sizeof(orc_job));
    for (uint64_t c0 = 0; c0 < n; c0 += chunk) {
        const uint64_t c1 = c0 + chunk < n ? c0 + chunk : n;
        for (int t = 0; t < nthreads; t++) { /* hash: keys split over threads */
            orc_job *j = &jobs[t];
            memset(j, 0, sizeof *j);
            j->bytes = bytes;
            j->offsets = offsets;
            j->i0 = c0 + (c1 - c0) * (uint64_t)t / (uint64_t)nthreads;
            j->i1 = c0 + (c1 - c0) * (uint64_t)(t + 1) / (uint64_t)nthreads;
            j->b0 = c0; /* index rows are relative to the chunk start */
            j->k = k;
            j->size = size;
            j->idx = idx;
            pthread_create(&th[t], NULL, hash_worker, j);
        }
        for (int t = 0; t < nthreads; t++) pthread_join(th[t], NULL);
        for (int t = 0; t < nthreads; t++) { /* SETBIT: bitmap bytes split over threads */
            orc_job *j = &jobs[t];
            memset(j, 0, sizeof *j);
            j->wbitmap = bitmap;
            j->i0 = c0;
            j->i1 = c1;
            j->k = k;
            j->idx = idx;
            j->out = out_new;
            j->b0 = nbytes * (uint64_t)t / (uint64_t)nthreads;
            j->b1 = nbytes * (uint64_t)(t + 1) / (uint64_t)nthreads;
            pthread_create(&th[t], NULL, setbit_worker, j);
        }
        for (int t = 0; t < nthreads; t++) {
            pthread_join(th[t], NULL);
            if (jobs[t].len_max > *redis_len) *redis_len = jobs[t].len_max;
        }
    }
    free(idx);
    free(th);
    free(jobs);
    int64_t c = 0;
    for (uint64_t i = 0; i < n; i++) c += out_new[i];
    return (int64_t)(int32_t)c;
}
