/*
 * rbx.h -- C ABI of the MI355X-native batched sketch engine (librbx.so).
 *
 * Drop-in boundary for Redisson's probabilistic-structure hot path.  Every entry
 * point below replaces a reference interface; the citation is given per function.
 * Abbreviation: M/ = /root/reference/redisson/src/main/java/org/redisson/
 *
 * Conventions
 *  - Every function returns int: RBX_OK (0) or a negative error class that mirrors
 *    the exception the reference throws.  rbx_last_error() returns the message
 *    (thread-local; valid until the next call on the same thread).
 *  - The caller owns every host buffer; the library never retains one past return.
 *    Object handles (rbx_bloom, rbx_hll) are library-owned and reference-counted.
 *  - Keys/elements are codec OUTPUT bytes (RedissonObject.encode,
 *    M/RedissonObject.java:319-321).  The engine is codec-agnostic.
 *  - A context owns one GPU.  Calls on one context are serialized (a batch is the
 *    unit of serialization, matching the reference's pipeline order); calls from
 *    several threads are safe.  Handles keep their context's memory alive: closing a
 *    handle after rbx_shutdown is safe, any other call on it returns RBX_E_ILLEGAL_STATE.
 *  - *_dev variants take DEVICE pointers and a hipStream_t (as void*; NULL = the
 *    context's stream), enqueue work and return without synchronizing.  Counts are
 *    accumulated into device-resident unsigned long long words.  Per-call device scratch
 *    of a context is stream-ordered: use one stream per context for *_dev calls (or
 *    synchronize before switching streams).
 */
#ifndef RBX_H
#define RBX_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RBX_ABI_VERSION 1

enum {
    RBX_OK = 0,
    RBX_E_ILLEGAL_ARGUMENT = -1, /* java.lang.IllegalArgumentException             */
    RBX_E_ILLEGAL_STATE = -2,    /* IllegalStateException "Bloom filter is not initialized!" */
    RBX_E_CONFIG_CHANGED = -3,   /* RedisException "Bloom filter config has been changed" */
    RBX_E_ARITHMETIC = -4,       /* ArithmeticException "/ by zero" (empty collection) */
    RBX_E_WRONGTYPE = -5,        /* RedisException WRONGTYPE / INVALIDOBJ            */
    RBX_E_DEVICE = -6,           /* HIP / RCCL runtime failure                       */
    RBX_E_OOM = -7,              /* device or host allocation failure                */
    RBX_E_NO_SUCH_KEY = -8,      /* RedisException "ERR no such key" (RENAME)        */
    RBX_E_REDIS = -9,            /* other RedisException replies, e.g. "ERR bit offset is not an
                                    integer or out of range": a filter with |size| > 2^32 (only from
                                    tryInit with a negative expectedInsertions,
                                    M/RedissonBloomFilter.java:262-277) whose batch reaches an index
                                    (hash % |size|) past the Redis offset limit 2^32 - 1.  As in the
                                    reference's pipelined batch, rbx_bloom_add[_n] has then set every
                                    in-range bit (and created the key only if one was set) and
                                    rbx_bloom_contains[_n] changed nothing; a batch with no such
                                    index gets the exact in-order replies.  Handles (rbx_bloom_open*,
                                    hence the *_dev / multi-tenant / stream calls) and replica
                                    copies of such a filter are refused up front with this code. */
    RBX_E_TIMEOUT = -10          /* rbx_future_wait: the call has not completed in time        */
};

typedef struct rbx_ctx rbx_ctx;
typedef struct rbx_bloom rbx_bloom;
typedef struct rbx_hll rbx_hll;
typedef struct rbx_future rbx_future;
typedef struct rbx_node rbx_node;
/* completion callback of an asynchronous call: rc = the call's return code (runs on the
 * context's executor thread; a JVM binds it as an FFM upcall completing a CompletableFuture) */
typedef void (*rbx_callback)(void *user, int rc);

/* A batch of n encoded keys.  Key i is bytes[offsets[i] .. offsets[i+1]) when
 * offsets != NULL (n+1 entries), else bytes[i*stride .. (i+1)*stride). */
typedef struct rbx_keys {
    const uint8_t *bytes;
    const uint64_t *offsets;
    uint64_t stride;
    uint64_t n;
} rbx_keys;

/* A key name of any bytes (Redis keys are binary-safe; Spring Data passes byte[] keys,
 * redisson-spring-data-32 RedissonConnection.java:2203).  The *_n entry points take these; the
 * others take NUL-terminated names. */
typedef struct rbx_name {
    const uint8_t *bytes;
    uint64_t len;
} rbx_name;

/* The {name}:config hash (M/RedissonBloomFilter.java:285-288). */
typedef struct rbx_bloom_config {
    int64_t size;                /* "size" (bits; Java long: tryInit with a negative
                                    expectedInsertions stores a negative size, :270-276) */
    uint32_t hash_iterations;    /* "hashIterations" (k)                    */
    int64_t expected_insertions; /* "expectedInsertions" (0 if raw-created) */
    double false_probability;    /* "falseProbability"                      */
    char false_probability_str[64]; /* BigDecimal.toPlainString form        */
} rbx_bloom_config;

/* ---- library / context ------------------------------------------------------- */
int rbx_abi_version(void);
const char *rbx_last_error(void);
int rbx_device_count(int *out);
/* Redisson.create(config) -- M/Redisson.java; one context per GPU. */
int rbx_init(int device, rbx_ctx **out);
/* RedissonClient.shutdown() */
int rbx_shutdown(rbx_ctx *ctx);
int rbx_synchronize(rbx_ctx *ctx);
/* The context's hipStream_t, as void*. */
void *rbx_stream(rbx_ctx *ctx);

/* Pinned (page-locked) host memory for key arenas: batches whose bytes live here are
 * uploaded by DMA at full PCIe rate (a JVM wraps it as a MemorySegment). */
int rbx_host_alloc(uint64_t bytes, void **out);
int rbx_host_free(void *p);
/* Host-buffer batches are uploaded in double-buffered chunks of this many key bytes while
 * the previous chunk computes (default 64 MiB). */
int rbx_set_staging(rbx_ctx *ctx, uint64_t bytes);

/* ---- sharding: M/connection/CRC16.java:51-57, M/cluster/ClusterConnectionManager.java:777-792 */
uint16_t rbx_crc16(const uint8_t *bytes, size_t len);
int rbx_calc_slot(const uint8_t *key, size_t len);
/* Slot range -> GPU of one node: slot * n_gpus / 16384. */
int rbx_slot_to_gpu(int slot, int n_gpus);

/* ---- Bloom sizing: RedissonBloomFilter.optimalNumOfBits/HashFunctions :79-88 ---- */
int rbx_bloom_optimal_config(int64_t expected_insertions, double false_probability,
                             int64_t *size_out, uint32_t *k_out);

/* ---- RBloomFilter (by name) -- M/api/RBloomFilter.java:27-113 ---------------------- */
/* tryInit(expectedInsertions, falseProbability)  M/RedissonBloomFilter.java:262-300 */
int rbx_bloom_try_init(rbx_ctx *ctx, const char *name, int64_t expected_insertions,
                       double false_probability, int *created);
/* Engine-level init with a raw (size, k) -- reaches m = 2^32, which tryInit caps at
 * getMaxSize() = 4,294,967,294 (:257-259). */
int rbx_bloom_init_raw(rbx_ctx *ctx, const char *name, uint64_t size, uint32_t k, int *created);
/* readConfig() HGETALL {name}:config  :240-255 (RBX_E_ILLEGAL_STATE if absent) */
int rbx_bloom_read_config(rbx_ctx *ctx, const char *name, rbx_bloom_config *out);
/* add(Collection) :104-137.  size/k are the caller's cached config (size = the Java long's
 * bits; 0 = read the config first, :106-108), checked like addConfigCheck :207-213.
 * out_new (nullable): 1 byte per key, 1 iff the key counts as newly added under the
 * reference's in-order SETBIT semantics. */
int rbx_bloom_add(rbx_ctx *ctx, const char *name, uint64_t size, uint32_t k,
                  const rbx_keys *keys, uint8_t *out_new, uint64_t *out_count);
/* contains(Collection) :153-186.  out_present (nullable): 1 byte per key. */
int rbx_bloom_contains(rbx_ctx *ctx, const char *name, uint64_t size, uint32_t k,
                       const rbx_keys *keys, uint8_t *out_present, uint64_t *out_count);
/* count() :215-227 (BITCOUNT + the host double formula) */
int rbx_bloom_count(rbx_ctx *ctx, const char *name, int64_t *out);
/* the same four with binary names */
int rbx_bloom_try_init_n(rbx_ctx *ctx, rbx_name name, int64_t expected_insertions, double false_probability,
                         int *created);
int rbx_bloom_read_config_n(rbx_ctx *ctx, rbx_name name, rbx_bloom_config *out);
int rbx_bloom_add_n(rbx_ctx *ctx, rbx_name name, uint64_t size, uint32_t k, const rbx_keys *keys,
                    uint8_t *out_new, uint64_t *out_count);
int rbx_bloom_contains_n(rbx_ctx *ctx, rbx_name name, uint64_t size, uint32_t k, const rbx_keys *keys,
                         uint8_t *out_present, uint64_t *out_count);
int rbx_bloom_count_n(rbx_ctx *ctx, rbx_name name, int64_t *out);
/* DEL k1..kn (*deleted = keys removed) and EXISTS k1..kn (*count = existing keys, repeats
 * counted) over keys of any type -- RObject.delete / isExists for any name */
int rbx_del_n(rbx_ctx *ctx, const rbx_name *names, uint32_t n, int *deleted);
/* sizeInMemory (M/RedissonObject.java:124-130): bytes the engine holds for the existing keys --
 * device allocation of a bitmap / HLL, config fields, key names (not Redis' allocator figures).
 * The Bloom form sums the bitmap and {name}:config (M/RedissonBloomFilter.java:234-238). */
int rbx_memory_usage_n(rbx_ctx *ctx, const rbx_name *names, uint32_t n, uint64_t *bytes);
int rbx_bloom_size_in_memory(rbx_ctx *ctx, const char *name, uint64_t *bytes);
int rbx_exists_n(rbx_ctx *ctx, const rbx_name *names, uint32_t n, int *count);
/* BITCOUNT name */
int rbx_bloom_bitcount(rbx_ctx *ctx, const char *name, uint64_t *out);
/* delete() :230-232 -- DEL name {name}:config; *deleted = number of keys removed */
int rbx_bloom_delete(rbx_ctx *ctx, const char *name, int *deleted);
/* isExists() :344-347 -- EXISTS name {name}:config > 0 */
int rbx_bloom_is_exists(rbx_ctx *ctx, const char *name, int *exists);
/* rename :349-364 and renamenx :366-385 */
int rbx_bloom_rename(rbx_ctx *ctx, const char *name, const char *new_name);
int rbx_bloom_renamenx(rbx_ctx *ctx, const char *name, const char *new_name, int *renamed);

/* ---- key timeouts: RExpirable (M/RedissonExpirable.java:53-251) ----------------------------
 * Keys are removed lazily once their timeout passes (Redis semantics); handles follow their name.
 * rbx_pexpire replaces expireAsync / expireAtAsync (:207-239): PEXPIRE (absolute = 0, when_ms
 * relative) or PEXPIREAT (absolute = 1, unix ms) on every key, *result = 1 iff any timeout was
 * set.  cond: 0 none, 1 NX, 2 XX, 3 GT, 4 LT (expireIfNotSet / expireIfSet / expireIfGreater /
 * expireIfLess).  RBloomFilter passes {name, "{name}:config"} (M/RedissonBloomFilter.java:303-310),
 * RHyperLogLog {name}. */
int rbx_pexpire(rbx_ctx *ctx, const char *const *names, uint32_t n, int64_t when_ms, int absolute, int cond,
                int *result);
int rbx_pexpire_n(rbx_ctx *ctx, const rbx_name *names, uint32_t n, int64_t when_ms, int absolute, int cond,
                  int *result);
/* clearExpireAsync (:241-251): PERSIST every key, *result = 1 iff any timeout was removed */
int rbx_persist(rbx_ctx *ctx, const char *const *names, uint32_t n, int *result);
/* remainTimeToLiveAsync (:193-195) = PTTL, getExpireTimeAsync (:203-205) = PEXPIRETIME of one key:
 * -2 when the key does not exist, -1 when it has no timeout */
int rbx_pttl(rbx_ctx *ctx, const char *name, int64_t *out);
int rbx_pexpiretime(rbx_ctx *ctx, const char *name, int64_t *out);
/* GET name: the Redis bitmap string (MSB-first, length = highest SETBIT byte + 1).
 * Writes min(cap, len) bytes; *redis_len = len. */
int rbx_bloom_export(rbx_ctx *ctx, const char *name, uint8_t *out, uint64_t cap, uint64_t *redis_len);
/* SET name <bytes>: replaces the bitmap string (warm start from Redis data). */
int rbx_bloom_import(rbx_ctx *ctx, const char *name, const uint8_t *bytes, uint64_t len);

/* SET name from a DEVICE buffer (device-resident snapshot restore); synchronous. */
int rbx_bloom_import_dev(rbx_ctx *ctx, const char *name, const uint8_t *d_bytes, uint64_t len, void *stream);

/* ---- replicas ("replicate the bitmap, split contains keys across GPUs") ---------
 * Redisson serves contains' GETBITs as reads that may go to a replica
 * (M/RedissonBitSet.java:277-279 readAsync, ReadMode.SLAVE M/config/BaseMasterSlaveServersConfig.java:60)
 * and SETBITs to the master.  These are the engine's replica primitives. */
/* Order-independent 64-bit digest of `GET name` (0 = missing key): equal replicas have equal
 * digests (compared over a collective instead of moving the bitmaps). */
int rbx_bloom_digest(rbx_ctx *ctx, const char *name, uint64_t *out);
int rbx_bloom_digest_n(rbx_ctx *ctx, rbx_name name, uint64_t *out);
/* Replica sync inside one process: dst's {name}:config and bitmap string := src's, copied
 * device to device (hipMemcpyPeerAsync over xGMI between GPUs).  Key timeouts are not copied. */
int rbx_bloom_copy_to(rbx_ctx *src, rbx_ctx *dst, rbx_name name);
/* dst_name on dst := src_name on src (HLL registers, encoding, cached cardinality), device to
 * device; a missing source deletes dst_name.  PFCOUNT / PFMERGE inputs from another GPU. */
int rbx_hll_copy_to(rbx_ctx *src, rbx_name src_name, rbx_ctx *dst, rbx_name dst_name);
/* Enables peer access from `device` to `peer` where the hardware allows (best effort). */
int rbx_enable_peer_access(int device, int peer);

/* ---- Bloom handles and the device-resident batch path ------------------------------ */
int rbx_bloom_open(rbx_ctx *ctx, const char *name, rbx_bloom **out);
int rbx_bloom_open_n(rbx_ctx *ctx, rbx_name name, rbx_bloom **out);
int rbx_bloom_close(rbx_bloom *b);
int rbx_bloom_handle_config(const rbx_bloom *b, uint64_t *size, uint32_t *k);
/* contains over device-resident keys; *d_count += present keys (device word). */
int rbx_bloom_contains_dev(rbx_ctx *ctx, rbx_bloom *b, const rbx_keys *d_keys,
                           uint8_t *d_out_present, unsigned long long *d_count, void *stream);
/* add over device-resident keys; *d_count += newly added keys (device word).
 * Exception to the *_dev convention: a large batch on a large filter (the region-partitioned add,
 * bitmap >= 8 MiB and >= max(2^17, bits / 2^12) keys) waits on the stream once per chunk of up to
 * ~55M keys, for the chunk's bucket-overflow flag -- an adversarial batch (one key repeated ~1e5
 * times) reruns that chunk on the first-setter table path before the next chunk starts. */
int rbx_bloom_add_dev(rbx_ctx *ctx, rbx_bloom *b, const rbx_keys *d_keys, uint8_t *d_out_new,
                      unsigned long long *d_count, void *stream);
/* Multi-tenant batch: segment s = keys [seg_offsets[s], seg_offsets[s+1]) tested
 * against filters[s] -- one Redisson contains(Collection) per segment.
 * Device pointers: d_seg_offsets (nseg+1 u64), d_counts (nseg u64, accumulated). */
int rbx_bloom_contains_multi_dev(rbx_ctx *ctx, rbx_bloom *const *filters, uint32_t nseg,
                                 const uint64_t *d_seg_offsets, const rbx_keys *d_keys,
                                 uint8_t *d_out_present, unsigned long long *d_counts, void *stream);
/* add() per segment, segments applied in order (same semantics as nseg calls).  Enqueued on `stream`;
 * when every filter of the batch is distinct and the batch holds more than 16,384 keys, the call waits
 * for its per-segment kernel (one flag read back) to learn whether a segment that long needs the
 * chunked path (M/RedissonBloomFilter.java:104-137). */
int rbx_bloom_add_multi_dev(rbx_ctx *ctx, rbx_bloom *const *filters, uint32_t nseg,
                            const uint64_t *d_seg_offsets, const rbx_keys *d_keys,
                            uint8_t *d_out_new, unsigned long long *d_counts, void *stream);
/* Host-buffer multi-tenant forms (synchronous). */
int rbx_bloom_contains_multi(rbx_ctx *ctx, rbx_bloom *const *filters, uint32_t nseg,
                             const uint64_t *seg_offsets, const rbx_keys *keys,
                             uint8_t *out_present, uint64_t *out_counts);
int rbx_bloom_add_multi(rbx_ctx *ctx, rbx_bloom *const *filters, uint32_t nseg,
                        const uint64_t *seg_offsets, const rbx_keys *keys, uint8_t *out_new,
                        uint64_t *out_counts);

/* Ordered mixed stream (BASELINE C5): key i is one contains(T) (key_op[i] = 0) or add(T)
 * (key_op[i] = 1) on filters[key_filter[i]], executed in key order -- an add is visible to
 * every later contains of the same filter, exactly as the commands would run one after
 * another (M/RedissonBloomFilter.java:99-102, :198-201).  out (nullable): per key, present /
 * newly added.  counts[0] = present contains, counts[1] = newly added.  k <= 32. */
int rbx_bloom_stream_dev(rbx_ctx *ctx, rbx_bloom *const *filters, uint32_t nfilters, const uint32_t *d_key_filter,
                         const uint8_t *d_key_op, const rbx_keys *d_keys, uint8_t *d_out,
                         unsigned long long *d_counts, void *stream);
int rbx_bloom_stream(rbx_ctx *ctx, rbx_bloom *const *filters, uint32_t nfilters, const uint32_t *key_filter,
                     const uint8_t *key_op, const rbx_keys *keys, uint8_t *out, uint64_t *counts);

/* ---- RHyperLogLog (by name) -- M/api/RHyperLogLog.java:27-68 -------------------- */
/* add / addAll -> PFADD name e1..en   M/RedissonHyperLogLog.java:71-81.
 * *changed = 1 iff the key was created or any register changed. */
int rbx_hll_add(rbx_ctx *ctx, const char *name, const rbx_keys *elements, int *changed);
/* A batch of PFADD commands: segment s adds elements [seg_offsets[s], seg_offsets[s+1])
 * to names[s]; out_changed[s] is the reply of command s (commands apply in order). */
int rbx_hll_add_multi(rbx_ctx *ctx, const char *const *names, uint32_t nseg,
                      const uint64_t *seg_offsets, const rbx_keys *elements, uint8_t *out_changed);
/* count / countWith -> PFCOUNT k1..kn (union when n > 1)  :84-94 */
int rbx_hll_count(rbx_ctx *ctx, const char *const *names, uint32_t n, uint64_t *out);
/* n independent single-key PFCOUNTs in one batch (one GPU pass). */
int rbx_hll_count_each(rbx_ctx *ctx, const char *const *names, uint32_t n, uint64_t *out);
/* mergeWith -> PFMERGE dest src1..srcn (dest's registers included)  :97-102 */
int rbx_hll_merge(rbx_ctx *ctx, const char *dest, const char *const *srcs, uint32_t nsrc);
/* GET name: Redis dense HLL string (16-byte "HYLL" header + 12288 bytes).  *len = 0 if absent. */
int rbx_hll_export(rbx_ctx *ctx, const char *name, uint8_t *out, uint64_t cap, uint64_t *len);
/* GET name in a chosen encoding ([redis-7.2] hyperloglog.c):
 *   RBX_HLL_DENSE      the dense string (as rbx_hll_export);
 *   RBX_HLL_SPARSE     ZERO / XZERO / VAL opcodes: a key Redis holds sparse exports its string
 *                      (below); a dense key the fewest-bytes opcodes of its registers
 *                      (ILLEGAL_ARGUMENT if a register > 32);
 *   RBX_HLL_AS_STORED  what GET returns in Redis: PFADD creates sparse strings and applies each
 *                      element in order through hllSparseSet, promoting to dense (one way) at the
 *                      first element that stores a value > 32 or grows the string past
 *                      hll-sparse-max-bytes (3000); SET keeps the imported string; PFMERGE's
 *                      destination is dense iff it or any source is, else its string takes the
 *                      maxima register by register (pfmergeCommand).
 * *len receives the full length; at most cap bytes are copied. */
enum { RBX_HLL_DENSE = 0, RBX_HLL_SPARSE = 1, RBX_HLL_AS_STORED = 2 };
int rbx_hll_export_enc(rbx_ctx *ctx, const char *name, int encoding, uint8_t *out, uint64_t cap, uint64_t *len);
/* SET name <Redis HLL string> (dense or sparse encoding) */
int rbx_hll_import(rbx_ctx *ctx, const char *name, const uint8_t *bytes, uint64_t len);
int rbx_hll_delete(rbx_ctx *ctx, const char *name, int *deleted);
int rbx_hll_exists(rbx_ctx *ctx, const char *name, int *exists);
/* binary-name forms (Spring Data pfAdd/pfCount/pfMerge with byte[] keys,
 * redisson-spring-data-32 RedissonConnection.java:2200-2226) */
int rbx_hll_add_multi_n(rbx_ctx *ctx, const rbx_name *names, uint32_t nseg, const uint64_t *seg_offsets,
                        const rbx_keys *elements, uint8_t *out_changed);
int rbx_hll_count_n(rbx_ctx *ctx, const rbx_name *names, uint32_t n, uint64_t *out);
int rbx_hll_merge_n(rbx_ctx *ctx, rbx_name dest, const rbx_name *srcs, uint32_t nsrc);
int rbx_hll_export_enc_n(rbx_ctx *ctx, rbx_name name, int encoding, uint8_t *out, uint64_t cap, uint64_t *len);
int rbx_hll_import_n(rbx_ctx *ctx, rbx_name name, const uint8_t *bytes, uint64_t len);

/* ---- HLL handles and the device-resident path ------------------------------------- */
/* Opens (creating an empty HLL if absent and create != 0). */
int rbx_hll_open(rbx_ctx *ctx, const char *name, int create, rbx_hll **out);
int rbx_hll_open_n(rbx_ctx *ctx, rbx_name name, int create, rbx_hll **out);
int rbx_hll_close(rbx_hll *h);
/* Device address of the 16384 u8 registers (raw, one byte per register). */
int rbx_hll_registers_dev(rbx_hll *h, void **d_regs);
/* PFADD batch over device-resident elements; d_changed[s] |= 1 when command s
 * changed a register.  Each handle may appear at most once per call. */
int rbx_hll_add_multi_dev(rbx_ctx *ctx, rbx_hll *const *hlls, uint32_t nseg,
                          const uint64_t *d_seg_offsets, const uint64_t *h_seg_offsets,
                          const rbx_keys *d_elements, uint32_t *d_changed, void *stream);
/* Single-key PFCOUNT of each handle into host out[i] (synchronous). */
int rbx_hll_count_each_handles(rbx_ctx *ctx, rbx_hll *const *hlls, uint32_t n, uint64_t *out);

/* Register exchange of an element-partitioned HLL set (any transport): pack copies the
 * registers of hlls[i] to d_buf[i*16384 .. (i+1)*16384) in the caller's order; unpack_max
 * merges them back (register = max(register, buffer byte), PFMERGE semantics) and invalidates
 * the cached cardinalities.  Both enqueue on `stream` (NULL = the context's) and return. */
int rbx_hll_pack_registers(rbx_ctx *ctx, rbx_hll *const *hlls, uint32_t n, void *d_buf, void *stream);
int rbx_hll_unpack_max_registers(rbx_ctx *ctx, rbx_hll *const *hlls, uint32_t n, const void *d_buf, void *stream);

/* ---- multi-GPU (RCCL over xGMI) ------------------------------------------------------ */
/* 128-byte ncclUniqueId, created on rank 0 and broadcast by the caller. */
int rbx_rccl_unique_id(uint8_t out[128]);
int rbx_rccl_init(rbx_ctx *ctx, const uint8_t id[128], int nranks, int rank);
/* The communicator as RCCL reports it (ncclCommCount / ncclCommUserRank). */
int rbx_rccl_info(rbx_ctx *ctx, int *nranks, int *rank);
/* In-place uint8 MAX all-reduce of the registers of hlls[0..n) across ranks: pack (in the
 * given order) -> ONE ncclAllReduce(ncclUint8, ncclMax) of n x 16384 bytes -> unpack_max, so
 * every rank issues the same collective whatever its register pool layout.  Every rank passes
 * the same names in the same order. */
int rbx_hll_allreduce_max(rbx_ctx *ctx, rbx_hll *const *hlls, uint32_t n);

/* ---- asynchronous calls: the RFuture surface of RHyperLogLogAsync ---------------------------
 * M/api/RHyperLogLogAsync.java:37-70 (addAsync, addAllAsync, countAsync, countWithAsync,
 * mergeWithAsync; RBloomFilter has no async API in the reference -- the Bloom forms are an
 * engine extension).  Each *_async call is queued on the context's serial executor and runs after
 * every call queued before it on that context; it returns at once with a future.  Names, segment
 * offsets and the rbx_keys descriptor are copied at submit time; key bytes and result buffers
 * must stay valid until the future completes.  `cb` (nullable) runs when the call completes. */
int rbx_future_wait(rbx_future *f, int64_t timeout_ms, int *call_rc); /* RBX_E_TIMEOUT if not done;
                                                                         timeout_ms < 0 waits for ever */
int rbx_future_done(rbx_future *f, int *done);
int rbx_future_free(rbx_future *f);  /* may be called before completion (the result is dropped) */
int rbx_bloom_add_async(rbx_ctx *ctx, const char *name, uint64_t size, uint32_t k, const rbx_keys *keys,
                        uint8_t *out_new, uint64_t *out_count, rbx_callback cb, void *user, rbx_future **out);
int rbx_bloom_contains_async(rbx_ctx *ctx, const char *name, uint64_t size, uint32_t k, const rbx_keys *keys,
                             uint8_t *out_present, uint64_t *out_count, rbx_callback cb, void *user,
                             rbx_future **out);
int rbx_hll_add_async(rbx_ctx *ctx, const char *name, const rbx_keys *elements, int *changed, rbx_callback cb,
                      void *user, rbx_future **out);
int rbx_hll_add_multi_async(rbx_ctx *ctx, const char *const *names, uint32_t nseg, const uint64_t *seg_offsets,
                            const rbx_keys *elements, uint8_t *out_changed, rbx_callback cb, void *user,
                            rbx_future **out);
int rbx_hll_count_async(rbx_ctx *ctx, const char *const *names, uint32_t n, uint64_t *result, rbx_callback cb,
                        void *user, rbx_future **out);
int rbx_hll_merge_async(rbx_ctx *ctx, const char *dest, const char *const *srcs, uint32_t nsrc, rbx_callback cb,
                        void *user, rbx_future **out);

/* ---- one process over the GPUs of a node -----------------------------------------------------
 * A node holds one context per GPU and routes every name by Redis Cluster slot, the way the
 * reference's client groups a batch per node (M/command/CommandBatchService.java:569-604,
 * M/cluster/ClusterConnectionManager.java:777-830): GPU = calc_slot(name) * n_gpus / 16384, so a
 * filter's bitmap `name` and its `{name}:config` live on one GPU.  devices: the HIP device of
 * each of the n_gpus contexts (NULL = 0..n_gpus-1; a device may repeat, e.g. to rehearse a node
 * on one GPU).  Multi-tenant batches are scattered by slot into per-GPU batches, run
 * concurrently (one host thread per GPU, each GPU its own context and stream) and gathered back
 * in segment order.  Calls on one node from several threads are safe. */
int rbx_node_init(int n_gpus, const int *devices, rbx_node **out);
int rbx_node_shutdown(rbx_node *node);
int rbx_node_size(const rbx_node *node, int *n_gpus);
int rbx_node_gpu_of(const rbx_node *node, rbx_name name, int *gpu);
int rbx_node_ctx(rbx_node *node, int gpu, rbx_ctx **out); /* the GPU's context (device-path calls) */
int rbx_node_bloom_try_init(rbx_node *node, rbx_name name, int64_t expected_insertions, double false_probability,
                            int *created);
int rbx_node_bloom_read_config(rbx_node *node, rbx_name name, rbx_bloom_config *out);
int rbx_node_bloom_add(rbx_node *node, rbx_name name, uint64_t size, uint32_t k, const rbx_keys *keys,
                       uint8_t *out_new, uint64_t *out_count);
int rbx_node_bloom_contains(rbx_node *node, rbx_name name, uint64_t size, uint32_t k, const rbx_keys *keys,
                            uint8_t *out_present, uint64_t *out_count);
int rbx_node_bloom_count(rbx_node *node, rbx_name name, int64_t *out);
int rbx_node_del(rbx_node *node, const rbx_name *names, uint32_t n, int *deleted);
/* Replicated filter (SURVEY 8e, C2 "replicas only"): on != 0 copies the filter (config hash +
 * bitmap) from its home GPU to every other GPU, device to device, then routes every add of it
 * to all replicas (the home GPU's reply is returned) and spreads its contains over them (one
 * key range per replica; multi-tenant segments round-robin) -- Redisson's reads-from-replicas
 * (GETBIT via readAsync, M/RedissonBitSet.java:277-279; ReadMode.SLAVE,
 * M/config/BaseMasterSlaveServersConfig.java:60).  on == 0 drops the copies.  DEL of the
 * filter's keys deletes every copy; deleting its config ends the replication. */
int rbx_node_bloom_replicate(rbx_node *node, rbx_name name, int on);
int rbx_node_bloom_is_replicated(rbx_node *node, rbx_name name, int *replicated);
/* segment s = keys [seg_offsets[s], seg_offsets[s+1]) of names[s] (host buffers; a segment must
 * be non-empty, as contains/add(Collection) of an empty collection throw); out_* nullable. */
int rbx_node_bloom_contains_multi(rbx_node *node, const rbx_name *names, uint32_t nseg, const uint64_t *seg_offsets,
                                  const rbx_keys *keys, uint8_t *out_present, uint64_t *out_counts);
int rbx_node_bloom_add_multi(rbx_node *node, const rbx_name *names, uint32_t nseg, const uint64_t *seg_offsets,
                             const rbx_keys *keys, uint8_t *out_new, uint64_t *out_counts);
/* PFADD commands routed per name (commands on one name keep their order) */
int rbx_node_hll_add_multi(rbx_node *node, const rbx_name *names, uint32_t nseg, const uint64_t *seg_offsets,
                           const rbx_keys *elements, uint8_t *out_changed);
/* PFCOUNT / PFMERGE over names that may live on different GPUs: every HLL held by another GPU is
 * peer-copied device to device (rbx_hll_copy_to: registers, encoding, cached cardinality and the
 * sparse string, over xGMI on a multi-GPU node) into a temporary key on the GPU of the first name
 * (PFCOUNT) or of the destination (PFMERGE), which is deleted after the call -- no host staging.
 * M/RedissonHyperLogLog.java:89-102 (countWith / mergeWith). */
int rbx_node_hll_count(rbx_node *node, const rbx_name *names, uint32_t n, uint64_t *out);
int rbx_node_hll_merge(rbx_node *node, rbx_name dest, const rbx_name *srcs, uint32_t nsrc);

#ifdef __cplusplus
}
#endif
#endif /* RBX_H */
