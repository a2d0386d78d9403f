// rbx_api.cpp -- librbx.so host side: contexts, the Redis-like keyspace the sketches
// live in, batching/chunking, and every extern "C" entry point of include/rbx.h.
//
// The keyspace mirrors how Redisson lays the structures out in Redis:
//   name          -> bitmap string (Bloom) | HLL string
//   {name}:config -> Bloom config hash    (RedissonObject.suffixName, M/RedissonObject.java:77-82)
// so delete/exists/rename keep the reference's key-level semantics.
// M/ = /root/reference/redisson/src/main/java/org/redisson/
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <unordered_map>
#include <vector>

#include "../../include/rbx.h"
#include "host_exec.h"
#include "keyspace.h"
#include "rbx_kernels.h"

using namespace rbx;

#define HIP_TRY(expr)                                                                          \
    do {                                                                                       \
        hipError_t e_ = (expr);                                                                \
        if (e_ != hipSuccess)                                                                  \
            return fail(e_ == hipErrorOutOfMemory ? RBX_E_OOM : RBX_E_DEVICE,                  \
                        std::string(#expr ": ") + hipGetErrorString(e_));                      \
    } while (0)

#define RBX_TRY(expr)             \
    do {                          \
        int r_ = (expr);          \
        if (r_ != RBX_OK) return r_; \
    } while (0)

// =====================================================================================
// device buffers
// =====================================================================================
struct DevBuf {
    void *p = nullptr;
    size_t cap = 0;
    ~DevBuf() {
        if (p) (void)hipFree(p);
    }
    int reserve(size_t n) {
        if (n <= cap) return RBX_OK;
        if (p) {
            (void)hipFree(p);
            p = nullptr;
            cap = 0;
        }
        size_t want = std::max<size_t>(n, 4096);
        HIP_TRY(hipMalloc(&p, want));
        cap = want;
        return RBX_OK;
    }
    template <class T> T *as() const { return (T *)p; }
};

// =====================================================================================
// device objects held by the keyspace (keyspace.h declares them opaque)
// =====================================================================================
// Small bitmaps (<= 64 MiB) come from 1 GiB slabs, exact-size free lists, so that
// 100k tenant filters do not cost 100k hipMalloc calls; large ones get their own buffer.
// Memory returned to a free list is reused only through new_bitmap / hll_alloc, whose zero
// fill runs on the calling stream after it waited for every earlier call of the context
// (ScratchOrder): so a freed bitmap or HLL still read by an in-flight *_dev call on another
// stream is never overwritten early.
struct SlabPool {
    std::mutex mu;
    std::vector<void *> slabs;
    std::map<uint64_t, std::vector<void *>> free_by_size;
    uint8_t *cur = nullptr;
    uint64_t left = 0;
    static constexpr uint64_t kSlab = 1ull << 30, kMaxSmall = 64ull << 20;
    void *get(uint64_t bytes) {
        std::lock_guard<std::mutex> g(mu);
        auto &fl = free_by_size[bytes];
        if (!fl.empty()) {
            void *p = fl.back();
            fl.pop_back();
            return p;
        }
        if (left < bytes) {
            void *s = nullptr;
            if (hipMalloc(&s, kSlab) != hipSuccess) return nullptr;
            slabs.push_back(s);
            cur = (uint8_t *)s;
            left = kSlab;
        }
        void *p = cur;
        cur += bytes;
        left -= bytes;
        return p;
    }
    void put(void *p, uint64_t bytes) {
        std::lock_guard<std::mutex> g(mu);
        free_by_size[bytes].push_back(p);
    }
    ~SlabPool() {
        for (void *s : slabs) (void)hipFree(s);
    }
};

namespace rbx {
struct Bitmap {  // a Redis string used with SETBIT/GETBIT
    int device = 0;
    uint32_t *d_words = nullptr;
    uint64_t cap_bytes = 0;                 // allocated bytes (multiple of 256)
    unsigned long long *d_len = nullptr;    // device word: Redis string length (in the slab too)
    std::shared_ptr<SlabPool> pool;         // set when d_words/d_len came from the pool
    ~Bitmap() {
        if (pool) {
            pool->put(d_words, cap_bytes + 256);
            return;
        }
        if (d_words) (void)hipFree(d_words);
        if (d_len) (void)hipFree(d_len);
    }
};

struct HllState {  // a Redis HLL string, registers unpacked (1 byte each) on the device
    uint8_t *d_regs = nullptr;  // 16384 bytes inside a pool chunk
    // device state words (HllReplay::state): [0] promoted -- a PFADD / PFMERGE promoted the sparse
    // string to dense --, [1] opcodes in d_sp_ops (0 = the createHLLObject string), [2] its bytes
    uint32_t *d_promoted = nullptr;
    uint16_t *d_sp_ops = nullptr;  // the sparse string as Redis built it, one u16 per opcode
    uint16_t *d_slot_ops = nullptr;  // the pool slot's opcode list (kHllSlotOps entries)
    uint16_t *d_big_ops = nullptr;   // own allocation (16384 entries) for a SET string past the slot
    uint64_t card = 0;          // the header's 8 cached-cardinality bytes (LE); bit 63 = invalid
    bool dense = false;         // Redis encoding: created sparse, promoted to dense once (never back)
    struct ::rbx_ctx *owner = nullptr;
    ~HllState();
};
}  // namespace rbx

// Handles are bound to a NAME, like a Redisson object: a call re-resolves the keys whenever the
// keyspace changed since the handle's last call (gen), so delete / rename / expire / re-import
// behave as they do through the name-based entry points.  A handle holds a reference on its
// context, so closing it after rbx_shutdown is safe (every other call on it then fails).
struct rbx_bloom {
    rbx_ctx *ctx;
    std::string name;
    int64_t size;  // the config's size (Java long)
    uint32_t k;
    std::shared_ptr<Bitmap> bm;
    uint64_t gen = 0;
    uint64_t serial = 0;  // unique per handle (a freed handle's address can be reused)
};
static std::atomic<uint64_t> g_handle_serial{1};

struct rbx_hll {
    rbx_ctx *ctx;
    std::string name;
    std::shared_ptr<HllState> st;
    uint64_t gen = 0;
};

struct rbx_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    Keyspace ks;  // names -> objects, and the context lock (ks.mu)
    // references: the API (rbx_init .. rbx_shutdown) + every open handle + every live HLL
    // state; the context's memory is released with the last one
    std::atomic<int> refs{1};
    bool shut = false;  // rbx_shutdown ran: device resources are gone, calls fail

    // first-setter table for add()
    DevBuf table;
    uint32_t log2cap = 0;
    uint32_t epoch = 255;  // 255 = table needs (re)initialisation
    DevBuf zmask;

    // staging for host-buffer calls
    DevBuf keys_bytes, keys_offs, out_bytes, seg_offs, counters, filt_table, ptrs, histo, misc, tile_segs, hll_tiles;
    DevBuf probe_table;  // ProbeDesc per entry of filt_table
    DevBuf pc_bits, pc_cnt, pc_pairs1, pc_pairs2, pc_mrec;  // partitioned contains
    DevBuf pa_p1, pa_p2, pa_cnt, pa_bits, pa_ctr, pa_recs;  // partitioned add
    DevBuf pa_stamps;  // add_partition_diag & 64: region-pass phase times (rbx_bench_add_stamps)
    DevBuf st_adds, st_nadds;    // ordered stream: add list, one add counter per chunk
    DevBuf st_t8;                // ordered stream (r04): 8-byte first-setter table (EMPTY between chunks)
    DevBuf st_fslot;             // ordered stream (r05): per add, the slot of its first zero bit's claim
    DevBuf madd_c;               // multi-tenant add (r05): conflict table C + its MaddxState (+ the `big` flag)
    uint64_t madd_maxseg_hint = ~0ULL;  // set by the host-arena add_multi: its largest segment (keys)
    uint64_t st_t8_entries = 0;  // initialized size of st_t8
    uint64_t st_geom[4] = {0, 0, 0, 0};             // last stream call: bb, fbits, pb, chunk
    DevBuf fid_table;            // bitmap words per table id (fid) of the filters of filt_table
    uint32_t filt_nfids = 0;     // distinct table ids of filt_table
    uint64_t filt_maxbits = 0;   // the largest of their bitmaps, in bits
    // all-zero words standing in for a missing bitmap in multi-tenant contains (GETBIT on a
    // missing key reads 0; the key is not created), grown on demand, never written by a kernel
    DevBuf zero_bm;
    DevBuf hll_pack;                                // contiguous registers for the RCCL merge
    DevBuf wide_table;  // first-setter table of |size| > 2^32 adds (bloom_wide_op)
    std::vector<HllSeg> tile_cache;  // content of hll_tiles (valid when tiles_valid)
    bool tiles_valid = false;
    std::vector<FilterDesc> filt_cache;  // content of filt_table
    uint64_t filt_generation = 0;
    // the handle list filt_table was built from (fast path for repeated multi-tenant calls)
    std::vector<std::pair<const rbx_bloom *, uint64_t>> filt_keys;
    uint64_t filt_key_generation = ~0ULL, filt_bytes = 0;
    bool filt_create = false;
    uint32_t filt_kmax = 1;

    std::shared_ptr<SlabPool> slab = std::make_shared<SlabPool>();

    // HLL register pool: chunks of kHllPerChunk x 16 KiB
    std::vector<uint8_t *> hll_chunks;
    struct HllSlot {
        uint8_t *regs;
        uint32_t *state;
        uint16_t *ops;
    };
    std::vector<HllSlot> hll_free;   // zeroed slots (registers, state words, sparse opcodes)
    std::vector<HllSlot> hll_dirty;  // slots of deleted HLLs, zeroed together when hll_free runs out
    DevBuf hll_zero_ptrs;            // their pointers for k_hll_zero
    DevBuf hll_checks;                     // k_hll_sparse_replay items (cached by content)
    std::vector<HllReplay> check_cache;

    ncclComm_t comm = nullptr;
    int nranks = 1, rank = 0;

    // host-buffer pipeline: uploads on copy_stream into two device slots while the
    // previous slot's kernels run on the compute stream
    hipStream_t copy_stream = nullptr;
    hipEvent_t ev_copied[2] = {nullptr, nullptr}, ev_done[2] = {nullptr, nullptr};
    DevBuf slot_bytes[2], slot_offs[2];
    uint64_t staging_bytes = 64ull << 20;
    // small host batches (bloom_host_small): a pinned copy of the keys, uploaded on `stream` with the
    // zeroed count word in one transfer; the count and flags come back into it
    void *pin_small = nullptr;
    size_t pin_small_cap = 0;
    uint64_t pin_small_limit = 0;  // the host_small_bytes the block was laid out for (its tail offset)
    unsigned long long *pin_word = nullptr;  // pinned readback words (counts, the partitioned add's overflow flag)
    // tiny host batches (bloom_host_tiny): coherent pinned memory the kernel reads the keys from and
    // writes the flags into, no transfer on either side
    uint8_t *pin_tiny = nullptr, *pin_tiny_dev = nullptr;
    uint32_t tiny_seq = 0;  // the last completion word a one-key kernel stored into the block

    // stream order of the scratch above across calls issued on different streams (ScratchOrder)
    hipEvent_t ev_scratch = nullptr;
    hipStream_t scratch_stream = nullptr;

    // the asynchronous entry points' serial executor (host_exec.h): its thread starts with the
    // first *_async call.  exec_mu guards the pointer: rbx_shutdown takes the executor out under
    // it, so a submit either lands before (and runs) or is refused.
    std::mutex exec_mu;
    std::unique_ptr<SerialExecutor> exec = std::make_unique<SerialExecutor>();
};

struct rbx_future {
    std::shared_ptr<Future> f;
};

static void ctx_release(rbx_ctx *c) {
    if (c->refs.fetch_sub(1) == 1) delete c;
}

// Every call that enqueues work touching the context's scratch (first-setter table, pair
// buckets, staging, descriptor tables, counters) or fills newly allocated object memory runs on
// the device after the previous such call, also when the two were issued on different streams:
// the new stream waits on an event the previous user recorded.  (The host mutex orders the
// calls; this orders their kernels.)
struct ScratchOrder {
    rbx_ctx *c;
    hipStream_t st;
    ScratchOrder(rbx_ctx *c_, hipStream_t st_) : c(c_), st(st_) {
        if (c->ev_scratch && c->scratch_stream && c->scratch_stream != st) (void)hipStreamWaitEvent(st, c->ev_scratch, 0);
    }
    ~ScratchOrder() {
        if (c->ev_scratch && hipEventRecord(c->ev_scratch, st) == hipSuccess) c->scratch_stream = st;
    }
};

static constexpr size_t kHllBytes = 16384;
static constexpr size_t kHllPerChunk = 4096;  // 192 MiB per pool chunk
static constexpr size_t kHllStateWords = 4;   // HllReplay::state, 16 bytes
// Opcode list capacity per pooled HLL.  A sparse string's opcodes never outnumber its bytes, and
// hllSparseSet promotes instead of growing a string past hll-sparse-max-bytes (3000), so a
// PFADD-built string fits 3072 entries (6 KiB per HLL instead of 32 KiB); a SET string
// longer than that (up to 16384 opcodes) moves to its own allocation (hll_ops_reserve), and
// from then on it can only shrink or promote.
static constexpr size_t kHllSlotOps = 3072;
static constexpr size_t kHllOpsBytes = kHllSlotOps * 2;
static constexpr size_t kHllMaxOps = 16384;

rbx::HllState::~HllState() {
    if (d_regs && owner) {
        {
            std::lock_guard<std::recursive_mutex> g(owner->ks.mu);
            if (!owner->shut) owner->hll_dirty.push_back({d_regs, d_promoted, d_slot_ops});
        }
        if (d_big_ops) (void)hipFree(d_big_ops);  // its own allocation: released also after a shutdown
        ctx_release(owner);
    }
}

// room for `nops` opcodes in h's list (the caller then overwrites the list)
static int hll_ops_reserve(HllState *h, uint64_t nops) {
    if (nops <= kHllSlotOps || h->d_big_ops) {
        if (nops > kHllMaxOps) return fail(RBX_E_WRONGTYPE, "a sparse HLL string holds at most 16384 opcodes");
        if (h->d_big_ops) h->d_sp_ops = h->d_big_ops;
        return RBX_OK;
    }
    if (nops > kHllMaxOps) return fail(RBX_E_WRONGTYPE, "a sparse HLL string holds at most 16384 opcodes");
    HIP_TRY(hipMalloc(&h->d_big_ops, kHllMaxOps * 2));
    h->d_sp_ops = h->d_big_ops;
    return RBX_OK;
}

// A fresh zeroed HLL register block; the fill runs on `st` (see SlabPool).
static int hll_alloc(rbx_ctx *c, hipStream_t st, std::shared_ptr<HllState> *out) {
    if (c->hll_free.empty() && !c->hll_dirty.empty()) {
        // the deleted HLLs' slots, zeroed in one launch on the caller's stream (creating 10k HLLs
        // cost 20k small fills, ~10 ms of enqueueing, when each slot was zeroed on its own)
        const size_t n = c->hll_dirty.size();
        std::vector<void *> ptrs(2 * n);
        for (size_t i = 0; i < n; ++i) {
            ptrs[i] = c->hll_dirty[i].regs;
            ptrs[n + i] = c->hll_dirty[i].state;
        }
        RBX_TRY(c->hll_zero_ptrs.reserve(ptrs.size() * sizeof(void *)));
        HIP_TRY(hipMemcpyAsync(c->hll_zero_ptrs.p, ptrs.data(), ptrs.size() * sizeof(void *), hipMemcpyHostToDevice, st));
        uint8_t *const *d_regs = c->hll_zero_ptrs.as<uint8_t *>();
        launch_hll_zero(d_regs, (uint32_t *const *)(d_regs + n), (uint32_t)n, st);
        HIP_TRY(hipGetLastError());
        // handed out last-deleted first, as before
        c->hll_free.insert(c->hll_free.end(), c->hll_dirty.begin(), c->hll_dirty.end());
        c->hll_dirty.clear();
    }
    if (c->hll_free.empty()) {
        // registers of kHllPerChunk HLLs, then their state words, then their sparse opcode lists
        uint8_t *chunk = nullptr;
        HIP_TRY(hipMalloc(&chunk, (kHllBytes + kHllStateWords * 4 + kHllOpsBytes) * kHllPerChunk));
        c->hll_chunks.push_back(chunk);
        uint32_t *words = (uint32_t *)(chunk + kHllBytes * kHllPerChunk);
        uint16_t *ops = (uint16_t *)(words + kHllStateWords * kHllPerChunk);
        // registers and state words of the whole chunk zeroed at once: creating 10k HLLs cost
        // 20k small fills (~10 ms of enqueueing) when each slot was zeroed on its own
        HIP_TRY(hipMemsetAsync(chunk, 0, (kHllBytes + kHllStateWords * 4) * kHllPerChunk, st));
        // hand out in reverse so that successive allocations are ascending
        for (size_t i = kHllPerChunk; i-- > 0;)
            c->hll_free.push_back({chunk + i * kHllBytes, words + i * kHllStateWords, ops + i * (kHllOpsBytes / 2)});
    }
    auto h = std::make_shared<HllState>();
    const auto slot = c->hll_free.back();
    h->d_regs = slot.regs;
    h->d_promoted = slot.state;
    h->d_sp_ops = h->d_slot_ops = slot.ops;
    c->hll_free.pop_back();
    h->owner = c;
    c->refs.fetch_add(1);
    // every slot in hll_free is zero: registers 0, state 0 (not promoted, the createHLLObject
    // sparse string: one XZERO)
    *out = h;
    return RBX_OK;
}

// =====================================================================================
// helpers
// =====================================================================================
static int set_device(rbx_ctx *c) {
    if (c->shut) return fail(RBX_E_ILLEGAL_STATE, "the context has been shut down");
    HIP_TRY(hipSetDevice(c->device));
    return RBX_OK;
}

static hipStream_t pick_stream(rbx_ctx *c, void *s) { return s ? (hipStream_t)s : c->stream; }

// A zeroed bitmap of size_bits bits; the fill runs on `st` inside the caller's ScratchOrder.
static int new_bitmap(rbx_ctx *c, uint64_t size_bits, hipStream_t st, std::shared_ptr<Bitmap> *out) {
    auto b = std::make_shared<Bitmap>();
    b->device = c->device;
    uint64_t bytes = ((size_bits + 7) / 8 + 255) & ~255ULL;
    if (bytes == 0) bytes = 256;
    if (bytes <= SlabPool::kMaxSmall) {  // words + a 256-byte tail holding the length word
        uint8_t *p = (uint8_t *)c->slab->get(bytes + 256);
        if (!p) return fail(RBX_E_OOM, "bitmap slab allocation failed");
        b->pool = c->slab;
        b->d_words = (uint32_t *)p;
        b->d_len = (unsigned long long *)(p + bytes);
    } else {
        HIP_TRY(hipMalloc(&b->d_words, bytes));
        HIP_TRY(hipMalloc(&b->d_len, sizeof(unsigned long long)));
    }
    if (b->pool) {  // the words and the length word's 256-byte tail: one fill
        HIP_TRY(hipMemsetAsync(b->d_words, 0, bytes + 256, st));
    } else {
        HIP_TRY(hipMemsetAsync(b->d_words, 0, bytes, st));
        HIP_TRY(hipMemsetAsync(b->d_len, 0, sizeof(unsigned long long), st));
    }
    b->cap_bytes = bytes;
    c->ks.generation++;
    *out = b;
    return RBX_OK;
}

static int grow_bitmap(rbx_ctx *c, Bitmap &b, uint64_t size_bits, hipStream_t st) {
    uint64_t bytes = ((size_bits + 7) / 8 + 255) & ~255ULL;
    if (bytes <= b.cap_bytes) return RBX_OK;
    // always move to a dedicated allocation (words + length word)
    uint32_t *nw = nullptr;
    unsigned long long *nl = nullptr;
    HIP_TRY(hipMalloc(&nw, bytes));
    HIP_TRY(hipMalloc(&nl, sizeof(unsigned long long)));
    HIP_TRY(hipMemsetAsync(nw, 0, bytes, st));
    HIP_TRY(hipMemcpyAsync(nw, b.d_words, b.cap_bytes, hipMemcpyDeviceToDevice, st));
    HIP_TRY(hipMemcpyAsync(nl, b.d_len, sizeof(unsigned long long), hipMemcpyDeviceToDevice, st));
    HIP_TRY(hipStreamSynchronize(st));
    if (b.pool) {
        b.pool->put(b.d_words, b.cap_bytes + 256);
        b.pool.reset();
    } else {
        HIP_TRY(hipFree(b.d_words));
        HIP_TRY(hipFree(b.d_len));
    }
    b.d_words = nw;
    b.d_len = nl;
    b.cap_bytes = bytes;
    c->ks.generation++;
    return RBX_OK;
}

static uint64_t read_dev_u64(rbx_ctx *c, const unsigned long long *p, int *rc) {
    unsigned long long v = 0;
    // into a pinned word: a pageable destination costs the runtime a staging copy
    hipError_t e = hipMemcpyAsync(c->pin_word, p, 8, hipMemcpyDeviceToHost, c->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    if (e == hipSuccess) v = *c->pin_word;
    *rc = e == hipSuccess ? RBX_OK : fail(RBX_E_DEVICE, hipGetErrorString(e));
    return v;
}

static const char *kWrongTypeMsg = "WRONGTYPE Operation against a key holding the wrong kind of value";

// Redis bit offsets end at 2^32 - 1: a filter whose |size| exceeds 2^32 (only reachable through
// tryInit with a negative expectedInsertions, M/RedissonBloomFilter.java:270-276) gets the error
// SETBIT/GETBIT would reply with.
static int check_offsets(int64_t size) {
    if (size_bits(size) > kEngineMaxSize) return fail(RBX_E_REDIS, "ERR bit offset is not an integer or out of range");
    return RBX_OK;
}

// =====================================================================================
// key arenas: host -> device staging
// =====================================================================================
static int fast_len(const KeysDev &k) {
    if (k.offsets) return 0;
    if (((uintptr_t)k.bytes & 15) != 0) return 0;
    if (k.stride == 16 || k.stride == 32 || k.stride == 64) return (int)k.stride;
    return 0;
}

static int fast_len_hll(const KeysDev &k) {
    if (k.offsets) return 0;
    if (k.stride == 16 || k.stride == 32 || k.stride == 64) return ((uintptr_t)k.bytes & 15) ? 0 : (int)k.stride;
    if (k.stride == 8 && ((uintptr_t)k.bytes & 7) == 0) return 8;
    return 0;
}

static int validate_keys(const rbx_keys *k) {
    if (!k) return fail(RBX_E_ILLEGAL_ARGUMENT, "keys is NULL");
    if (k->n && !k->bytes && !(k->offsets == nullptr && k->stride == 0))
        return fail(RBX_E_ILLEGAL_ARGUMENT, "keys->bytes is NULL");
    return RBX_OK;
}

// Copies keys [i0, i1) of a host arena to device buffers; returns a device view with keys renumbered
// from 0 (the offsets as the caller's: KeysDev.off_base = offsets[i0]).
static int upload_keys(rbx_ctx *c, const rbx_keys *k, uint64_t i0, uint64_t i1, KeysDev *out) {
    uint64_t n = i1 - i0;
    if (k->offsets) {
        uint64_t b0 = k->offsets[i0], b1 = k->offsets[i1];
        RBX_TRY(c->keys_bytes.reserve(b1 - b0 + 16));
        RBX_TRY(c->keys_offs.reserve((n + 1) * 8));
        if (b1 > b0) HIP_TRY(hipMemcpyAsync(c->keys_bytes.p, k->bytes + b0, b1 - b0, hipMemcpyHostToDevice, c->stream));
        // the caller's offsets as they are (the kernels subtract off_base): no rebased copy on the stack,
        // so no sync before returning (a pageable source is staged by the runtime before the call returns)
        HIP_TRY(hipMemcpyAsync(c->keys_offs.p, k->offsets + i0, (n + 1) * 8, hipMemcpyHostToDevice, c->stream));
        *out = KeysDev{c->keys_bytes.as<uint8_t>(), c->keys_offs.as<uint64_t>(), 0, n, b0};
    } else {
        uint64_t bytes = n * k->stride;
        RBX_TRY(c->keys_bytes.reserve(bytes + 16));
        if (bytes) HIP_TRY(hipMemcpyAsync(c->keys_bytes.p, k->bytes + i0 * k->stride, bytes, hipMemcpyHostToDevice, c->stream));
        *out = KeysDev{c->keys_bytes.as<uint8_t>(), nullptr, k->stride, n};
    }
    return RBX_OK;
}

static uint64_t chunk_keys_for_upload(const rbx_keys *k, uint64_t i0) {
    // ~256 MiB of key bytes per upload chunk
    const uint64_t budget = 256ull << 20;
    if (!k->offsets) {
        uint64_t per = k->stride ? budget / k->stride : k->n;
        return std::max<uint64_t>(1, per);
    }
    uint64_t lo = i0, hi = k->n;
    // largest i1 with offsets[i1] - offsets[i0] <= budget (at least one key)
    while (hi - lo > 1) {
        uint64_t mid = (lo + hi) / 2;
        if (k->offsets[mid] - k->offsets[i0] <= budget) lo = mid;
        else hi = mid;
    }
    uint64_t i1 = (k->offsets[hi] - k->offsets[i0] <= budget) ? hi : lo;
    return std::max<uint64_t>(1, i1 - i0);
}

// =====================================================================================
// add(): chunked probe/commit over the first-setter table
// =====================================================================================
static int ensure_table(rbx_ctx *c, uint64_t want_pairs, hipStream_t st) {
    // capacity >= 2 * pairs per chunk; between 2^16 and 2^27 entries (2 GiB)
    uint32_t lg = 16;
    while (lg < 27 && (1ULL << lg) < 2 * want_pairs) ++lg;
    if (lg > c->log2cap) {
        RBX_TRY(c->table.reserve(sizeof(HTEntry) << lg));
        c->log2cap = lg;
        c->epoch = 255;
    }
    if (c->epoch >= 254) {
        HIP_TRY(hipMemsetAsync(c->table.p, 0xff, sizeof(HTEntry) << c->log2cap, st));
        c->epoch = 0;
    } else {
        c->epoch++;
    }
    return RBX_OK;
}

static int run_add_table(rbx_ctx *c, const KeysDev &keys, const FilterDesc *d_filt, const uint64_t *d_seg_off,
                         uint32_t nseg, const FilterDesc &single, uint32_t kmax, uint8_t *d_out_new,
                         unsigned long long *d_count, unsigned long long *d_seg_counts, hipStream_t st) {
    if (keys.n == 0) return RBX_OK;
    const uint64_t k = std::max<uint32_t>(kmax, 1);
    const bool narrow = d_filt == nullptr && kmax <= 32;
    // chunk so that pairs per chunk <= 2^26 (table <= 2^27 entries at load <= 1/2)
    uint64_t chunk = std::min<uint64_t>(keys.n, (1ULL << 26) / k);
    chunk = std::max<uint64_t>(chunk, 1);
    const size_t zbytes = kmax <= 32 ? chunk * 4 : chunk * (size_t)kmax;
    RBX_TRY(c->zmask.reserve(zbytes));
    const int fl = fast_len(keys);
    for (uint64_t base = 0; base < keys.n; base += chunk) {
        const uint64_t nch = std::min<uint64_t>(chunk, keys.n - base);
        AddChunkArgs a{};
        if (narrow) {
            uint32_t lg = 16;
            while (lg < 27 && (1ULL << lg) < 2 * nch * k) ++lg;
            RBX_TRY(c->table.reserve(8ull << lg));
            HIP_TRY(hipMemsetAsync(c->table.p, 0xff, 8ull << lg, st));
            c->epoch = 255;  // the wide (16-byte) layout must be re-initialised before reuse
            a.log2cap = lg;
        } else {
            RBX_TRY(ensure_table(c, nch * k, st));
            a.log2cap = c->log2cap;
            a.epoch = c->epoch;
        }
        a.keys = keys;
        a.base = base;
        a.nchunk = nch;
        a.filt = d_filt;
        a.seg_off = d_seg_off;
        a.nseg = nseg;
        a.tile_seg0 = c->tile_segs.as<uint32_t>();
        a.single = single;
        a.table = c->table.as<HTEntry>();
        a.zmask = c->zmask.as<uint32_t>();
        a.kmax = kmax;
        a.out_new = d_out_new;
        a.count = d_count;
        a.seg_counts = d_seg_counts;
        a.narrow = narrow;
        launch_bloom_add_chunk(a, fl, st);
        HIP_TRY(hipGetLastError());
    }
    return RBX_OK;
}

// Partitioned add (add_partitioned.hip) for one large filter.  Mode: 0 never, 1 whenever
// k <= 16, 2 (default) when the bitmap is >= 8 MiB and the batch has >= max(2^17, size / 2^12)
// keys.  The region pass reads and writes every touched region of the bitmap, so its floor
// grows with the bitmap (0.7 ms at 512 MiB) while the table path's cost grows with the batch
// (0.7 us per 1K keys): crossovers ~150K keys at 12-32 MiB, ~1M at 512 MiB
// (tools/microbench.py addsweep, profiles/r02/r02h_addsweep_table_vs_partitioned.jsonl).
static std::atomic<int> g_add_partition_mode{2};
static std::atomic<int> g_add_partition_diag{0};
static std::atomic<int> g_add_record_policy{2};

static bool use_add_partitioned(uint64_t size, uint32_t k, uint64_t n) {
    if (k < 1 || k > 16 || size > (1ULL << 32) || size < (1ULL << 15)) return false;
    if (g_add_partition_mode == 0) return false;
    if (g_add_partition_mode == 1) return true;
    return size >= (1ULL << 26) && n >= std::max<uint64_t>(1ULL << 17, size >> 12);
}

static KeysDev keys_slice(const KeysDev &k, uint64_t i0, uint64_t n) {
    KeysDev s = k;
    s.n = n;
    if (k.offsets) s.offsets = k.offsets + i0;  // offsets stay absolute (off_base unchanged)
    else s.bytes = k.bytes + i0 * k.stride;
    return s;
}

static int run_add_partitioned(rbx_ctx *c, const KeysDev &keys, const FilterDesc &f, uint8_t *d_out_new,
                               unsigned long long *d_count, hipStream_t st) {
    const uint32_t k = f.k;
    const uint64_t size = f.mp.size;
    const uint32_t nregions = (uint32_t)((size + (1ULL << kBaRegionBits) - 1) >> kBaRegionBits);
    uint32_t L = 0;
    while ((1ULL << L) < nregions) ++L;
    // two radix passes: stage 1 into 2^(L - f3) <= 256 buckets, one rebucket of fan-out 2^f3 <= 256
    const uint32_t f3 = std::min<uint32_t>(8, L);
    const uint32_t s3 = kBaRegionBits, s1 = s3 + f3;
    const uint32_t ncoarse = (uint32_t)((size + (1ULL << s1) - 1) >> s1);  // <= 256 for size <= 2^32
    // chunk: key ids < 2^26 and the expected pairs per region (x 1.3 slack) within the block's registers
    const double per_region = (double)k * (double)(1ULL << kBaRegionBits) / (double)size;  // pairs per key
    uint64_t chunk = (uint64_t)((kBaMaxRegionPairs - 512) / 1.3 / per_region);
    chunk = std::min<uint64_t>(chunk, 1ULL << 26);
    const uint64_t nch = (keys.n + chunk - 1) / chunk;
    chunk = (keys.n + nch - 1) / nch;
    const double pairs = (double)chunk * k;
    auto cap_of = [&](uint32_t shift, double slack, uint64_t add, uint64_t round) {
        const double frac = std::min(1.0, (double)(1ULL << shift) / (double)size);
        uint64_t cap = (uint64_t)(pairs * frac * slack) + add;
        return (cap + round - 1) / round * round;
    };
    const uint64_t cap1 = cap_of(s1, 1.15 / kBaSub, 8192, 8192);
    const uint64_t cap3 = std::min<uint64_t>(kBaMaxRegionPairs, cap_of(s3, 1.3, 256, 64));
    RBX_TRY(c->pa_p1.reserve((uint64_t)ncoarse * kBaSub * cap1 * 8));
    RBX_TRY(c->pa_p2.reserve((uint64_t)nregions * cap3 * 8));
    const uint32_t nranges = (uint32_t)((chunk + (1ULL << kBaKeyRangeBits) - 1) >> kBaKeyRangeBits);
    const uint64_t cap_rec = (uint64_t)k << kBaKeyRangeBits;  // a range's owner records <= 2^20 keys x k
    RBX_TRY(c->pa_recs.reserve((uint64_t)nranges * cap_rec * 4));
    const uint64_t ncnt = (uint64_t)ncoarse * kBaSub + nregions + nranges + 2;
    RBX_TRY(c->pa_cnt.reserve(ncnt * 4));
    const uint64_t nbw = (uint64_t)nranges << (kBaKeyRangeBits - 5);  // whole ranges (the records kernel's images)
    RBX_TRY(c->pa_bits.reserve(nbw * 4));
    // per-key non-owner counters (one byte per key; k_ba_final zeroes what it read): zeroed once
    // when (re)allocated
    if (c->pa_ctr.cap < nbw * 32) {
        RBX_TRY(c->pa_ctr.reserve(nbw * 32));
        HIP_TRY(hipMemsetAsync(c->pa_ctr.p, 0, c->pa_ctr.cap, st));
    }
    const int fl = fast_len(keys);
    for (uint64_t base = 0; base < keys.n; base += chunk) {
        BaArgs a{};
        a.keys = keys;
        a.base = base;
        a.nchunk = std::min<uint64_t>(chunk, keys.n - base);
        a.f = f;
        a.ncoarse = ncoarse;
        a.s1 = s1;
        a.s3 = s3;
        a.f3 = f3;
        a.nregions = nregions;
        a.cap1 = cap1;
        a.cap3 = cap3;
        a.p1 = c->pa_p1.as<unsigned long long>();
        a.p3 = c->pa_p2.as<unsigned long long>();
        a.cnt1 = c->pa_cnt.as<uint32_t>();
        a.cnt3 = a.cnt1 + (uint64_t)ncoarse * kBaSub;
        a.rec_cnt = a.cnt3 + nregions;
        a.overflow = a.rec_cnt + nranges;
        a.mode = a.overflow + 1;
        a.recs = c->pa_recs.as<uint32_t>();
        a.cap_rec = cap_rec;
        a.nranges = (uint32_t)((a.nchunk + (1ULL << kBaKeyRangeBits) - 1) >> kBaKeyRangeBits);
        a.record_policy = (uint32_t)g_add_record_policy;
        a.new_bits = c->pa_bits.as<uint32_t>();
        a.ctr = c->pa_ctr.as<uint32_t>();
        a.nwords4 = (size + 127) / 128 * 4;
        a.out_new = d_out_new;
        a.count = d_count;
        a.diag = (uint32_t)g_add_partition_diag;
        if (a.diag & 64) {
            if (c->pa_stamps.cap == 0) {
                RBX_TRY(c->pa_stamps.reserve(16 * 8));
                HIP_TRY(hipMemsetAsync(c->pa_stamps.p, 0, 16 * 8, st));
            }
            a.stamps = c->pa_stamps.as<unsigned long long>();
        }
        // the counters (but the mode word) and new_bits are zeroed by k_ba_mode, the chunk's first kernel
        launch_add_partitioned_chunk(a, fl, st);
        HIP_TRY(hipGetLastError());
        HIP_TRY(hipMemcpyAsync(c->pin_word, a.overflow, 4, hipMemcpyDeviceToHost, st));  // pinned: no staging copy
        HIP_TRY(hipStreamSynchronize(st));
        uint32_t ovf;
        memcpy(&ovf, c->pin_word, 4);
        if (ovf) {
            // a bucket overflowed before any bitmap word changed: this chunk on the table path
            const KeysDev sub = keys_slice(keys, base, a.nchunk);
            RBX_TRY(run_add_table(c, sub, nullptr, nullptr, 0, f, k, d_out_new ? d_out_new + base : nullptr, d_count,
                                  nullptr, st));
        }
    }
    return RBX_OK;
}

// Small single-filter adds (<= add_single_seg_keys keys, k <= 16): the per-segment kernel on one segment --
// one workgroup, the batch's first setters in LDS (§3.9) -- instead of the table path's memset, probe and
// commit: one launch.  Its plain word stores need the bitmap to itself, which the context's call order
// gives (every call waits for the previous one's stream, ScratchOrder).
static std::atomic<uint64_t> g_seg_single_keys{256};  // rbx_tune("add_single_seg_keys"): 0 = off
static std::atomic<int> g_add_one{1};  // rbx_tune("add_one_key"): 1 = a 1-key add takes k_bloom_add_one

static bool use_seg_single(const FilterDesc &f, uint64_t n, uint64_t lim) { return f.k <= 16 && n <= lim; }

static void launch_seg_single(const KeysDev &keys, const FilterDesc &f, uint8_t *d_out_new,
                              unsigned long long *d_count, hipStream_t st) {
    MaddSegArgs a{};
    a.keys = keys;
    a.single = f;
    a.kmax = f.k;
    a.segmax = kSegMaxKeys;  // >= keys.n: the `big` flag stays unused
    a.out_new = d_out_new;
    a.seg_counts = d_count;
    launch_madd_seg(a, fast_len(keys), st);
}

static int run_add(rbx_ctx *c, const KeysDev &keys, const FilterDesc *d_filt, const uint64_t *d_seg_off,
                   uint32_t nseg, const FilterDesc &single, uint32_t kmax, uint8_t *d_out_new,
                   unsigned long long *d_count, unsigned long long *d_seg_counts, hipStream_t st) {
    if (keys.n == 0) return RBX_OK;
    if (d_filt == nullptr && keys.n == 1 && single.k <= 16 && g_add_one) {
        launch_bloom_one(true, keys, fast_len(keys), single, d_out_new, d_count, nullptr, 0, st);
        HIP_TRY(hipGetLastError());
        return RBX_OK;
    }
    if (d_filt == nullptr && use_seg_single(single, keys.n, g_seg_single_keys)) {
        launch_seg_single(keys, single, d_out_new, d_count, st);
        HIP_TRY(hipGetLastError());
        return RBX_OK;
    }
    if (d_filt == nullptr && use_add_partitioned(single.mp.size, single.k, keys.n))
        return run_add_partitioned(c, keys, single, d_out_new, d_count, st);
    return run_add_table(c, keys, d_filt, d_seg_off, nseg, single, kmax, d_out_new, d_count, d_seg_counts, st);
}

// Partitioned contains (contains_partitioned.hip) for one large filter.  Mode: 0 never,
// 1 whenever k in [2, 16], 2 (default) when the bitmap is >= 256 MiB and the batch >= 4M keys.
// Below 256 MiB the direct kernel measured faster (its early exit costs ~1 gather per absent
// key, and smaller bitmaps gather partly from L2/MALL); DESIGN.md §3.6 has the size sweep.
static std::atomic<int> g_partition_mode{2};
static std::atomic<int> g_partition_flags{0};

static bool use_partitioned(uint64_t size, uint32_t k, uint64_t n) {
    if (k < 2 || k > 16 || size > (1ULL << 32)) return false;
    if (g_partition_mode == 0) return false;
    if (g_partition_mode == 1) return true;
    return size >= (1ULL << 31) && n >= (1ULL << 22);
}

static int run_contains_partitioned(rbx_ctx *c, const KeysDev &keys, const FilterDesc &f, uint8_t *d_out,
                                    unsigned long long *d_count, hipStream_t st) {
    const uint32_t k = f.k;
    const uint64_t size = f.mp.size;
    const uint32_t nregions = (uint32_t)((size + (1ULL << kBkRegionBits) - 1) >> kBkRegionBits);
    uint32_t lg = 0;
    while ((1ULL << lg) < nregions) ++lg;
    const uint32_t fb = lg > 6 ? lg - 6 : 0;
    const uint32_t ncoarse = (nregions + (1u << fb) - 1) >> fb;
    // keys per chunk: key ids fit 27 bits (6-byte region pairs) and a chunk's pairs stay <= 2^30
    uint64_t chunk = std::min<uint64_t>(1ULL << 27, (1ULL << 30) / (k - 1));
    const uint64_t nch = (keys.n + chunk - 1) / chunk;
    chunk = (keys.n + nch - 1) / nch;
    chunk = (chunk + 1023) / 1024 * 1024;
    const uint64_t ngroups = (chunk + 63) / 64;
    // capacities assume every key survives stage 1; pairs spread uniformly over [0, size)
    const double pairs_max = (double)chunk * (k - 1);
    const double frac1 = std::min(1.0, (double)(1ULL << (kBkRegionBits + fb)) / (double)size);
    const double frac2 = std::min(1.0, (double)(1ULL << kBkRegionBits) / (double)size);
    uint64_t cap1 = (uint64_t)(pairs_max * frac1 / kBkSub * 1.15) + 8192;
    uint64_t cap2 = (uint64_t)(pairs_max * frac2 * 1.2) + 4096;
    cap1 = (cap1 + 8191) / 8192 * 8192;
    cap2 = (cap2 + 63) / 64 * 64;
    RBX_TRY(c->pc_bits.reserve(ngroups * 16));
    const uint32_t nmranges = (uint32_t)((chunk + (1ULL << kBkMissRangeBits) - 1) >> kBkMissRangeBits);
    // miss records: sized for 2 per key (C2-like batches hold ~0.2); beyond that the probe falls
    // back to a direct atomicOr per clear bit, so the answer never depends on the capacity
    const uint64_t capm = 2ULL << kBkMissRangeBits;
    RBX_TRY(c->pc_mrec.reserve((uint64_t)nmranges * capm * 4));
    const uint64_t ncnt = 64 * kBkSub + (uint64_t)nregions + 256;  // cnt1 (padded), cnt2, mcnt
    RBX_TRY(c->pc_cnt.reserve(ncnt * 4));
    RBX_TRY(c->pc_pairs1.reserve((uint64_t)ncoarse * kBkSub * cap1 * 8));
    RBX_TRY(c->pc_pairs2.reserve((uint64_t)nregions * cap2 * 6));  // 6-byte region pairs (lo u32 + hi u16)
    const int fl = fast_len(keys);
    for (uint64_t base = 0; base < keys.n; base += chunk) {
        PcArgs a{};
        a.keys = keys;
        a.base = base;
        a.nchunk = std::min<uint64_t>(chunk, keys.n - base);
        a.bm = f.bm;
        a.mp = f.mp;
        a.k = k;
        a.nregions = nregions;
        a.fb = fb;
        a.cshift = kBkRegionBits + fb;
        a.ncoarse = ncoarse;
        a.cap1 = cap1;
        a.cap2 = cap2;
        a.nwords4 = (size + 127) / 128 * 4;
        a.alive = c->pc_bits.as<unsigned long long>();
        a.miss = a.alive + ngroups;
        a.cnt1 = c->pc_cnt.as<uint32_t>();
        a.cnt2 = a.cnt1 + 64 * kBkSub;
        a.pairs1 = c->pc_pairs1.as<unsigned long long>();
        a.p2lo = c->pc_pairs2.as<uint32_t>();
        a.p2hi = (uint16_t *)(a.p2lo + (uint64_t)nregions * cap2);
        a.mrec = c->pc_mrec.as<uint32_t>();
        a.mcnt = a.cnt2 + nregions;
        a.capm = capm;
        a.nmranges = (uint32_t)((a.nchunk + (1ULL << kBkMissRangeBits) - 1) >> kBkMissRangeBits);
        a.out = d_out;
        a.count = d_count;
        a.flags = (uint32_t)g_partition_flags;
        if (a.flags & 64) {
            if (c->pa_stamps.cap == 0) {
                RBX_TRY(c->pa_stamps.reserve(16 * 8));
                HIP_TRY(hipMemsetAsync(c->pa_stamps.p, 0, 16 * 8, st));
            }
            a.stamps = c->pa_stamps.as<unsigned long long>();
        }
        HIP_TRY(hipMemsetAsync(a.miss, 0, ngroups * 8, st));
        HIP_TRY(hipMemsetAsync(a.cnt1, 0, ncnt * 4, st));
        launch_contains_partitioned_chunk(a, fl, st);
        HIP_TRY(hipGetLastError());
    }
    return RBX_OK;
}

// contains over device keys for one filter: direct (staged early exit) or partitioned
static int run_contains(rbx_ctx *c, const KeysDev &keys, const FilterDesc &f, uint8_t *d_out,
                        unsigned long long *d_count, hipStream_t st) {
    if (use_partitioned(f.mp.size, f.k, keys.n)) return run_contains_partitioned(c, keys, f, d_out, d_count, st);
    launch_bloom_contains(keys, fast_len(keys), f.bm, f.mp, f.k, d_out, d_count, st);
    HIP_TRY(hipGetLastError());
    return RBX_OK;
}

static FilterDesc desc_of(const Bitmap &b, uint64_t size, uint32_t k, uint32_t fid) {
    FilterDesc f{};
    f.bm = b.d_words;
    f.redis_len = b.d_len;
    f.mp = make_mod_params(size);
    f.k = k;
    f.fid = fid;
    return f;
}

// =====================================================================================
// extern "C"
// =====================================================================================
// Names arrive as NUL-terminated strings or, in the *_n forms, as (bytes, length) pairs that may
// hold any byte (Spring Data's byte[] keys, RedissonConnection.java:2203).
static std::string name_of(const rbx_name &n) { return std::string((const char *)n.bytes, (size_t)n.len); }

extern "C" {

int rbx_abi_version(void) { return RBX_ABI_VERSION; }

const char *rbx_last_error(void) { return last_error_message(); }

int rbx_device_count(int *out) {
    int n = 0;
    hipError_t e = hipGetDeviceCount(&n);
    if (e != hipSuccess) n = 0;
    if (out) *out = n;
    return RBX_OK;
}

int rbx_init(int device, rbx_ctx **out) {
    if (!out) return fail(RBX_E_ILLEGAL_ARGUMENT, "out is NULL");
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n == 0) return fail(RBX_E_DEVICE, "no HIP device available");
    if (device < 0 || device >= n) return fail(RBX_E_ILLEGAL_ARGUMENT, "device index out of range");
    auto *c = new rbx_ctx();
    c->device = device;
    hipError_t e = hipSetDevice(device);
    if (e == hipSuccess) e = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking);
    if (e == hipSuccess) e = hipStreamCreateWithFlags(&c->copy_stream, hipStreamNonBlocking);
    for (int i = 0; i < 2 && e == hipSuccess; ++i) {
        e = hipEventCreateWithFlags(&c->ev_copied[i], hipEventDisableTiming);
        if (e == hipSuccess) e = hipEventCreateWithFlags(&c->ev_done[i], hipEventDisableTiming);
        if (e == hipSuccess && i == 0) e = hipEventCreateWithFlags(&c->ev_scratch, hipEventDisableTiming);
    }
    if (e == hipSuccess) e = hipHostMalloc((void **)&c->pin_word, 64, hipHostMallocDefault);
    if (e != hipSuccess) {
        delete c;
        return fail(RBX_E_DEVICE, hipGetErrorString(e));
    }
    *out = c;
    return RBX_OK;
}

// Frees the device resources now; the context object itself lives until its last handle is
// closed (closing a handle after shutdown is safe, every other call on it fails).
int rbx_shutdown(rbx_ctx *c) {
    if (!c) return RBX_OK;
    // Queued asynchronous calls run to completion first (they take the context lock themselves):
    // the executor is taken out under exec_mu (later submits are refused), then destroyed, which
    // runs its queue and joins its thread.  From a completion callback (the executor's own
    // thread) it cannot join itself: it is detached, runs what is queued -- those calls fail with
    // RBX_E_ILLEGAL_STATE once the context is shut -- and frees itself.
    std::unique_ptr<SerialExecutor> ex;
    {
        std::lock_guard<std::mutex> g(c->exec_mu);
        ex = std::move(c->exec);
    }
    if (ex) {
        if (ex->on_executor_thread()) SerialExecutor::release_from_inside(ex.release());
        else ex.reset();
    }
    {
        std::lock_guard<std::recursive_mutex> g(c->ks.mu);
        if (c->shut) return fail(RBX_E_ILLEGAL_STATE, "the context has already been shut down");
        (void)hipSetDevice(c->device);
        (void)hipDeviceSynchronize();  // work queued on caller streams may still use the memory
        if (c->comm) ncclCommDestroy(c->comm);
        c->comm = nullptr;
        c->shut = true;  // from here on released HLL blocks are not recycled
        c->ks.clear();
        for (auto *p : c->hll_chunks) (void)hipFree(p);
        c->hll_chunks.clear();
        c->hll_free.clear();
        c->hll_dirty.clear();
        c->st_t8_entries = 0;
        c->slab.reset();  // bitmaps still held by open handles keep their slab alive
        for (DevBuf *b : {&c->table, &c->zmask, &c->keys_bytes, &c->keys_offs, &c->out_bytes, &c->seg_offs,
                          &c->counters, &c->filt_table, &c->probe_table, &c->ptrs, &c->histo, &c->misc, &c->tile_segs,
                          &c->hll_tiles, &c->pc_bits, &c->pc_cnt, &c->pc_pairs1, &c->pc_pairs2, &c->pc_mrec,
                          &c->pa_p1, &c->pa_p2, &c->pa_cnt, &c->pa_bits, &c->pa_ctr, &c->pa_recs, &c->st_adds,
                          &c->st_nadds, &c->zero_bm, &c->hll_pack, &c->slot_bytes[0], &c->slot_bytes[1],
                          &c->slot_offs[0], &c->slot_offs[1], &c->st_t8, &c->fid_table,
                          &c->hll_zero_ptrs, &c->wide_table, &c->st_fslot, &c->madd_c}) {
            if (b->p) (void)hipFree(b->p);
            b->p = nullptr;
            b->cap = 0;
        }
        for (int i = 0; i < 2; ++i) {
            if (c->ev_copied[i]) (void)hipEventDestroy(c->ev_copied[i]);
            if (c->ev_done[i]) (void)hipEventDestroy(c->ev_done[i]);
            c->ev_copied[i] = c->ev_done[i] = nullptr;
        }
        if (c->ev_scratch) (void)hipEventDestroy(c->ev_scratch);
        c->ev_scratch = nullptr;
        if (c->pin_small) (void)hipHostFree(c->pin_small);
        c->pin_small = nullptr;
        c->pin_small_cap = 0;
        c->pin_small_limit = 0;
        if (c->pin_word) (void)hipHostFree(c->pin_word);
        c->pin_word = nullptr;
        if (c->pin_tiny) (void)hipHostFree(c->pin_tiny);
        c->pin_tiny = c->pin_tiny_dev = nullptr;
        if (c->copy_stream) (void)hipStreamDestroy(c->copy_stream);
        if (c->stream) (void)hipStreamDestroy(c->stream);
        c->copy_stream = c->stream = nullptr;
    }
    ctx_release(c);
    return RBX_OK;
}

int rbx_synchronize(rbx_ctx *c) {
    if (!c) return fail(RBX_E_ILLEGAL_ARGUMENT, "ctx is NULL");
    std::lock_guard<std::recursive_mutex> g(c->ks.mu);
    RBX_TRY(set_device(c));
    HIP_TRY(hipStreamSynchronize(c->stream));
    return RBX_OK;
}

void *rbx_stream(rbx_ctx *c) { return c && !c->shut ? (void *)c->stream : nullptr; }

// ---- CRC16 / slots (keyspace.cpp) ------------------------------------------------------------
uint16_t rbx_crc16(const uint8_t *bytes, size_t len) { return crc16(bytes, len); }
int rbx_calc_slot(const uint8_t *key, size_t len) { return calc_slot(key, len); }
int rbx_slot_to_gpu(int slot, int n_gpus) { return slot_to_gpu(slot, n_gpus); }

int rbx_bloom_optimal_config(int64_t n, double p, int64_t *size, uint32_t *k) {
    int64_t s;
    uint32_t kk;
    RBX_TRY(optimal_config(n, p, kRedissonMaxSize, &s, &kk));
    if (size) *size = s;
    if (k) *k = kk;
    return RBX_OK;
}

// ---- Bloom: config (keyspace.cpp) -----------------------------------------------------------------
int rbx_bloom_try_init_n(rbx_ctx *c, rbx_name name, int64_t expected, double fpp, int *created) {
    if (!c || (!name.bytes && name.len)) return fail(RBX_E_ILLEGAL_ARGUMENT, "ctx/name is NULL");
    return ks_bloom_try_init(c->ks, name_of(name), expected, fpp, created);
}

int rbx_bloom_try_init(rbx_ctx *c, const char *name, int64_t expected, double fpp, int *created) {
    if (!c || !name) return fail(RBX_E_ILLEGAL_ARGUMENT, "ctx/name is NULL");
    return ks_bloom_try_init(c->ks, name, expected, fpp, created);
}

int rbx_bloom_init_raw(rbx_ctx *c, const char *name, uint64_t size, uint32_t k, int *created) {
    if (!c || !name) return fail(RBX_E_ILLEGAL_ARGUMENT, "ctx/name is NULL");
    return ks_bloom_init_raw(c->ks, name, size, k, created);
}

static int read_config(rbx_ctx *c, const std::string &name, rbx_bloom_config *out) {
    BloomConfig cfg;
    RBX_TRY(ks_get_config(c->ks, name, &cfg));
    out->size = cfg.size;
    out->hash_iterations = cfg.k;
    out->expected_insertions = cfg.expected;
    out->false_probability = cfg.fpp;
    snprintf(out->false_probability_str, sizeof out->false_probability_str, "%s", cfg.fpp_str.c_str());
    return RBX_OK;
}

int rbx_bloom_read_config(rbx_ctx *c, const char *name, rbx_bloom_config *out) {
    if (!c || !name || !out) return fail(RBX_E_ILLEGAL_ARGUMENT, "NULL argument");
    return read_config(c, name, out);
}

int rbx_bloom_read_config_n(rbx_ctx *c, rbx_name name, rbx_bloom_config *out) {
    if (!c || (!name.bytes && name.len) || !out) return fail(RBX_E_ILLEGAL_ARGUMENT, "NULL argument");
    return read_config(c, name_of(name), out);
}

// bitmap key for add (created by the first SETBIT) / contains (may be absent).  size_bits_ =
// |size|; a new or grown bitmap is zero-filled on `st` (the caller holds a ScratchOrder on it).
static int bitmap_for(rbx_ctx *c, const std::string &name, uint64_t nbits, bool create, hipStream_t st,
                      std::shared_ptr<Bitmap> *out) {
    Entry *e = c->ks.find(name);
    if (e) {
        if (e->type != KType::Bitmap) return fail(RBX_E_WRONGTYPE, kWrongTypeMsg);
        RBX_TRY(grow_bitmap(c, *e->bm, nbits, st));
        *out = e->bm;
        return RBX_OK;
    }
    if (!create) {
        out->reset();
        return RBX_OK;
    }
    std::shared_ptr<Bitmap> b;
    RBX_TRY(new_bitmap(c, nbits, st, &b));
    c->ks.put(name, Entry{KType::Bitmap, nullptr, b, nullptr});
    *out = b;
    return RBX_OK;
}

// Runs fn(chunk view, chunk index range) over a host arena in chunks of ~staging_bytes:
// chunk j is uploaded on copy_stream into slot j%2 while chunk j-1 computes on `st`.
}  // extern "C"
template <class Fn>
static int pipelined_host_batches(rbx_ctx *c, const rbx_keys *k, hipStream_t st, Fn &&fn) {
    uint64_t j = 0;
    for (uint64_t i0 = 0; i0 < k->n; ++j) {
        // chunk [i0, i1) of <= staging_bytes key bytes (at least one key)
        uint64_t i1;
        if (k->offsets) {
            uint64_t lo = i0 + 1, hi = k->n;
            const uint64_t b0 = k->offsets[i0];
            if (k->offsets[hi] - b0 <= c->staging_bytes) {
                lo = hi;
            } else {
                while (hi - lo > 0) {  // largest i1 >= i0+1 with bytes <= staging
                    const uint64_t mid = (lo + hi + 1) / 2;
                    if (k->offsets[mid] - b0 <= c->staging_bytes) lo = mid;
                    else hi = mid - 1;
                }
            }
            i1 = lo;
        } else {
            const uint64_t per = k->stride ? std::max<uint64_t>(1, c->staging_bytes / k->stride) : k->n;
            i1 = std::min<uint64_t>(k->n, i0 + per);
        }
        const int s = (int)(j & 1);
        const uint64_t n = i1 - i0;
        const uint64_t b0 = k->offsets ? k->offsets[i0] : i0 * k->stride;
        const uint64_t nb = k->offsets ? k->offsets[i1] - b0 : n * k->stride;
        RBX_TRY(c->slot_bytes[s].reserve(nb + 16));
        if (k->offsets) RBX_TRY(c->slot_offs[s].reserve((n + 1) * 8));
        HIP_TRY(hipStreamWaitEvent(c->copy_stream, c->ev_done[s], 0));
        if (nb) HIP_TRY(hipMemcpyAsync(c->slot_bytes[s].p, k->bytes + b0, nb, hipMemcpyHostToDevice, c->copy_stream));
        if (k->offsets)
            HIP_TRY(hipMemcpyAsync(c->slot_offs[s].p, k->offsets + i0, (n + 1) * 8, hipMemcpyHostToDevice, c->copy_stream));
        HIP_TRY(hipEventRecord(c->ev_copied[s], c->copy_stream));
        HIP_TRY(hipStreamWaitEvent(st, c->ev_copied[s], 0));
        KeysDev dk{c->slot_bytes[s].as<uint8_t>(), k->offsets ? c->slot_offs[s].as<uint64_t>() : nullptr, k->stride, n,
                   k->offsets ? b0 : 0};
        RBX_TRY(fn(dk, i0));
        HIP_TRY(hipEventRecord(c->ev_done[s], st));
        i0 = i1;
    }
    return RBX_OK;
}
extern "C" {

// add / contains of a filter whose |size| exceeds 2^32 bits (tryInit with a negative
// expectedInsertions, M/RedissonBloomFilter.java:262-277), with the reference's semantics: indexes
// are taken mod |size| in 64 bits; a SETBIT / GETBIT past the Redis offset limit is an error reply
// that leaves the key alone while every other command of the batch runs; the call then fails with
// RBX_E_REDIS (RedisException) -- an add has set every in-range bit.  Without such an index the
// replies are the in-order ones.  Chunks run in key order (each sees the previous chunks' bits).
// rbx_tune("wide_subchunk", n): keys per sub-chunk cap (0 = default 2^29 / k; tests split small batches)
static std::atomic<uint64_t> g_wide_subchunk{0};
static int bloom_wide_op(rbx_ctx *c, const rbx_keys *keys, uint64_t m, uint32_t k, Bitmap *bm, uint8_t *out_flags,
                         uint64_t *out_count, bool is_add) {
    RBX_TRY(c->counters.reserve(64));
    auto *d_count = c->counters.as<unsigned long long>();
    auto *d_oob = d_count + 4;
    HIP_TRY(hipMemsetAsync(d_count, 0, 8, c->stream));
    HIP_TRY(hipMemsetAsync(d_oob, 0, 8, c->stream));
    uint8_t *d_out = nullptr;
    if (out_flags) {
        RBX_TRY(c->out_bytes.reserve(keys->n));
        d_out = c->out_bytes.as<uint8_t>();
    }
    HIP_TRY(hipStreamSynchronize(c->stream));
    RBX_TRY(pipelined_host_batches(c, keys, c->stream, [&](const KeysDev &dk, uint64_t i0) -> int {
        // Sub-chunks of <= 2^29 / k keys, run in key order (each sees the previous one's bits), so
        // the first-setter table (>= 2x the sub-chunk's bit indexes) stays <= 2^30 entries (8 GiB)
        // and its 32-bit slot mask well-defined however short the keys (a staging
        // chunk of empty keys is unbounded in count).
        uint64_t sub = std::max<uint64_t>(1, (1ULL << 29) / k);
        if (g_wide_subchunk) sub = std::min<uint64_t>(sub, g_wide_subchunk);
        for (uint64_t j0 = 0; j0 < dk.n; j0 += sub) {
            KeysDev sk = dk;
            sk.n = std::min<uint64_t>(sub, dk.n - j0);
            if (dk.offsets) sk.offsets = dk.offsets + j0;
            else sk.bytes = dk.bytes + j0 * dk.stride;
            uint32_t tl = 10;  // table >= 2x the sub-chunk's bit indexes
            while ((1ULL << tl) < 2 * sk.n * k) ++tl;
            if (tl > 30) return fail(RBX_E_ILLEGAL_ARGUMENT, "wide-filter table past 2^30 entries");
            unsigned long long *table = nullptr;
            if (is_add) {
                RBX_TRY(c->wide_table.reserve(8ULL << tl));
                table = c->wide_table.as<unsigned long long>();
                HIP_TRY(hipMemsetAsync(table, 0xff, 8ULL << tl, c->stream));
            }
            launch_bloom_wide(sk, m, k, bm ? bm->d_words : nullptr, bm ? bm->d_len : nullptr, table, tl, is_add,
                              d_out ? d_out + i0 + j0 : nullptr, d_count, d_oob, c->stream);
            HIP_TRY(hipGetLastError());
        }
        return RBX_OK;
    }));
    int rc;
    const uint64_t oob = read_dev_u64(c, d_oob, &rc);
    RBX_TRY(rc);
    if (oob) return fail(RBX_E_REDIS, "ERR bit offset is not an integer or out of range");
    if (out_flags) HIP_TRY(hipMemcpyAsync(out_flags, d_out, keys->n, hipMemcpyDeviceToHost, c->stream));
    const uint64_t cnt = read_dev_u64(c, d_count, &rc);
    RBX_TRY(rc);
    if (out_count) *out_count = is_add ? (uint64_t)(int64_t)(int32_t)cnt : cnt;  // add(): `int c`
    return RBX_OK;
}

// Small host batches -- the single-key add(T) / contains(T) Redisson sends most, and collections of up
// to host_small_bytes of key bytes (and a quarter as many keys): the keys are copied into pinned memory behind a zero
// count word and uploaded on the context stream in ONE transfer (no copy-stream hand-off, no sync before
// the launch: the slot's previous reader is waited for by its event), and the count and flags come back
// into the same pinned block with one sync.  (The pipelined path costs a fill, a sync, a copy-stream
// upload from pageable memory with two event hops, and a second sync: ~62 us for one key on the r05
// boxes, tools/microbench.py smallbatch.)
static std::atomic<int> g_small_host{1};  // rbx_tune("host_small_batches"): 0 = every host batch on the pipelined path
static std::atomic<uint64_t> g_small_bytes{4 << 20};  // rbx_tune("host_small_bytes"): the byte limit (keys <= limit / 4)
static constexpr uint64_t kSmallHead = 64 << 10;  // zeroed result area ahead of the keys (counts, changed words)
static size_t small_pin_bytes(uint64_t limit) { return kSmallHead + limit + limit / 4 + 64; }  // head | keys | tail

// the pinned block of the one-transfer path, laid out for host_small_bytes = limit (or a larger limit it
// already had); false (the caller takes the pipelined path) when pinned memory cannot be had
static bool small_pinned(rbx_ctx *c, uint64_t limit) {
    if (c->pin_small && c->pin_small_limit >= limit) return true;
    if (c->pin_small) (void)hipHostFree(c->pin_small);
    c->pin_small = nullptr;
    c->pin_small_cap = 0;
    c->pin_small_limit = 0;
    const size_t pin = small_pin_bytes(limit);
    if (hipHostMalloc(&c->pin_small, pin, hipHostMallocDefault) != hipSuccess) {
        (void)hipGetLastError();
        c->pin_small = nullptr;
        return false;
    }
    c->pin_small_cap = pin;
    c->pin_small_limit = limit;
    return true;
}

// the process-wide limit is read ONCE here (rbx_tune may change it on another thread);
// the staging below uses the block's own layout (c->pin_small_limit >= the limit checked here)
static bool bloom_small_fits(rbx_ctx *c, const rbx_keys *k) {
    const uint64_t limit = g_small_bytes;
    if (!g_small_host || k->n == 0 || k->n > limit / 4) return false;
    const uint64_t nb = k->offsets ? k->offsets[k->n] - k->offsets[0] : k->n * k->stride;
    return nb + (k->offsets ? (k->n + 1) * 8 + 8 : 0) <= limit && small_pinned(c, limit);
}

// an error after small_stage queued the upload: the copy and any launches may still be reading the pinned
// block and slot 0, which the next small call overwrites -- drain the stream first
static int small_fail(rbx_ctx *c, int rc) {
    (void)hipStreamSynchronize(c->stream);
    return rc;
}

// One-transfer staging of a small host arena (bloom_small_fits): pinned [0, head) zeroed, the key bytes
// from `head`, then the offsets (absolute: KeysDev.off_base), uploaded with one copy into staging slot 0
// on the context stream after slot 0's last reader (its event).  The caller records c->ev_done[0] after
// its launches, reads results back into hp / tail_h and syncs; the pinned block stays untouched until then.
struct SmallStage {
    uint8_t *hp = nullptr, *dp = nullptr, *tail_h = nullptr;  // pinned block, its device copy, readback area
    KeysDev dk{};
};
static int small_stage(rbx_ctx *c, const rbx_keys *keys, uint64_t head, SmallStage *s, const void *head_src = nullptr,
                       uint64_t head_src_at = 0, uint64_t head_src_len = 0) {
    const size_t pin = c->pin_small_cap;  // allocated by bloom_small_fits (small_pinned)
    head = (std::max<uint64_t>(head, 8) + 63) / 64 * 64;  // <= kSmallHead (callers bound it)
    uint8_t *hp = (uint8_t *)c->pin_small;
    const uint64_t n = keys->n, b0 = keys->offsets ? keys->offsets[0] : 0;
    const uint64_t nb = keys->offsets ? keys->offsets[n] - b0 : n * keys->stride;
    const uint64_t off_at = keys->offsets ? (head + nb + 7) / 8 * 8 : 0, end = off_at ? off_at + (n + 1) * 8 : head + nb;
    memset(hp, 0, head);
    if (head_src_len) memcpy(hp + head_src_at, head_src, head_src_len);  // e.g. segment offsets behind the counts
    if (nb) memcpy(hp + head, keys->bytes + b0, nb);
    if (off_at) memcpy(hp + off_at, keys->offsets, (n + 1) * 8);
    RBX_TRY(c->slot_bytes[0].reserve(pin));
    uint8_t *dp = c->slot_bytes[0].as<uint8_t>();
    HIP_TRY(hipStreamWaitEvent(c->stream, c->ev_done[0], 0));  // slot 0's last reader (any stream)
    HIP_TRY(hipMemcpyAsync(dp, hp, end, hipMemcpyHostToDevice, c->stream));
    s->hp = hp;
    s->dp = dp;
    s->tail_h = hp + kSmallHead + c->pin_small_limit;
    s->dk = KeysDev{dp + head, off_at ? (const uint64_t *)(dp + off_at) : nullptr, keys->stride, n, off_at ? b0 : 0};
    return RBX_OK;
}

static int bloom_host_small(rbx_ctx *c, const FilterDesc &f, uint32_t k, const rbx_keys *keys, uint8_t *out_flags,
                            uint64_t *out_count, bool is_add) {
    SmallStage s;
    RBX_TRY(small_stage(c, keys, 8, &s));
    const uint64_t n = keys->n;
    uint8_t *d_out = nullptr;
    if (out_flags) {
        RBX_TRY(c->out_bytes.reserve(n));
        d_out = c->out_bytes.as<uint8_t>();
    }
    auto *d_count = (unsigned long long *)s.dp;
    const int rc = is_add ? run_add(c, s.dk, nullptr, nullptr, 0, f, k, d_out, d_count, nullptr, c->stream)
                          : run_contains(c, s.dk, f, d_out, d_count, c->stream);
    (void)hipEventRecord(c->ev_done[0], c->stream);  // slot 0 read by what was queued, whatever rc
    if (rc != RBX_OK) return small_fail(c, rc);
    // the readback lands in the pinned block: its upload precedes it on the stream
    HIP_TRY(hipMemcpyAsync(s.hp, s.dp, 8, hipMemcpyDeviceToHost, c->stream));
    if (out_flags) HIP_TRY(hipMemcpyAsync(s.tail_h, d_out, n, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    if (out_flags) memcpy(out_flags, s.tail_h, n);
    uint64_t cnt;
    memcpy(&cnt, s.hp, 8);
    if (out_count) *out_count = is_add ? (uint64_t)(int64_t)(int32_t)cnt : cnt;  // add(): `int c`
    return RBX_OK;
}

// Tiny host batches -- add(T) / contains(T) and collections of up to host_tiny_keys keys and 64 KiB of key
// bytes: the keys are copied into coherent (uncached, device-mapped) pinned memory, the kernels read them
// from there over the host link and write their flags back into it, so the call is its launches and a wait
// for a completion word in the same block: no upload, no readback, no zeroed count word.  Counts are the flags' sums on the host
// (add(Collection) and contains(Collection) both count the keys whose reply is true,
// M/RedissonBloomFilter.java:104-137,208-236; per segment for the multi-tenant calls).
static std::atomic<uint64_t> g_tiny_keys{16384};  // rbx_tune("host_tiny_keys"): 0 = off
static constexpr uint64_t kTinyBytes = 64 << 10;
// block: flags | segment offsets | key bytes | key offsets (every segment holds a key: nseg <= n)
// (regions 64-byte aligned: 16-byte keys at a 16-byte boundary take the kernels' fixed-length loads, fast_len)
static constexpr uint64_t kTinySegAt = kSegMaxKeys, kTinyKeysAt = kTinySegAt + (kSegMaxKeys + 8) * 8;
static constexpr uint64_t kTinyOffsAt = kTinyKeysAt + kTinyBytes;
// then the small tables a call would upload (PFADD's tile list and sparse-replay items: TinyArena)
static constexpr uint64_t kTinyArenaAt = kTinyOffsAt + (kSegMaxKeys + 8) * 8, kTinyArenaBytes = 64 << 10;
static_assert(kTinyKeysAt % 64 == 0 && kTinyOffsAt % 64 == 0 && kTinyArenaAt % 64 == 0, "aligned regions");
static constexpr uint64_t kTinyDoneAt = kTinyArenaAt + kTinyArenaBytes;  // one-key kernels' completion word
static constexpr size_t kTinyBlock = kTinyDoneAt + 64;

// bump allocation in the block's arena region: the device view of a copy of src, nullptr when full (the
// caller then uploads as usual).  Every copy stays put until the call's final sync.
struct TinyArena {
    uint8_t *h, *d;
    size_t cap, used;
    const void *put(const void *src, size_t n) {
        const size_t at = (used + 63) / 64 * 64;
        if (at + n > cap) return nullptr;
        memcpy(h + at, src, n);
        used = at + n;
        return d + at;
    }
};

static bool bloom_tiny_fits(rbx_ctx *c, const rbx_keys *keys) {
    const uint64_t lim = g_tiny_keys;  // once per call
    if (!g_small_host || keys->n == 0 || keys->n > lim || keys->n > kSegMaxKeys) return false;
    const uint64_t nb = keys->offsets ? keys->offsets[keys->n] - keys->offsets[0] : keys->n * keys->stride;
    if (nb > kTinyBytes) return false;
    if (c->pin_tiny) return true;
    void *h = nullptr, *d = nullptr;
    if (hipHostMalloc(&h, kTinyBlock, hipHostMallocCoherent | hipHostMallocMapped) != hipSuccess) {
        (void)hipGetLastError();
        return false;
    }
    if (hipHostGetDevicePointer(&d, h, 0) != hipSuccess) {
        (void)hipGetLastError();
        (void)hipHostFree(h);
        return false;
    }
    memset(h, 0, kTinyBlock);  // the completion word starts below every sequence number
    c->pin_tiny = (uint8_t *)h;
    c->pin_tiny_dev = (uint8_t *)d;
    c->tiny_seq = 0;
    return true;
}

// the keys into the block (the previous call's kernels were done when it returned: tiny_wait); their device view
static KeysDev tiny_stage(rbx_ctx *c, const rbx_keys *keys) {
    uint8_t *hp = c->pin_tiny, *dp = c->pin_tiny_dev;
    const uint64_t n = keys->n, b0 = keys->offsets ? keys->offsets[0] : 0;
    const uint64_t nb = keys->offsets ? keys->offsets[n] - b0 : n * keys->stride;
    if (nb) memcpy(hp + kTinyKeysAt, keys->bytes + b0, nb);
    if (keys->offsets) memcpy(hp + kTinyOffsAt, keys->offsets, (n + 1) * 8);
    return KeysDev{dp + kTinyKeysAt, keys->offsets ? (const uint64_t *)(dp + kTinyOffsAt) : nullptr, keys->stride, n,
                   keys->offsets ? b0 : 0};
}

// A tiny call learns that its kernels are done from a completion word in the block, not from the stream
// (`host_tiny_spin`, default 1): a one-key call's one-lane kernel stores a sequence number there last
// (system-scope release), other calls launch k_done_word behind their kernels, and the host spins on it --
// 7.2 / 9.6 us against 11.5 us for a one-wave kernel and a stream sync (tools/syncbench.hip).  After 2 ms
// without it (a queue still busy with earlier work, or a fault) the host waits for the stream, which also
// reports any error.
static std::atomic<int> g_tiny_spin{1};

static uint32_t tiny_next_seq(rbx_ctx *c) {
    uint32_t seq = ++c->tiny_seq;
    if (seq == 0) seq = c->tiny_seq = 1;
    return seq;
}

// rc: the launches' result; word_launched: seq is on its way (else the call falls back to the stream)
static int tiny_wait(rbx_ctx *c, int rc, uint32_t seq, bool word_launched) {
    const hipError_t e = hipGetLastError();
    if (rc != RBX_OK || e != hipSuccess || !word_launched) {
        const hipError_t es = hipStreamSynchronize(c->stream);
        RBX_TRY(rc);
        HIP_TRY(e);
        HIP_TRY(es);
        return RBX_OK;
    }
    const auto *h_done = (const uint32_t *)(c->pin_tiny + kTinyDoneAt);
    const auto t0 = std::chrono::steady_clock::now();
    while (__atomic_load_n(h_done, __ATOMIC_ACQUIRE) != seq) {
        if (std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(2)) {
            HIP_TRY(hipStreamSynchronize(c->stream));
            if (__atomic_load_n(h_done, __ATOMIC_ACQUIRE) != seq)
                return fail(RBX_E_DEVICE, "tiny call finished without its completion word");
            break;
        }
    }
    return RBX_OK;
}

// the launches' result -> the completion word behind them (or the stream when spinning is off) -> errors;
// spin: host_tiny_spin as the call read it
static int tiny_done(rbx_ctx *c, int rc, bool spin) {
    spin = spin && rc == RBX_OK;
    const uint32_t seq = spin ? tiny_next_seq(c) : 0;
    if (spin) launch_done_word((uint32_t *)(c->pin_tiny_dev + kTinyDoneAt), seq, c->stream);
    return tiny_wait(c, rc, seq, spin);
}

static int tiny_one(rbx_ctx *c, const FilterDesc &f, const KeysDev &dk, bool is_add) {
    const uint32_t seq = tiny_next_seq(c);
    launch_bloom_one(is_add, dk, fast_len(dk), f, c->pin_tiny_dev, nullptr, (uint32_t *)(c->pin_tiny_dev + kTinyDoneAt),
                     seq, c->stream);
    return tiny_wait(c, RBX_OK, seq, true);
}

static int bloom_host_tiny(rbx_ctx *c, const FilterDesc &f, uint32_t k, const rbx_keys *keys, uint8_t *out_flags,
                           uint64_t *out_count, bool is_add) {
    const KeysDev dk = tiny_stage(c, keys);
    uint8_t *d_flags = c->pin_tiny_dev;
    const bool spin = g_tiny_spin;  // once per call
    if (keys->n == 1 && f.k <= 16 && spin && (!is_add || g_add_one)) {
        RBX_TRY(tiny_one(c, f, dk, is_add));
        const uint8_t v = c->pin_tiny[0];
        if (out_flags) out_flags[0] = v;
        if (out_count) *out_count = v;
        return RBX_OK;
    }
    RBX_TRY(tiny_done(c, is_add ? run_add(c, dk, nullptr, nullptr, 0, f, k, d_flags, nullptr, nullptr, c->stream)
                                  : run_contains(c, dk, f, d_flags, nullptr, c->stream), spin));
    const uint8_t *fl = c->pin_tiny;
    uint64_t cnt = 0;
    for (uint64_t i = 0; i < keys->n; ++i) cnt += fl[i];
    if (out_flags) memcpy(out_flags, fl, keys->n);
    if (out_count) *out_count = is_add ? (uint64_t)(int64_t)(int32_t)cnt : cnt;  // add(): `int c`
    return RBX_OK;
}

static int bloom_host_op(rbx_ctx *c, const std::string &name, int64_t size, uint32_t k, const rbx_keys *keys,
                         uint8_t *out_flags, uint64_t *out_count, bool is_add) {
    RBX_TRY(validate_keys(keys));
    std::lock_guard<std::recursive_mutex> g(c->ks.mu);
    RBX_TRY(set_device(c));
    ScratchOrder so_(c, c->stream);
    // add()/contains() first read the config if the caller has none cached (:106-108)
    if (size == 0) {
        BloomConfig cfg;
        RBX_TRY(ks_get_config(c->ks, name, &cfg));
        size = cfg.size;
        k = cfg.k;
    }
    RBX_TRY(ks_config_check(c->ks, name, size, k));
    if (keys->n == 0) return fail(RBX_E_ARITHMETIC, "/ by zero");
    std::shared_ptr<Bitmap> bm;
    if (size_bits(size) > kEngineMaxSize) {  // indexes may pass the Redis offset limit (bloom_wide_op)
        const bool existed = c->ks.find(name) != nullptr;
        RBX_TRY(bitmap_for(c, name, kEngineMaxSize, is_add, c->stream, &bm));
        const int rc = bloom_wide_op(c, keys, size_bits(size), k, bm.get(), out_flags, out_count, is_add);
        if (bm && !existed) {  // only valid SETBITs create the key: a batch of error replies leaves none
            int r2;
            const uint64_t len = read_dev_u64(c, bm->d_len, &r2);
            if (r2 == RBX_OK && len == 0) c->ks.erase(name);
        }
        return rc;
    }
    RBX_TRY(bitmap_for(c, name, size_bits(size), is_add, c->stream, &bm));
    if (!bm) {  // GETBIT on a missing key: every bit is 0
        if (out_flags) memset(out_flags, 0, keys->n);
        if (out_count) *out_count = 0;
        return RBX_OK;
    }
    FilterDesc f = desc_of(*bm, size_bits(size), k, 0);
    if (bloom_tiny_fits(c, keys)) return bloom_host_tiny(c, f, k, keys, out_flags, out_count, is_add);
    if (bloom_small_fits(c, keys)) return bloom_host_small(c, f, k, keys, out_flags, out_count, is_add);
    RBX_TRY(c->counters.reserve(64));
    auto *d_count = c->counters.as<unsigned long long>();
    HIP_TRY(hipMemsetAsync(d_count, 0, 8, c->stream));
    uint8_t *d_out = nullptr;
    if (out_flags) {
        RBX_TRY(c->out_bytes.reserve(keys->n));
        d_out = c->out_bytes.as<uint8_t>();
    }
    HIP_TRY(hipStreamSynchronize(c->stream));  // slots may still be read by an earlier call's stream
    RBX_TRY(pipelined_host_batches(c, keys, c->stream, [&](const KeysDev &dk, uint64_t i0) -> int {
        uint8_t *o = d_out ? d_out + i0 : nullptr;
        if (is_add) return run_add(c, dk, nullptr, nullptr, 0, f, k, o, d_count, nullptr, c->stream);
        return run_contains(c, dk, f, o, d_count, c->stream);
    }));
    if (out_flags) HIP_TRY(hipMemcpyAsync(out_flags, d_out, keys->n, hipMemcpyDeviceToHost, c->stream));
    int rc;
    uint64_t cnt = read_dev_u64(c, d_count, &rc);
    RBX_TRY(rc);
    if (out_count) *out_count = is_add ? (uint64_t)(int64_t)(int32_t)cnt : cnt;  // add(): `int c`
    return RBX_OK;
}

int rbx_bloom_add(rbx_ctx *c, const char *name, uint64_t size, uint32_t k, const rbx_keys *keys,
                  uint8_t *out_new, uint64_t *out_count) {
    if (!c || !name) return fail(RBX_E_ILLEGAL_ARGUMENT, "ctx/name is NULL");
    return bloom_host_op(c, name, (int64_t)size, k, keys, out_new, out_count, true);
}

int rbx_bloom_contains(rbx_ctx *c, const char *name, uint64_t size, uint32_t k, const rbx_keys *keys,
                       uint8_t *out_present, uint64_t *out_count) {
    if (!c || !name) return fail(RBX_E_ILLEGAL_ARGUMENT, "ctx/name is NULL");
    return bloom_host_op(c, name, (int64_t)size, k, keys, out_present, out_count, false);
}

int rbx_bloom_add_n(rbx_ctx *c, rbx_name name, uint64_t size, uint32_t k, const rbx_keys *keys, uint8_t *out_new,
                    uint64_t *out_count) {
    if (!c || (!name.bytes && name.len)) return fail(RBX_E_ILLEGAL_ARGUMENT, "ctx/name is NULL");
    return bloom_host_op(c, name_of(name), (int64_t)size, k, keys, out_new, out_count, true);
}

int rbx_bloom_contains_n(rbx_ctx *c, rbx_name name, uint64_t size, uint32_t k, const rbx_keys *keys,
                         uint8_t *out_present, uint64_t *out_count) {
    if (!c || (!name.bytes && name.len)) return fail(RBX_E_ILLEGAL_ARGUMENT, "ctx/name is NULL");
    return bloom_host_op(c, name_of(name), (int64_t)size, k, keys, out_present, out_count, false);
}

static int bitcount_locked(rbx_ctx *c, const std::string &name, uint64_t *out) {
    Entry *e = c->ks.find(name);
    if (!e) {
        *out = 0;
        return RBX_OK;
    }
    if (e->type != KType::Bitmap) return fail(RBX_E_WRONGTYPE, kWrongTypeMsg);
    int rc;
    uint64_t len = read_dev_u64(c, e->bm->d_len, &rc);
    RBX_TRY(rc);
    RBX_TRY(c->counters.reserve(64));
    auto *d = c->counters.as<unsigned long long>() + 1;
    HIP_TRY(hipMemsetAsync(d, 0, 8, c->stream));
    if (len) launch_bitcount((const uint8_t *)e->bm->d_words, len, d, c->stream);
    HIP_TRY(hipGetLastError());
    *out = read_dev_u64(c, d, &rc);
    return rc;
}

int rbx_bloom_bitcount(rbx_ctx *c, const char *name, uint64_t *out) {
    if (!c || !name || !out) return fail(RBX_E_ILLEGAL_ARGUMENT, "NULL argument");
    std::lock_guard<std::recursive_mutex> g(c->ks.mu);
    RBX_TRY(set_device(c));
    ScratchOrder so_(c, c->stream);
    return bitcount_locked(c, name, out);
}

// count() :215-227 (the size is the config's Java long, negative sizes included)
static int bloom_count(rbx_ctx *c, const std::string &name, int64_t *out) {
    std::lock_guard<std::recursive_mutex> g(c->ks.mu);
    RBX_TRY(set_device(c));
    ScratchOrder so_(c, c->stream);
    BloomConfig cfg;
    RBX_TRY(ks_get_config(c->ks, name, &cfg));
    uint64_t bits;
    RBX_TRY(bitcount_locked(c, name, &bits));
    const double v = (double)(int64_t)(0 - (uint64_t)cfg.size) / ((double)cfg.k) *
                     std::log(1 - (double)bits / ((double)cfg.size));
    *out = java_math_round(v);
    return RBX_OK;
}

int rbx_bloom_count(rbx_ctx *c, const char *name, int64_t *out) {
    if (!c || !name || !out) return fail(RBX_E_ILLEGAL_ARGUMENT, "NULL argument");
    return bloom_count(c, name, out);
}

int rbx_bloom_count_n(rbx_ctx *c, rbx_name name, int64_t *out) {
    if (!c || (!name.bytes && name.len) || !out) return fail(RBX_E_ILLEGAL_ARGUMENT, "NULL argument");
    return bloom_count(c, name_of(name), out);
}

// delete / isExists / rename / renamenx (keyspace.cpp)
int rbx_bloom_delete(rbx_ctx *c, const char *name, int *deleted) {
    if (!c || !name) return fail(RBX_E_ILLEGAL_ARGUMENT, "NULL argument");
    return ks_bloom_delete(c->ks, name, deleted);
}

int rbx_bloom_is_exists(rbx_ctx *c, const char *name, int *exists) {
    if (!c || !name || !exists) return fail(RBX_E_ILLEGAL_ARGUMENT, "NULL argument");
    return ks_bloom_is_exists(c->ks, name, exists);
}

int rbx_bloom_rename(rbx_ctx *c, const char *name, const char *new_name) {
    if (!c || !name || !new_name) return fail(RBX_E_ILLEGAL_ARGUMENT, "NULL argument");
    return ks_bloom_rename(c->ks, name, new_name);
}

int rbx_bloom_renamenx(rbx_ctx *c, const char *name, const char *new_name, int *renamed) {
    if (!c || !name || !new_name) return fail(RBX_E_ILLEGAL_ARGUMENT, "NULL argument");
    return ks_bloom_renamenx(c->ks, name, new_name, renamed);
}

// DEL / EXISTS over any keys (binary names)
static int names_of(const rbx_name *names, uint32_t n, std::vector<std::string> *out) {
    if (n && !names) return fail(RBX_E_ILLEGAL_ARGUMENT, "NULL names");
    out->clear();
    for (uint32_t i = 0; i < n; ++i) {
        if (!names[i].bytes && names[i].len) return fail(RBX_E_ILLEGAL_ARGUMENT, "NULL key name");
        out->push_back(name_of(names[i]));
    }
    return RBX_OK;
}

int rbx_del_n(rbx_ctx *c, const rbx_name *names, uint32_t n, int *deleted) {
    if (!c) return fail(RBX_E_ILLEGAL_ARGUMENT, "NULL argument");
    std::vector<std::string> v;
    RBX_TRY(names_of(names, n, &v));
    return ks_del(c->ks, v, deleted);
}

int rbx_exists_n(rbx_ctx *c, const rbx_name *names, uint32_t n, int *count) {
    if (!c) return fail(RBX_E_ILLEGAL_ARGUMENT, "NULL argument");
    std::vector<std::string> v;
    RBX_TRY(names_of(names, n, &v));
    return ks_exists(c->ks, v, count);
}

int rbx_bloom_export(rbx_ctx *c, const char *name, uint8_t *out, uint64_t cap, uint64_t *redis_len) {
    if (!c || !name) return fail(RBX_E_ILLEGAL_ARGUMENT, "NULL argument");
    std::lock_guard<std::recursive_mutex> g(c->ks.mu);
    RBX_TRY(set_device(c));
    ScratchOrder so_(c, c->stream);
    Entry *e = c->ks.find(name);
    if (!e) {
        if (redis_len) *redis_len = 0;
        return RBX_OK;
    }
    if (e->type != KType::Bitmap) return fail(RBX_E_WRONGTYPE, kWrongTypeMsg);
    int rc;
    uint64_t len = read_dev_u64(c, e->bm->d_len, &rc);
    RBX_TRY(rc);
    if (redis_len) *redis_len = len;
    uint64_t n = std::min(cap, len);
    if (out && n) {
        HIP_TRY(hipMemcpyAsync(out, e->bm->d_words, n, hipMemcpyDeviceToHost, c->stream));
        HIP_TRY(hipStreamSynchronize(c->stream));
    }
    return RBX_OK;
}

// bits a bitmap imported under `name` must cover: the string, and the config's |size|
static uint64_t import_bits(rbx_ctx *c, const std::string &name, uint64_t len) {
    uint64_t bits = len * 8;
    Entry *cfg = c->ks.find(config_name(name));
    if (cfg && cfg->type == KType::Config) bits = std::max<uint64_t>(bits, size_bits(cfg->cfg->size));
    return std::min<uint64_t>(bits, kEngineMaxSize);
}

int rbx_bloom_import(rbx_ctx *c, const char *name, const uint8_t *bytes, uint64_t len) {
    if (!c || !name || (len && !bytes)) return fail(RBX_E_ILLEGAL_ARGUMENT, "NULL argument");
    if (len > (1ULL << 29)) return fail(RBX_E_ILLEGAL_ARGUMENT, "string exceeds the 512 MiB Redis limit");
    std::lock_guard<std::recursive_mutex> g(c->ks.mu);
    RBX_TRY(set_device(c));
    ScratchOrder so_(c, c->stream);
    std::shared_ptr<Bitmap> b;
    RBX_TRY(new_bitmap(c, import_bits(c, name, len), c->stream, &b));
    if (len) HIP_TRY(hipMemcpyAsync(b->d_words, bytes, len, hipMemcpyHostToDevice, c->stream));
    unsigned long long L = len;
    HIP_TRY(hipMemcpyAsync(b->d_len, &L, 8, hipMemcpyHostToDevice, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    c->ks.put(name, Entry{KType::Bitmap, nullptr, b, nullptr});
    return RBX_OK;
}

// SET name <len bytes from a device buffer> (device-resident snapshot restore)
int rbx_bloom_import_dev(rbx_ctx *c, const char *name, const uint8_t *d_bytes, uint64_t len, void *stream) {
    if (!c || !name || (len && !d_bytes)) return fail(RBX_E_ILLEGAL_ARGUMENT, "NULL argument");
    if (len > (1ULL << 29)) return fail(RBX_E_ILLEGAL_ARGUMENT, "string exceeds the 512 MiB Redis limit");
    std::lock_guard<std::recursive_mutex> g(c->ks.mu);
    RBX_TRY(set_device(c));
    hipStream_t st = pick_stream(c, stream);
    ScratchOrder so_(c, st);
    const uint64_t bits = import_bits(c, name, len);
    std::shared_ptr<Bitmap> b;
    Entry *e = c->ks.find(name);
    if (e && e->type == KType::Bitmap && e->bm->cap_bytes >= ((bits + 7) / 8)) {
        b = e->bm;  // reuse in place (open handles keep seeing it)
        HIP_TRY(hipMemsetAsync(b->d_words, 0, b->cap_bytes, st));
    } else {
        RBX_TRY(new_bitmap(c, bits, st, &b));
    }
    if (len) HIP_TRY(hipMemcpyAsync(b->d_words, d_bytes, len, hipMemcpyDeviceToDevice, st));
    static thread_local unsigned long long L;
    L = len;
    HIP_TRY(hipMemcpyAsync(b->d_len, &L, 8, hipMemcpyHostToDevice, st));
    HIP_TRY(hipStreamSynchronize(st));
    c->ks.put(name, Entry{KType::Bitmap, nullptr, b, nullptr});
    return RBX_OK;
}

// ---- Bloom: handles / device path ---------------------------------------------------------
static int bloom_open(rbx_ctx *c, const std::string &name, rbx_bloom **out) {
    std::lock_guard<std::recursive_mutex> g(c->ks.mu);
    RBX_TRY(set_device(c));
    ScratchOrder so_(c, c->stream);
    BloomConfig cfg;
    RBX_TRY(ks_get_config(c->ks, name, &cfg));
    RBX_TRY(check_offsets(cfg.size));
    // Opening a handle is RedissonBloomFilter's constructor + readConfig: it creates no bitmap
    // key (the first SETBIT does), so EXISTS / DEL / sizeInMemory see what the reference sees.
    std::shared_ptr<Bitmap> bm;
    RBX_TRY(bitmap_for(c, name, size_bits(cfg.size), false, c->stream, &bm));
    HIP_TRY(hipStreamSynchronize(c->stream));
    // gen 0 (never current: generations start at 1) makes the first call bind a missing bitmap
    *out = new rbx_bloom{c, name, cfg.size, cfg.k, bm, bm ? c->ks.generation : 0, g_handle_serial++};
    c->refs.fetch_add(1);
    return RBX_OK;
}

int rbx_bloom_open(rbx_ctx *c, const char *name, rbx_bloom **out) {
    if (!c || !name || !out) return fail(RBX_E_ILLEGAL_ARGUMENT, "NULL argument");
    return bloom_open(c, name, out);
}

int rbx_bloom_open_n(rbx_ctx *c, rbx_name name, rbx_bloom **out) {
    if (!c || (!name.bytes && name.len) || !out) return fail(RBX_E_ILLEGAL_ARGUMENT, "NULL argument");
    return bloom_open(c, name_of(name), out);
}

int rbx_bloom_close(rbx_bloom *b) {
    if (!b) return RBX_OK;
    rbx_ctx *c = b->ctx;
    {
        std::lock_guard<std::recursive_mutex> g(c->ks.mu);
        delete b;
    }
    ctx_release(c);
    return RBX_OK;
}

int rbx_bloom_handle_config(const rbx_bloom *b, uint64_t *size, uint32_t *k) {
    if (!b) return fail(RBX_E_ILLEGAL_ARGUMENT, "NULL handle");
    if (size) *size = (uint64_t)b->size;
    if (k) *k = b->k;
    return RBX_OK;
}

static KeysDev keys_dev(const rbx_keys *k) { return KeysDev{k->bytes, k->offsets, k->stride, k->n}; }

// Re-resolves a Bloom handle's keys if the keyspace changed since its last call: the config
// must still hold the handle's (size, k) (addConfigCheck, M/RedissonBloomFilter.java:207-213) and
// the handle follows whatever bitmap the name holds now; *absent: no bitmap (GETBIT reads 0s).
// A bitmap created here is zero-filled on `st`.
static int bloom_bind(rbx_ctx *c, rbx_bloom *b, bool create, hipStream_t st, bool *absent) {
    c->ks.sweep();
    *absent = false;
    if (b->ctx != c) return fail(RBX_E_ILLEGAL_ARGUMENT, "the handle belongs to another context");
    if (b->gen == c->ks.generation) return RBX_OK;
    RBX_TRY(ks_config_check(c->ks, b->name, b->size, b->k));
    std::shared_ptr<Bitmap> bm;
    RBX_TRY(bitmap_for(c, b->name, size_bits(b->size), create, st, &bm));
    if (!bm) {
        *absent = true;
        b->bm.reset();  // a deleted bitmap's memory is not held by the handle
        return RBX_OK;  // (gen stays stale: the next call binds again)
    }
    b->bm = bm;
    b->gen = c->ks.generation;
    return RBX_OK;
}

int rbx_bloom_contains_dev(rbx_ctx *c, rbx_bloom *b, const rbx_keys *d_keys, uint8_t *d_out,
                           unsigned long long *d_count, void *stream) {
    if (!c || !b) return fail(RBX_E_ILLEGAL_ARGUMENT, "NULL argument");
    RBX_TRY(validate_keys(d_keys));
    if (d_keys->n == 0) return fail(RBX_E_ARITHMETIC, "/ by zero");
    std::lock_guard<std::recursive_mutex> g(c->ks.mu);
    RBX_TRY(set_device(c));
    hipStream_t st = pick_stream(c, stream);
    ScratchOrder so_(c, st);
    bool absent;
    RBX_TRY(bloom_bind(c, b, false, st, &absent));
    if (absent) {  // GETBIT on a missing key: every bit is 0 (the count is unchanged)
        if (d_out) HIP_TRY(hipMemsetAsync(d_out, 0, d_keys->n, st));
        return RBX_OK;
    }
    KeysDev k = keys_dev(d_keys);
    FilterDesc f = desc_of(*b->bm, size_bits(b->size), b->k, 0);
    return run_contains(c, k, f, d_out, d_count, st);
}

int rbx_bloom_add_dev(rbx_ctx *c, rbx_bloom *b, const rbx_keys *d_keys, uint8_t *d_out_new,
                      unsigned long long *d_count, void *stream) {
    if (!c || !b) return fail(RBX_E_ILLEGAL_ARGUMENT, "NULL argument");
    RBX_TRY(validate_keys(d_keys));
    if (d_keys->n == 0) return fail(RBX_E_ARITHMETIC, "/ by zero");
    std::lock_guard<std::recursive_mutex> g(c->ks.mu);
    RBX_TRY(set_device(c));
    hipStream_t st = pick_stream(c, stream);
    ScratchOrder so_(c, st);
    bool absent;
    RBX_TRY(bloom_bind(c, b, true, st, &absent));
    KeysDev k = keys_dev(d_keys);
    FilterDesc f = desc_of(*b->bm, size_bits(b->size), b->k, 0);
    return run_add(c, k, nullptr, nullptr, 0, f, b->k, d_out_new, d_count, nullptr, st);
}

// Uploads the per-segment descriptor table (cached by content + bitmap generation).
// Multi-tenant contains takes the per-lane slot kernel (one gather per key per round trip) when
// the distinct bitmaps of a call exceed this many bytes (past the caches, the request count
// binds); below it the staged kernel (fewer instructions per key) is faster.  rbx_tune
// "contains_multi_slots": 0 never, 1 always, 2 by this threshold (default).
static std::atomic<int> g_multi_slots{2};
constexpr uint64_t kSlotsMinBytes = 64ULL << 20;

// create: a missing bitmap is created (add, stream); otherwise (contains) it reads as all zero
// through c->zero_bm and stays missing.
static int upload_filters(rbx_ctx *c, rbx_bloom *const *filters, uint32_t nseg, uint32_t *kmax, hipStream_t st,
                          bool create, uint64_t *distinct_bytes = nullptr) {
    c->ks.sweep();
    // same handles as the previous call and no keyspace change since: filt_table is current
    // (100k tenants: ~5 ms of host work per call otherwise, more than the kernel takes)
    if (c->filt_key_generation == c->ks.generation && c->filt_keys.size() == nseg && c->filt_create == create) {
        bool same = true;
        for (uint32_t s = 0; s < nseg && same; ++s)
            same = filters[s] && c->filt_keys[s].first == filters[s] && c->filt_keys[s].second == filters[s]->serial;
        if (same) {
            *kmax = c->filt_kmax;
            if (distinct_bytes) *distinct_bytes = c->filt_bytes;
            return RBX_OK;
        }
    }
    std::vector<FilterDesc> v(nseg);
    std::unordered_map<const Bitmap *, uint32_t> fid;
    uint32_t km = 1;
    uint64_t bytes = 0;
    std::vector<uint32_t> absent_segs;
    uint64_t zero_bytes = 0;
    for (uint32_t s = 0; s < nseg; ++s) {
        rbx_bloom *b = filters[s];
        if (!b) return fail(RBX_E_ILLEGAL_ARGUMENT, "NULL filter handle");
        if (b->gen != c->ks.generation) {
            bool absent;
            RBX_TRY(bloom_bind(c, b, create, st, &absent));
        }
        RBX_TRY(check_offsets(b->size));
        km = std::max(km, b->k);
        if (!b->bm) {  // contains on a missing key: every GETBIT reads 0
            absent_segs.push_back(s);
            zero_bytes = std::max<uint64_t>(zero_bytes, (size_bits(b->size) + 7) / 8);
            continue;
        }
        auto it = fid.find(b->bm.get());
        uint32_t id = it == fid.end() ? (uint32_t)fid.size() : it->second;
        if (it == fid.end()) {
            fid[b->bm.get()] = id;
            bytes += (size_bits(b->size) + 7) / 8;
        }
        if (id >= (1u << 24)) return fail(RBX_E_ILLEGAL_ARGUMENT, "more than 2^24 distinct filters in one call");
        v[s] = desc_of(*b->bm, size_bits(b->size), b->k, id);
    }
    if (!absent_segs.empty()) {
        // zero words for the largest missing bitmap + a zero Redis-length word (never written)
        const uint64_t need = ((zero_bytes + 255) & ~255ULL) + 256;
        if (c->zero_bm.cap < need) {
            RBX_TRY(c->zero_bm.reserve(need));
            HIP_TRY(hipMemsetAsync(c->zero_bm.p, 0, c->zero_bm.cap, st));
        }
        const uint32_t zid = (uint32_t)fid.size();
        for (uint32_t s : absent_segs) {
            rbx_bloom *b = filters[s];
            FilterDesc f{};
            f.bm = c->zero_bm.as<uint32_t>();
            f.redis_len = (unsigned long long *)((uint8_t *)c->zero_bm.p + need - 256);
            f.mp = make_mod_params(size_bits(b->size));
            f.k = b->k;
            f.fid = zid;
            v[s] = f;
        }
    }
    *kmax = km;
    bool same = c->filt_generation == c->ks.generation && c->filt_cache.size() == v.size() &&
                memcmp(c->filt_cache.data(), v.data(), v.size() * sizeof(FilterDesc)) == 0;
    if (!same) {
        RBX_TRY(c->filt_table.reserve(v.size() * sizeof(FilterDesc)));
        // pageable source: the runtime has staged it when the call returns
        HIP_TRY(hipMemcpyAsync(c->filt_table.p, v.data(), v.size() * sizeof(FilterDesc), hipMemcpyHostToDevice, st));
        std::vector<ProbeDesc> pd(v.size());
        for (size_t s = 0; s < v.size(); ++s) pd[s] = ProbeDesc{v[s].bm, mod_compact(v[s].mp), v[s].k, v[s].fid};
        RBX_TRY(c->probe_table.reserve(pd.size() * sizeof(ProbeDesc)));
        HIP_TRY(hipMemcpyAsync(c->probe_table.p, pd.data(), pd.size() * sizeof(ProbeDesc), hipMemcpyHostToDevice, st));
        // bitmap words per fid (the stream's table walk finds a bit's bitmap by its fid)
        uint32_t nf = 0;
        uint64_t maxbits = 1;
        for (size_t s = 0; s < v.size(); ++s) {
            nf = std::max(nf, v[s].fid + 1);
            maxbits = std::max<uint64_t>(maxbits, v[s].mp.size);
        }
        std::vector<uint32_t *> fb(std::max<uint32_t>(nf, 1), nullptr);
        for (size_t s = 0; s < v.size(); ++s) fb[v[s].fid] = v[s].bm;
        RBX_TRY(c->fid_table.reserve(fb.size() * sizeof(uint32_t *)));
        HIP_TRY(hipMemcpyAsync(c->fid_table.p, fb.data(), fb.size() * sizeof(uint32_t *), hipMemcpyHostToDevice, st));
        c->filt_nfids = nf;
        c->filt_maxbits = maxbits;
        c->filt_cache.swap(v);
        c->filt_generation = c->ks.generation;
    }
    c->filt_keys.resize(nseg);
    for (uint32_t s = 0; s < nseg; ++s) c->filt_keys[s] = {filters[s], filters[s]->serial};
    c->filt_key_generation = c->ks.generation;
    c->filt_create = create;
    c->filt_kmax = km;
    c->filt_bytes = bytes;
    if (distinct_bytes) *distinct_bytes = bytes;
    return RBX_OK;
}

// d_tile_seg0 (nullable): each 256-key tile's first segment, already in device-visible memory (the tiny host
// path computes it on the host); else k_tile_seg0 finds it
static int contains_multi_run(rbx_ctx *c, rbx_bloom *const *filters, uint32_t nseg, const uint64_t *d_seg_offsets,
                              const rbx_keys *d_keys, uint8_t *d_out, unsigned long long *d_counts, hipStream_t st,
                              const uint32_t *d_tile_seg0) {
    uint32_t kmax;
    uint64_t bytes = 0;
    RBX_TRY(upload_filters(c, filters, nseg, &kmax, st, false, &bytes));
    if (d_keys->n == 0) return RBX_OK;
    KeysDev k = keys_dev(d_keys);
    if (!d_tile_seg0) {
        RBX_TRY(c->tile_segs.reserve(((d_keys->n + 255) / 256) * 4));
        launch_tile_seg0(d_seg_offsets, nseg, d_keys->n, c->tile_segs.as<uint32_t>(), st);
        d_tile_seg0 = c->tile_segs.as<uint32_t>();
    }
    const bool slots = g_multi_slots == 1 || (g_multi_slots == 2 && bytes >= kSlotsMinBytes);
    launch_bloom_contains_multi(k, fast_len(k), c->filt_table.as<FilterDesc>(), d_seg_offsets, nseg, d_tile_seg0, kmax,
                                d_out, d_counts, st, slots);
    HIP_TRY(hipGetLastError());
    return RBX_OK;
}

int rbx_bloom_contains_multi_dev(rbx_ctx *c, rbx_bloom *const *filters, uint32_t nseg,
                                 const uint64_t *d_seg_offsets, const rbx_keys *d_keys, uint8_t *d_out,
                                 unsigned long long *d_counts, void *stream) {
    if (!c || !filters || !d_seg_offsets || nseg == 0) return fail(RBX_E_ILLEGAL_ARGUMENT, "NULL/empty argument");
    RBX_TRY(validate_keys(d_keys));
    std::lock_guard<std::recursive_mutex> g(c->ks.mu);
    RBX_TRY(set_device(c));
    ScratchOrder so_(c, pick_stream(c, stream));
    return contains_multi_run(c, filters, nseg, d_seg_offsets, d_keys, d_out, d_counts, pick_stream(c, stream), nullptr);
}

// rbx_tune("stream_chunk", n) caps a chunk of the ordered stream and of the 8-byte multi-tenant add at
// n commands (tests: many chunks on small batches).
static std::atomic<uint64_t> g_stream_chunk{0};
// rbx_tune("add_multi_table8"): multi-tenant adds whenever (filter id, bit) fits 41 bits and k <= 32:
// 2 (default) optimistic SETBITs with conflict repair (k_maddx_*, r05), 0 the r03 16-byte table path
// (the fallback past 41 bits or k > 32; tests).  (1, the 8-byte first-setter table with the walk
// commit, measured 74.5 vs 53.3 ms at C3 and was removed in r06.)
static std::atomic<int> g_add_multi_t8{2};
// rbx_tune("add_multi_conflict_log2"): entries of the conflict table C, log2 (default 17: 1 MiB, L2-
// resident; tests use small ones to run the overflow path)
static std::atomic<uint32_t> g_maddx_lgc{17};
// rbx_tune("add_multi_segment"): 1 (default) a batch whose filters are all distinct runs its segments of
// <= add_multi_segmax keys one workgroup each (k_madd_seg: LDS first setters, plain word stores, no
// memory-side atomics), longer segments on the chunked path; 0 everything on the chunked path
static std::atomic<int> g_madd_seg{1};
static std::atomic<uint64_t> g_madd_segmax{16384};
// rbx_tune("add_multi_seg_grid"): the per-segment kernel's workgroups, grid-stride over the segments
// (8192: C3 add 28.5 ms; 4096 28.9, 2048 29.9, 1024 31.1, 512 32.7; profiles/r06/r06d_*)
static std::atomic<uint32_t> g_madd_seg_grid{8192};

// Multi-tenant add by optimistic SETBITs with conflict repair (k_maddx_*): chunks of <= min(2^pb - 1,
// 2^27 / k) keys in key order (a chunk's bits are set before the next gathers).  The 8-byte table (an
// overflowed chunk's first setters) and its EMPTY state are shared with the ordered stream (st_t8 /
// st_t8_entries).
static int run_add_multi8(rbx_ctx *c, const KeysDev &keys, const uint64_t *d_seg_off, uint32_t nseg,
                          uint32_t kmax, uint32_t bb, uint32_t pb, uint8_t *d_out_new,
                          unsigned long long *d_seg_counts, hipStream_t st, uint64_t lgc,
                          const uint32_t *big = nullptr, uint64_t segmax = 0) {
    const uint64_t k = std::max<uint32_t>(kmax, 1);
    const uint64_t cap = std::min<uint64_t>((1ULL << std::min<uint32_t>(pb, 40)) - 1, (1ULL << 27) / k);
    uint64_t chunk = std::max<uint64_t>(1, std::min<uint64_t>(keys.n, cap));
    const uint64_t chunk_cap = g_stream_chunk;  // the knob, once per call
    if (chunk_cap) chunk = std::min<uint64_t>(chunk, chunk_cap);
    const uint32_t lgmax = t8_log2((uint32_t)chunk, (uint32_t)k);
    const uint64_t entries = 1ULL << lgmax;
    if (c->st_t8_entries < entries) {
        c->st_t8_entries = 0;
        RBX_TRY(c->st_t8.reserve(entries * 8));
        HIP_TRY(hipMemsetAsync(c->st_t8.p, 0xff, entries * 8, st));
        c->st_t8_entries = entries;
    }
    RBX_TRY(c->zmask.reserve(chunk * 4));
    RBX_TRY(c->madd_c.reserve((8ULL << lgc) + 64));
    struct ResetOnError {  // see rbx_bloom_stream_dev
        rbx_ctx *c;
        bool ok = false;
        ~ResetOnError() {
            if (!ok) c->st_t8_entries = 0;
        }
    } guard{c};
    const int fl = fast_len(keys);
    for (uint64_t base = 0; base < keys.n; base += chunk) {
        MaddChunkArgs a{};
        a.keys = keys;
        a.base = base;
        a.nchunk = std::min<uint64_t>(chunk, keys.n - base);
        a.filt = c->filt_table.as<FilterDesc>();
        a.seg_off = d_seg_off;
        a.nseg = nseg;
        a.tile_seg0 = c->tile_segs.as<uint32_t>();
        a.kmax = kmax;
        a.t8 = c->st_t8.as<unsigned long long>();
        a.lg = t8_log2((uint32_t)a.nchunk, (uint32_t)k);
        a.bb = bb;
        a.pb = pb;
        a.fid_bm = c->fid_table.as<uint32_t *>();
        a.zmask = c->zmask.as<uint32_t>();
        a.out_new = d_out_new;
        a.seg_counts = d_seg_counts;
        a.c8 = c->madd_c.as<unsigned long long>();
        a.lgC = (uint32_t)lgc;
        a.cst = (MaddxState *)(a.c8 + (1ULL << lgc));
        a.big = big;
        a.segmax = segmax;
        launch_madd8_chunk(a, fl, st);
        HIP_TRY(hipGetLastError());
    }
    guard.ok = true;
    return RBX_OK;
}

int rbx_bloom_add_multi_dev(rbx_ctx *c, rbx_bloom *const *filters, uint32_t nseg, const uint64_t *d_seg_offsets,
                            const rbx_keys *d_keys, uint8_t *d_out_new, unsigned long long *d_counts,
                            void *stream) {
    if (!c || !filters || !d_seg_offsets || nseg == 0) return fail(RBX_E_ILLEGAL_ARGUMENT, "NULL/empty argument");
    RBX_TRY(validate_keys(d_keys));
    std::lock_guard<std::recursive_mutex> g(c->ks.mu);
    RBX_TRY(set_device(c));
    ScratchOrder so_(c, pick_stream(c, stream));
    hipStream_t st = pick_stream(c, stream);
    uint32_t kmax;
    RBX_TRY(upload_filters(c, filters, nseg, &kmax, st, true));
    if (d_keys->n == 0) return RBX_OK;
    KeysDev k = keys_dev(d_keys);
    // the chunked and table paths find each tile's first segment in tile_seg0 (the per-segment kernel does not)
    auto tiles = [&]() -> int {
        RBX_TRY(c->tile_segs.reserve(((d_keys->n + 255) / 256) * 4));
        launch_tile_seg0(d_seg_offsets, nseg, d_keys->n, c->tile_segs.as<uint32_t>(), st);
        return RBX_OK;
    };
    uint32_t bb = 1, fbits = 0;
    while ((1ULL << bb) < c->filt_maxbits) ++bb;
    while ((1ULL << fbits) < c->filt_nfids) ++fbits;
    // the knobs, once per call (rbx_tune may run on another thread)
    const int mode = g_add_multi_t8;
    const uint64_t lgc = g_maddx_lgc, segmax = g_madd_segmax;
    if (mode == 2 && g_madd_seg && kmax <= 16 && c->filt_nfids == nseg && bb + fbits <= 41) {
        // every filter in one segment only: k_madd_seg, one workgroup per segment; the chunked path
        // then handles only segments past segmax
        RBX_TRY(c->madd_c.reserve((8ULL << lgc) + 64));
        uint32_t *big = (uint32_t *)(c->madd_c.as<unsigned long long>() + (1ULL << lgc)) + 4;
        // no segment past segmax (known from the host, or the batch is that short): the flag is never
        // raised nor read, so it needs no zeroing launch
        const bool may_big = !(c->madd_maxseg_hint <= segmax || d_keys->n <= segmax);
        if (may_big) HIP_TRY(hipMemsetAsync(big, 0, 4, st));
        MaddSegArgs a{};
        a.keys = k;
        a.filt = c->filt_table.as<FilterDesc>();
        a.seg_off = d_seg_offsets;
        a.nseg = nseg;
        a.kmax = kmax;
        a.grid = g_madd_seg_grid;
        a.segmax = segmax;
        a.out_new = d_out_new;
        a.seg_counts = d_counts;
        a.big = big;
        launch_madd_seg(a, fast_len(k), st);
        HIP_TRY(hipGetLastError());
        if (!may_big) return RBX_OK;  // no long segment
        // device offsets: read the flag (one sync) rather than launch the chunked path's kernels for
        // nothing -- 60 empty launches per C3 call in r05
        HIP_TRY(hipMemcpyAsync(c->pin_word, big, 4, hipMemcpyDeviceToHost, st));  // pinned: no staging copy
        HIP_TRY(hipStreamSynchronize(st));
        uint32_t has_big;
        memcpy(&has_big, c->pin_word, 4);
        if (!has_big) return RBX_OK;
        RBX_TRY(tiles());
        return run_add_multi8(c, k, d_seg_offsets, nseg, kmax, bb, 64 - bb - fbits, d_out_new, d_counts, st, lgc, big,
                              segmax);
    }
    RBX_TRY(tiles());
    if (mode && kmax <= 32 && bb + fbits <= 41)
        return run_add_multi8(c, k, d_seg_offsets, nseg, kmax, bb, 64 - bb - fbits, d_out_new, d_counts, st, lgc);
    FilterDesc dummy{};
    return run_add(c, k, c->filt_table.as<FilterDesc>(), d_seg_offsets, nseg, dummy, kmax, d_out_new, nullptr,
                   d_counts, st);
}

// Ordered mixed stream (C5): see rbx.h.  Chunks of <= 2^26 pairs run probe -> contains -> commit.
// rbx_tune("stream_table8"): 1 (default) the 8-byte first-setter table + walk commit (r04) when
// (fid, bit) fits 41 bits, 0 the r03 16-byte epoch-tagged table (the fallback past 41 bits; tests)
static std::atomic<int> g_stream_table8{1};
int rbx_bloom_stream_dev(rbx_ctx *c, rbx_bloom *const *filters, uint32_t nfilters, const uint32_t *d_key_filter,
                         const uint8_t *d_key_op, const rbx_keys *d_keys, uint8_t *d_out,
                         unsigned long long *d_counts, void *stream) {
    if (!c || !filters || nfilters == 0 || !d_key_filter || !d_key_op)
        return fail(RBX_E_ILLEGAL_ARGUMENT, "NULL/empty argument");
    RBX_TRY(validate_keys(d_keys));
    std::lock_guard<std::recursive_mutex> g(c->ks.mu);
    RBX_TRY(set_device(c));
    ScratchOrder so_(c, pick_stream(c, stream));
    hipStream_t st = pick_stream(c, stream);
    uint32_t kmax;
    RBX_TRY(upload_filters(c, filters, nfilters, &kmax, st, true));
    if (kmax > 32) return fail(RBX_E_ILLEGAL_ARGUMENT, "stream batches support k <= 32");
    if (d_keys->n == 0) return RBX_OK;
    KeysDev keys = keys_dev(d_keys);
    const uint64_t k = std::max<uint32_t>(kmax, 1);
    // r04: 8-byte first-setter entries when (fid, bit) leaves >= 23 bits for a chunk position
    uint32_t bb = 1, fbits = 0;
    while ((1ULL << bb) < c->filt_maxbits) ++bb;
    while ((1ULL << fbits) < c->filt_nfids) ++fbits;
    const bool t8 = g_stream_table8 && bb + fbits <= 41;
    const uint32_t pb = 64 - bb - fbits;
    // Chunks: <= 2^26 (add, bit) pairs for the 16-byte table; with 8-byte entries as many commands
    // as a position field holds, <= 2^27 pairs (a worst-case table of <= 1-2 GiB): C5 8.4M commands
    // per chunk instead of 6.7M.  What that bought (fresh C5, 16.2 vs 17.0 ms) is the table's load:
    // 838K adds size it at 2^24 entries (~27% used) where 671K gave 2^23 (~43%); 6.7M-command chunks
    // on a 2^24 table run as fast (16.34 / 16.41 vs 16.60 / 16.54 ms, r04l_c5_chunk_vs_table_load),
    // larger tables again slower (r04s_c5_table_scale).  Smaller chunks: 3.4M / 1.7M 18.5 / 20.3 ms.
    const uint64_t cap8 = std::min<uint64_t>((1ULL << std::min<uint32_t>(pb, 40)) - 1, (1ULL << 27) / k);
    uint64_t chunk = std::max<uint64_t>(1, std::min<uint64_t>(keys.n, t8 ? cap8 : (1ULL << 26) / k));
    // chunk bases on 128-command boundaries keep the replies' range images line-aligned
    if (chunk < keys.n && chunk > 128) chunk &= ~127ULL;
    if (g_stream_chunk) chunk = std::min<uint64_t>(chunk, g_stream_chunk);
    c->st_geom[0] = bb;
    c->st_geom[1] = fbits;
    c->st_geom[2] = t8 ? pb : 0;
    c->st_geom[3] = chunk;
    RBX_TRY(c->zmask.reserve(chunk * 4));
    RBX_TRY(c->st_adds.reserve(chunk * 4));
    if (t8) RBX_TRY(c->st_fslot.reserve(chunk * 4));
    // one add counter per chunk (zeroed once per call: one fill, not one per chunk)
    const uint64_t nchunks = (keys.n + chunk - 1) / chunk;
    RBX_TRY(c->st_nadds.reserve(nchunks * 4));
    HIP_TRY(hipMemsetAsync(c->st_nadds.p, 0, nchunks * 4, st));
    const int fl = fast_len(keys);
    if (t8) {
        const uint64_t entries = 1ULL << t8_log2((uint32_t)chunk, (uint32_t)k);
        if (c->st_t8_entries < entries) {
            c->st_t8_entries = 0;
            RBX_TRY(c->st_t8.reserve(entries * 8));
            HIP_TRY(hipMemsetAsync(c->st_t8.p, 0xff, entries * 8, st));
            c->st_t8_entries = entries;
        }
    }
    // The 8-byte table is cleared only when it grows: every chunk's walk restores EMPTY.  A launch
    // failing inside the loop breaks that, so the guard then marks it as uninitialized and the next
    // call clears it again.
    struct ResetOnError {
        rbx_ctx *c;
        bool ok = false;
        ~ResetOnError() {
            if (!ok) c->st_t8_entries = 0;
        }
    } guard{c};
    for (uint64_t base = 0; base < keys.n; base += chunk) {
        const uint64_t nch = std::min<uint64_t>(chunk, keys.n - base);
        if (!t8) RBX_TRY(ensure_table(c, nch * k, st));
        StreamChunkArgs s{};
        if (t8) {
            s.t8 = c->st_t8.as<unsigned long long>();
            s.bb = bb;
            s.pb = pb;
            s.fid_bm = c->fid_table.as<uint32_t *>();
            s.tkmax = kmax;
            s.fslot = c->st_fslot.as<uint32_t>();
        }
        s.adds = c->st_adds.as<uint32_t>();
        s.nadds = c->st_nadds.as<uint32_t>() + base / chunk;
        s.keys = keys;
        s.base = base;
        s.nchunk = nch;
        s.filt = c->filt_table.as<FilterDesc>();
        s.pdesc = c->probe_table.as<ProbeDesc>();
        s.kf = d_key_filter;
        s.op = d_key_op;
        s.table = c->table.as<HTEntry>();
        s.log2cap = c->log2cap;
        s.epoch = c->epoch;
        s.zmask = c->zmask.as<uint32_t>();
        s.kmax = kmax;
        s.out = d_out;
        s.counts = d_counts;
        launch_stream_chunk(s, fl, st);
        HIP_TRY(hipGetLastError());
    }
    guard.ok = true;
    return RBX_OK;
}

int rbx_bloom_stream(rbx_ctx *c, rbx_bloom *const *filters, uint32_t nfilters, const uint32_t *key_filter,
                     const uint8_t *key_op, const rbx_keys *keys, uint8_t *out, uint64_t *counts) {
    if (!c || !filters || nfilters == 0 || !key_filter || !key_op) return fail(RBX_E_ILLEGAL_ARGUMENT, "NULL argument");
    RBX_TRY(validate_keys(keys));
    for (uint64_t i = 0; i < keys->n; ++i)
        if (key_filter[i] >= nfilters) return fail(RBX_E_ILLEGAL_ARGUMENT, "key_filter index out of range");
    std::lock_guard<std::recursive_mutex> g(c->ks.mu);
    RBX_TRY(set_device(c));
    ScratchOrder so_(c, c->stream);
    KeysDev dk;
    RBX_TRY(upload_keys(c, keys, 0, keys->n, &dk));
    const uint64_t n = keys->n;
    RBX_TRY(c->seg_offs.reserve(n * 4 + n + 64));
    auto *d_kf = c->seg_offs.as<uint32_t>();
    auto *d_op = (uint8_t *)(d_kf + n);
    if (n) {
        HIP_TRY(hipMemcpyAsync(d_kf, key_filter, n * 4, hipMemcpyHostToDevice, c->stream));
        HIP_TRY(hipMemcpyAsync(d_op, key_op, n, hipMemcpyHostToDevice, c->stream));
    }
    RBX_TRY(c->counters.reserve(64));
    auto *d_cnt = c->counters.as<unsigned long long>() + 2;
    HIP_TRY(hipMemsetAsync(d_cnt, 0, 16, c->stream));
    uint8_t *d_out = nullptr;
    if (out) {
        RBX_TRY(c->out_bytes.reserve(n));
        d_out = c->out_bytes.as<uint8_t>();
    }
    // the *_dev ABI has no off_base: shift the base so that bytes + offsets[i] is key i (never read below)
    rbx_keys kd{dk.bytes - dk.off_base, dk.offsets, dk.stride, dk.n};
    RBX_TRY(rbx_bloom_stream_dev(c, filters, nfilters, d_kf, d_op, &kd, d_out, d_cnt, c->stream));
    if (out && n) HIP_TRY(hipMemcpyAsync(out, d_out, n, hipMemcpyDeviceToHost, c->stream));
    unsigned long long cnt[2];
    HIP_TRY(hipMemcpyAsync(cnt, d_cnt, 16, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    if (counts) {
        counts[0] = cnt[0];
        counts[1] = cnt[1];
    }
    return RBX_OK;
}

static int multi_host(rbx_ctx *c, rbx_bloom *const *filters, uint32_t nseg, const uint64_t *seg_offsets,
                      const rbx_keys *keys, uint8_t *out_flags, uint64_t *out_counts, bool is_add) {
    if (!c || !filters || !seg_offsets || nseg == 0) return fail(RBX_E_ILLEGAL_ARGUMENT, "NULL/empty argument");
    RBX_TRY(validate_keys(keys));
    if (seg_offsets[0] != 0 || seg_offsets[nseg] != keys->n)
        return fail(RBX_E_ILLEGAL_ARGUMENT, "segment offsets must span [0, n]");
    for (uint32_t s = 0; s < nseg; ++s) {
        if (seg_offsets[s + 1] < seg_offsets[s]) return fail(RBX_E_ILLEGAL_ARGUMENT, "segment offsets must be ascending");
        if (seg_offsets[s + 1] == seg_offsets[s]) return fail(RBX_E_ARITHMETIC, "/ by zero");
    }
    std::lock_guard<std::recursive_mutex> g(c->ks.mu);
    RBX_TRY(set_device(c));
    ScratchOrder so_(c, c->stream);
    uint64_t mx = 0;  // the largest segment: the per-segment add then skips the chunked path's launches
    for (uint32_t q = 0; q < nseg; ++q) mx = std::max<uint64_t>(mx, seg_offsets[q + 1] - seg_offsets[q]);
    if (bloom_tiny_fits(c, keys)) {
        // keys, segment offsets and flags in coherent pinned memory (bloom_host_tiny); the per-segment counts
        // are the flags' sums (every segment holds a key, so nseg <= n fits the block)
        const KeysDev dk = tiny_stage(c, keys);
        memcpy(c->pin_tiny + kTinySegAt, seg_offsets, (uint64_t)(nseg + 1) * 8);
        const auto *d_seg = (const uint64_t *)(c->pin_tiny_dev + kTinySegAt);
        uint8_t *d_flags = c->pin_tiny_dev;
        rbx_keys kd{dk.bytes - dk.off_base, dk.offsets, dk.stride, dk.n};  // the *_dev ABI has no off_base
        int rc;
        if (is_add) {
            c->madd_maxseg_hint = mx;
            rc = rbx_bloom_add_multi_dev(c, filters, nseg, d_seg, &kd, d_flags, nullptr, c->stream);
            c->madd_maxseg_hint = ~0ULL;
        } else {
            // each 256-key tile's first segment from the host (no k_tile_seg0 launch)
            std::vector<uint32_t> ts((keys->n + 255) / 256);
            for (uint32_t q = 0, t = 0; t < ts.size(); ++t) {
                while (seg_offsets[q + 1] <= (uint64_t)t * 256) ++q;
                ts[t] = q;
            }
            TinyArena ta{c->pin_tiny + kTinyArenaAt, c->pin_tiny_dev + kTinyArenaAt, kTinyArenaBytes, 0};
            rc = contains_multi_run(c, filters, nseg, d_seg, &kd, d_flags, nullptr, c->stream,
                                    (const uint32_t *)ta.put(ts.data(), ts.size() * 4));
        }
        RBX_TRY(tiny_done(c, rc, g_tiny_spin));
        const uint8_t *fl = c->pin_tiny;
        if (out_counts)
            for (uint32_t q = 0; q < nseg; ++q) {
                uint64_t t = 0;
                for (uint64_t i = seg_offsets[q]; i < seg_offsets[q + 1]; ++i) t += fl[i];
                out_counts[q] = t;
            }
        if (out_flags) memcpy(out_flags, fl, keys->n);
        return RBX_OK;
    }
    if ((uint64_t)nseg * 16 + 8 <= kSmallHead && bloom_small_fits(c, keys)) {
        // one transfer: the zeroed per-segment counts, the segment offsets, the keys (bloom_host_small)
        SmallStage sm;
        const uint64_t so_at = (uint64_t)nseg * 8;
        RBX_TRY(small_stage(c, keys, so_at + (uint64_t)(nseg + 1) * 8, &sm, seg_offsets, so_at, (uint64_t)(nseg + 1) * 8));
        auto *d_counts = (unsigned long long *)sm.dp;
        const auto *d_seg = (const uint64_t *)(sm.dp + so_at);
        uint8_t *d_out = nullptr;
        if (out_flags) {
            RBX_TRY(c->out_bytes.reserve(keys->n));
            d_out = c->out_bytes.as<uint8_t>();
        }
        // the *_dev ABI has no off_base: shift the base so that bytes + offsets[i] is key i
        rbx_keys kd{sm.dk.bytes - sm.dk.off_base, sm.dk.offsets, sm.dk.stride, sm.dk.n};
        int rc;
        if (is_add) {
            c->madd_maxseg_hint = mx;
            rc = rbx_bloom_add_multi_dev(c, filters, nseg, d_seg, &kd, d_out, d_counts, c->stream);
            c->madd_maxseg_hint = ~0ULL;
        } else {
            rc = rbx_bloom_contains_multi_dev(c, filters, nseg, d_seg, &kd, d_out, d_counts, c->stream);
        }
        (void)hipEventRecord(c->ev_done[0], c->stream);
        if (rc != RBX_OK) return small_fail(c, rc);
        HIP_TRY(hipMemcpyAsync(sm.hp, sm.dp, (size_t)nseg * 8, hipMemcpyDeviceToHost, c->stream));
        if (out_flags) HIP_TRY(hipMemcpyAsync(sm.tail_h, d_out, keys->n, hipMemcpyDeviceToHost, c->stream));
        HIP_TRY(hipStreamSynchronize(c->stream));
        if (out_flags) memcpy(out_flags, sm.tail_h, keys->n);
        if (out_counts) memcpy(out_counts, sm.hp, (size_t)nseg * 8);
        return RBX_OK;
    }
    KeysDev dk;
    RBX_TRY(upload_keys(c, keys, 0, keys->n, &dk));
    RBX_TRY(c->seg_offs.reserve((nseg + 1) * 8));
    HIP_TRY(hipMemcpyAsync(c->seg_offs.p, seg_offsets, (nseg + 1) * 8, hipMemcpyHostToDevice, c->stream));
    RBX_TRY(c->misc.reserve(nseg * 8));
    auto *d_counts = c->misc.as<unsigned long long>();
    HIP_TRY(hipMemsetAsync(d_counts, 0, nseg * 8, c->stream));
    uint8_t *d_out = nullptr;
    if (out_flags) {
        RBX_TRY(c->out_bytes.reserve(keys->n));
        d_out = c->out_bytes.as<uint8_t>();
    }
    // the *_dev ABI has no off_base: shift the base so that bytes + offsets[i] is key i (never read below)
    rbx_keys kd{dk.bytes - dk.off_base, dk.offsets, dk.stride, dk.n};
    if (is_add) {
        c->madd_maxseg_hint = mx;
        const int rc = rbx_bloom_add_multi_dev(c, filters, nseg, c->seg_offs.as<uint64_t>(), &kd, d_out, d_counts,
                                               c->stream);
        c->madd_maxseg_hint = ~0ULL;
        RBX_TRY(rc);
    }
    else RBX_TRY(rbx_bloom_contains_multi_dev(c, filters, nseg, c->seg_offs.as<uint64_t>(), &kd, d_out, d_counts, c->stream));
    if (out_flags) HIP_TRY(hipMemcpyAsync(out_flags, d_out, keys->n, hipMemcpyDeviceToHost, c->stream));
    std::vector<unsigned long long> cnt(nseg);
    HIP_TRY(hipMemcpyAsync(cnt.data(), d_counts, nseg * 8, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    if (out_counts)
        for (uint32_t s = 0; s < nseg; ++s) out_counts[s] = cnt[s];
    return RBX_OK;
}

int rbx_bloom_contains_multi(rbx_ctx *c, rbx_bloom *const *filters, uint32_t nseg, const uint64_t *seg_offsets,
                             const rbx_keys *keys, uint8_t *out_present, uint64_t *out_counts) {
    return multi_host(c, filters, nseg, seg_offsets, keys, out_present, out_counts, false);
}

int rbx_bloom_add_multi(rbx_ctx *c, rbx_bloom *const *filters, uint32_t nseg, const uint64_t *seg_offsets,
                        const rbx_keys *keys, uint8_t *out_new, uint64_t *out_counts) {
    return multi_host(c, filters, nseg, seg_offsets, keys, out_new, out_counts, true);
}

// ---- HyperLogLog ------------------------------------------------------------------------------
static constexpr uint64_t kTileElems = 65536;  // elements per PFADD workgroup
constexpr uint64_t kHllSparseMaxBytes = 3000;  // redis.conf hll-sparse-max-bytes (default)

static const char *kHllWrongType = "WRONGTYPE Key is not a valid HyperLogLog string value.";

// The HLL under `name`; with create, PFADD's createHLLObject (registers zero-filled on `st`).
static int hll_get(rbx_ctx *c, const std::string &name, bool create, hipStream_t st, std::shared_ptr<HllState> *out,
                   bool *created) {
    if (created) *created = false;
    Entry *e = c->ks.find(name);
    if (e) {
        if (e->type != KType::Hll) return fail(RBX_E_WRONGTYPE, kHllWrongType);
        *out = e->hll;
        return RBX_OK;
    }
    if (!create) {
        out->reset();
        return RBX_OK;
    }
    std::shared_ptr<HllState> h;
    RBX_TRY(hll_alloc(c, st, &h));
    h->card = 0;  // createHLLObject: cached cardinality 0, valid
    c->ks.put(name, Entry{KType::Hll, nullptr, nullptr, h});
    c->ks.generation++;
    *out = h;
    if (created) *created = true;
    return RBX_OK;
}

// HLL handles follow the name too; PFADD on a missing key creates it (createHLLObject), PFCOUNT
// reads it as empty (h->st = null) without creating it
static int hll_bind(rbx_ctx *c, rbx_hll *h, bool create, hipStream_t st) {
    c->ks.sweep();
    if (h->ctx != c) return fail(RBX_E_ILLEGAL_ARGUMENT, "the handle belongs to another context");
    if (h->gen == c->ks.generation && h->st) return RBX_OK;
    std::shared_ptr<HllState> s;
    RBX_TRY(hll_get(c, h->name, create, st, &s, nullptr));
    h->st = s;
    if (s) h->gen = c->ks.generation;
    return RBX_OK;
}

// Redis keeps a PFADD-created HLL sparse until an update would store a value > 32 or grow the
// string past hll-sparse-max-bytes, then promotes it to dense for good ([redis-7.2]
// hyperloglog.c hllSparseSet), and the sparse bytes depend on the order of the updates.
// k_hll_sparse_replay applies each command's updates, in order, to the sparse HLLs' strings on
// the device (the registers are updated by the PFADD / merge kernels as for dense keys) and sets
// the sticky promotion word at the first promotion.  `items` = one per sparse HLL of a round.
static int replay_sparse(rbx_ctx *c, std::vector<HllReplay> &items, const KeysDev &dk, int fl, hipStream_t st,
                         TinyArena *ta = nullptr) {
    if (items.empty()) return RBX_OK;
    if (const void *d = ta ? ta->put(items.data(), items.size() * sizeof(HllReplay)) : nullptr) {  // tiny call
        launch_hll_sparse_replay(dk, fl, (const HllReplay *)d, (uint32_t)items.size(), kHllSparseMaxBytes, st);
        HIP_TRY(hipGetLastError());
        return RBX_OK;
    }
    const bool same = c->check_cache.size() == items.size() &&
                      memcmp(c->check_cache.data(), items.data(), items.size() * sizeof(HllReplay)) == 0;
    if (!same) {
        RBX_TRY(c->hll_checks.reserve(items.size() * sizeof(HllReplay)));
        HIP_TRY(hipMemcpyAsync(c->hll_checks.p, items.data(), items.size() * sizeof(HllReplay), hipMemcpyHostToDevice, st));
        c->check_cache = items;
    }
    launch_hll_sparse_replay(dk, fl, c->hll_checks.as<HllReplay>(), (uint32_t)items.size(), kHllSparseMaxBytes, st);
    HIP_TRY(hipGetLastError());
    return RBX_OK;
}

// PFMERGE-style write-back (ascending registers) of the sparse HLLs among hl; their registers
// already hold the merged maxima
static int replay_merge(rbx_ctx *c, const std::vector<HllState *> &hl, hipStream_t st) {
    std::vector<HllReplay> items;
    std::unordered_map<HllState *, int> seen;
    for (HllState *h : hl)
        if (h && !h->dense && !seen.count(h)) {
            seen[h] = 1;
            items.push_back(HllReplay{h->d_sp_ops, h->d_promoted, h->d_regs, 0, 0, h->d_regs});
        }
    return replay_sparse(c, items, KeysDev{}, 0, st);
}

// host view of the promotion word (the caller holds a ScratchOrder on c->stream)
static int resolve_dense(rbx_ctx *c, HllState *h) {
    if (h->dense) return RBX_OK;
    uint32_t w = 0;
    HIP_TRY(hipMemcpyAsync(&w, h->d_promoted, 4, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    if (w) h->dense = true;
    return RBX_OK;
}

// PFADD batch: device elements, commands in order.  Commands naming the same HLL are
// split into successive launches so each reply sees the previous commands' effect.
static int pfadd_run(rbx_ctx *c, const std::vector<HllState *> &hl, const uint64_t *h_seg, const KeysDev &dk,
                     uint32_t *d_changed, hipStream_t st, TinyArena *ta = nullptr) {
    const uint32_t nseg = (uint32_t)hl.size();
    std::vector<HllSeg> tiles;
    uint32_t s0 = 0;
    const int fl = fast_len_hll(dk);
    while (s0 < nseg) {
        // a round: maximal run of commands with distinct HLLs
        std::unordered_map<HllState *, int> seen;
        uint32_t s1 = s0;
        while (s1 < nseg && !seen.count(hl[s1])) seen[hl[s1++]] = 1;
        tiles.clear();
        for (uint32_t s = s0; s < s1; ++s) {
            for (uint64_t b = h_seg[s]; b < h_seg[s + 1]; b += kTileElems)
                tiles.push_back(HllSeg{hl[s]->d_regs, b, std::min(h_seg[s + 1], b + kTileElems), s, 0});
        }
        if (!tiles.empty()) {
            // a tiny call's tile list is read from the coherent block (each round its own copy)
            const HllSeg *d_tiles = ta ? (const HllSeg *)ta->put(tiles.data(), tiles.size() * sizeof(HllSeg)) : nullptr;
            if (!d_tiles) {
                // the tile table is cached by content (a steady PFADD pipeline re-sends the same one)
                const bool single_round = s0 == 0 && s1 == nseg;
                const bool same = single_round && c->tiles_valid && c->tile_cache.size() == tiles.size() &&
                                  memcmp(c->tile_cache.data(), tiles.data(), tiles.size() * sizeof(HllSeg)) == 0;
                if (!same) {
                    RBX_TRY(c->hll_tiles.reserve(tiles.size() * sizeof(HllSeg)));
                    // pageable source: staged by the runtime before the call returns; stream order
                    // keeps the previous round's kernel ahead of this overwrite
                    HIP_TRY(hipMemcpyAsync(c->hll_tiles.p, tiles.data(), tiles.size() * sizeof(HllSeg), hipMemcpyHostToDevice, st));
                    c->tiles_valid = single_round;
                    if (single_round) c->tile_cache = tiles;
                }
                d_tiles = c->hll_tiles.as<HllSeg>();
            }
            launch_hll_pfadd(dk, fl, d_tiles, (uint32_t)tiles.size(), d_changed, st);
            HIP_TRY(hipGetLastError());
            std::vector<HllReplay> items;  // the round's HLLs are distinct
            for (uint32_t s = s0; s < s1; ++s)
                if (!hl[s]->dense && h_seg[s + 1] > h_seg[s])
                    items.push_back(HllReplay{hl[s]->d_sp_ops, hl[s]->d_promoted, nullptr, h_seg[s], h_seg[s + 1],
                                              hl[s]->d_regs});
            RBX_TRY(replay_sparse(c, items, dk, fl, st, ta));
        }
        s0 = s1;
    }
    return RBX_OK;
}

static int hll_add_multi(rbx_ctx *c, const std::vector<std::string> &names, const uint64_t *seg_offsets,
                         const rbx_keys *elements, uint8_t *out_changed) {
    const uint32_t nseg = (uint32_t)names.size();
    RBX_TRY(validate_keys(elements));
    if (nseg == 0) return RBX_OK;
    if (seg_offsets[0] != 0 || seg_offsets[nseg] != elements->n)
        return fail(RBX_E_ILLEGAL_ARGUMENT, "segment offsets must span [0, n]");
    for (uint32_t s = 0; s < nseg; ++s)
        if (seg_offsets[s + 1] < seg_offsets[s]) return fail(RBX_E_ILLEGAL_ARGUMENT, "segment offsets must be ascending");
    std::lock_guard<std::recursive_mutex> g(c->ks.mu);
    RBX_TRY(set_device(c));
    ScratchOrder so_(c, c->stream);
    std::vector<HllState *> hl(nseg);
    std::vector<std::shared_ptr<HllState>> keep(nseg);
    std::vector<uint8_t> created(nseg, 0);
    for (uint32_t s = 0; s < nseg; ++s) {
        bool cr;
        RBX_TRY(hll_get(c, names[s], true, c->stream, &keep[s], &cr));
        hl[s] = keep[s].get();
        created[s] = cr;
    }
    std::vector<uint32_t> ch(nseg);
    if (nseg <= kSegMaxKeys && bloom_tiny_fits(c, elements)) {
        // elements, changed words, tile list and replay items in coherent pinned memory (bloom_host_tiny)
        auto *ch_h = (uint32_t *)(c->pin_tiny + kTinySegAt);
        memset(ch_h, 0, (size_t)nseg * 4);
        const KeysDev dk = tiny_stage(c, elements);
        TinyArena ta{c->pin_tiny + kTinyArenaAt, c->pin_tiny_dev + kTinyArenaAt, kTinyArenaBytes, 0};
        RBX_TRY(tiny_done(c, pfadd_run(c, hl, seg_offsets, dk, (uint32_t *)(c->pin_tiny_dev + kTinySegAt), c->stream,
                                       &ta),
                          g_tiny_spin));
        memcpy(ch.data(), ch_h, (size_t)nseg * 4);
        for (uint32_t s = 0; s < nseg; ++s) {
            if (ch[s]) hl[s]->card |= 1ULL << 63;  // HLL_INVALIDATE_CACHE
            if (out_changed) out_changed[s] = ch[s] || created[s];
        }
        return RBX_OK;
    }
    if (nseg <= kSmallHead / 4 && bloom_small_fits(c, elements)) {
        // one transfer for the elements and the zeroed changed words, one readback (bloom_host_small)
        SmallStage sm;
        RBX_TRY(small_stage(c, elements, nseg * 4, &sm));
        const int rc = pfadd_run(c, hl, seg_offsets, sm.dk, (uint32_t *)sm.dp, c->stream);
        (void)hipEventRecord(c->ev_done[0], c->stream);
        if (rc != RBX_OK) return small_fail(c, rc);
        HIP_TRY(hipMemcpyAsync(sm.hp, sm.dp, nseg * 4, hipMemcpyDeviceToHost, c->stream));
        HIP_TRY(hipStreamSynchronize(c->stream));
        memcpy(ch.data(), sm.hp, nseg * 4);
        for (uint32_t s = 0; s < nseg; ++s) {
            if (ch[s]) hl[s]->card |= 1ULL << 63;  // HLL_INVALIDATE_CACHE
            if (out_changed) out_changed[s] = ch[s] || created[s];
        }
        return RBX_OK;
    }
    RBX_TRY(c->misc.reserve(nseg * 4));
    auto *d_changed = c->misc.as<uint32_t>();
    HIP_TRY(hipMemsetAsync(d_changed, 0, nseg * 4, c->stream));
    auto span_bytes = [&](uint64_t e0, uint64_t e1) {
        return elements->offsets ? elements->offsets[e1] - elements->offsets[e0] : (e1 - e0) * elements->stride;
    };
    const uint64_t budget = 256ull << 20;
    for (uint32_t s0 = 0; s0 < nseg;) {
        // commands [s0, s1) whose elements fit one staging upload (at least one command)
        uint32_t s1 = s0 + 1;
        while (s1 < nseg && span_bytes(seg_offsets[s0], seg_offsets[s1 + 1]) <= budget) ++s1;
        const uint64_t e0 = seg_offsets[s0], e1 = seg_offsets[s1];
        KeysDev dk{};
        if (e1 > e0) RBX_TRY(upload_keys(c, elements, e0, e1, &dk));
        std::vector<uint64_t> reb(s1 - s0 + 1);
        for (uint32_t s = s0; s <= s1; ++s) reb[s - s0] = seg_offsets[s] - e0;
        std::vector<HllState *> grp(hl.begin() + s0, hl.begin() + s1);
        RBX_TRY(pfadd_run(c, grp, reb.data(), dk, d_changed + s0, c->stream));
        s0 = s1;
    }
    HIP_TRY(hipMemcpyAsync(ch.data(), d_changed, nseg * 4, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    for (uint32_t s = 0; s < nseg; ++s) {
        if (ch[s]) hl[s]->card |= 1ULL << 63;  // HLL_INVALIDATE_CACHE
        if (out_changed) out_changed[s] = ch[s] || created[s];
    }
    return RBX_OK;
}

static int cstr_names(const char *const *names, uint32_t n, std::vector<std::string> *out) {
    if (n && !names) return fail(RBX_E_ILLEGAL_ARGUMENT, "NULL names");
    out->clear();
    for (uint32_t i = 0; i < n; ++i) {
        if (!names[i]) return fail(RBX_E_ILLEGAL_ARGUMENT, "NULL key name");
        out->emplace_back(names[i]);
    }
    return RBX_OK;
}

int rbx_hll_add_multi(rbx_ctx *c, const char *const *names, uint32_t nseg, const uint64_t *seg_offsets,
                      const rbx_keys *elements, uint8_t *out_changed) {
    if (!c || !names || !seg_offsets) return fail(RBX_E_ILLEGAL_ARGUMENT, "NULL argument");
    std::vector<std::string> v;
    RBX_TRY(cstr_names(names, nseg, &v));
    return hll_add_multi(c, v, seg_offsets, elements, out_changed);
}

int rbx_hll_add_multi_n(rbx_ctx *c, const rbx_name *names, uint32_t nseg, const uint64_t *seg_offsets,
                        const rbx_keys *elements, uint8_t *out_changed) {
    if (!c || !names || !seg_offsets) return fail(RBX_E_ILLEGAL_ARGUMENT, "NULL argument");
    std::vector<std::string> v;
    RBX_TRY(names_of(names, nseg, &v));
    return hll_add_multi(c, v, seg_offsets, elements, out_changed);
}

int rbx_hll_add(rbx_ctx *c, const char *name, const rbx_keys *elements, int *changed) {
    if (!c || !name || !elements) return fail(RBX_E_ILLEGAL_ARGUMENT, "NULL argument");
    uint64_t seg[2] = {0, elements->n};
    uint8_t ch = 0;
    RBX_TRY(hll_add_multi(c, {std::string(name)}, seg, elements, &ch));
    if (changed) *changed = ch;
    return RBX_OK;
}

// glibc-side hllTau fallback and the full estimator from a histogram (redis hllCount)
static double hll_tau_host(double x) {
    if (x == 0. || x == 1.) return 0.;
    double zPrime;
    double y = 1.0;
    double z = 1 - x;
    do {
        x = std::sqrt(x);
        zPrime = z;
        y *= 0.5;
        z -= std::pow(1 - x, 2) * y;
    } while (zPrime != z);
    return z / 3;
}

static double hll_sigma_host(double x) {
    if (x == 1.) return INFINITY;
    double zPrime;
    double y = 1;
    double z = x;
    do {
        x *= x;
        zPrime = z;
        z += x * y;
        y += y;
    } while (zPrime != z);
    return z;
}

static uint64_t hll_count_from_histo(const int *reghisto) {
    double m = 16384;
    double z = m * hll_tau_host((m - reghisto[51]) / (double)m);
    for (int j = 50; j >= 1; --j) {
        z += reghisto[j];
        z *= 0.5;
    }
    z += m * hll_sigma_host(reghisto[0] / (double)m);
    double E = (double)llroundl(0.721347520444481703680 * m * m / z);
    return (uint64_t)E;
}

// Computes counts for raw register arrays (device pointers) -> host out.
static int count_regs(rbx_ctx *c, const std::vector<uint8_t *> &regs, uint64_t *out) {
    uint32_t n = (uint32_t)regs.size();
    if (!n) return RBX_OK;
    RBX_TRY(c->ptrs.reserve(n * sizeof(uint8_t *)));
    RBX_TRY(c->histo.reserve((size_t)n * 64 * sizeof(int)));
    RBX_TRY(c->misc.reserve(n * 8));
    HIP_TRY(hipMemcpyAsync(c->ptrs.p, regs.data(), n * sizeof(uint8_t *), hipMemcpyHostToDevice, c->stream));
    launch_hll_count(c->ptrs.as<uint8_t *>(), n, c->histo.as<int>(), c->misc.as<unsigned long long>(), c->stream);
    HIP_TRY(hipGetLastError());
    std::vector<unsigned long long> res(n);
    HIP_TRY(hipMemcpyAsync(res.data(), c->misc.p, n * 8, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    std::vector<int> h;
    for (uint32_t i = 0; i < n; ++i) {
        if (res[i] == ~0ULL) {  // tau branch: histogram to host, glibc pow
            if (h.empty()) {
                h.resize((size_t)n * 64);
                HIP_TRY(hipMemcpy(h.data(), c->histo.p, h.size() * sizeof(int), hipMemcpyDeviceToHost));
            }
            res[i] = hll_count_from_histo(&h[(size_t)i * 64]);
        }
        out[i] = res[i];
    }
    return RBX_OK;
}

// single-key PFCOUNT with the header cache (valid cache -> cached value; else compute+store)
static int pfcount_each(rbx_ctx *c, const std::vector<HllState *> &hl, uint64_t *out) {
    std::vector<uint8_t *> regs;
    std::vector<uint32_t> idx;
    for (uint32_t i = 0; i < hl.size(); ++i) {
        if (!hl[i]) {
            out[i] = 0;
            continue;
        }
        if (!(hl[i]->card >> 63)) {
            out[i] = hl[i]->card;
            continue;
        }
        regs.push_back(hl[i]->d_regs);
        idx.push_back(i);
    }
    std::vector<uint64_t> r(regs.size());
    RBX_TRY(count_regs(c, regs, r.data()));
    for (size_t j = 0; j < idx.size(); ++j) {
        out[idx[j]] = r[j];
        hl[idx[j]]->card = r[j];  // store the (valid) cached cardinality
    }
    return RBX_OK;
}

static int hll_count_each(rbx_ctx *c, const std::vector<std::string> &names, uint64_t *out) {
    std::lock_guard<std::recursive_mutex> g(c->ks.mu);
    RBX_TRY(set_device(c));
    ScratchOrder so_(c, c->stream);
    const uint32_t n = (uint32_t)names.size();
    std::vector<HllState *> hl(n);
    std::vector<std::shared_ptr<HllState>> keep(n);
    for (uint32_t i = 0; i < n; ++i) {
        RBX_TRY(hll_get(c, names[i], false, c->stream, &keep[i], nullptr));
        hl[i] = keep[i].get();
    }
    return pfcount_each(c, hl, out);
}

// PFCOUNT k1..kn: one key = the cached single-key count; several = count of the union
static int hll_count(rbx_ctx *c, const std::vector<std::string> &names, uint64_t *out) {
    if (names.size() == 1) return hll_count_each(c, names, out);
    std::lock_guard<std::recursive_mutex> g(c->ks.mu);
    RBX_TRY(set_device(c));
    ScratchOrder so_(c, c->stream);
    std::vector<std::shared_ptr<HllState>> keep;
    std::vector<uint8_t *> srcs;
    for (const auto &nm : names) {
        std::shared_ptr<HllState> h;
        RBX_TRY(hll_get(c, nm, false, c->stream, &h, nullptr));
        if (h) {
            srcs.push_back(h->d_regs);
            keep.push_back(h);
        }
    }
    if (srcs.empty()) {
        *out = 0;
        return RBX_OK;
    }
    RBX_TRY(c->ptrs.reserve(srcs.size() * sizeof(uint8_t *)));
    RBX_TRY(c->out_bytes.reserve(kHllBytes));
    HIP_TRY(hipMemcpyAsync(c->ptrs.p, srcs.data(), srcs.size() * sizeof(uint8_t *), hipMemcpyHostToDevice, c->stream));
    launch_hll_union(c->ptrs.as<uint8_t *>(), (uint32_t)srcs.size(), c->out_bytes.as<uint8_t>(), c->stream);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipStreamSynchronize(c->stream));
    std::vector<uint8_t *> u{c->out_bytes.as<uint8_t>()};
    return count_regs(c, u, out);
}

int rbx_hll_count_each(rbx_ctx *c, const char *const *names, uint32_t n, uint64_t *out) {
    if (!c || (n && (!names || !out))) return fail(RBX_E_ILLEGAL_ARGUMENT, "NULL argument");
    std::vector<std::string> v;
    RBX_TRY(cstr_names(names, n, &v));
    return hll_count_each(c, v, out);
}

int rbx_hll_count(rbx_ctx *c, const char *const *names, uint32_t n, uint64_t *out) {
    if (!c || !names || !out || n == 0) return fail(RBX_E_ILLEGAL_ARGUMENT, "NULL/empty argument");
    std::vector<std::string> v;
    RBX_TRY(cstr_names(names, n, &v));
    return hll_count(c, v, out);
}

int rbx_hll_count_n(rbx_ctx *c, const rbx_name *names, uint32_t n, uint64_t *out) {
    if (!c || !names || !out || n == 0) return fail(RBX_E_ILLEGAL_ARGUMENT, "NULL/empty argument");
    std::vector<std::string> v;
    RBX_TRY(names_of(names, n, &v));
    return hll_count(c, v, out);
}

// PFMERGE dest src1..srcn (dest's own registers included)
static int hll_merge(rbx_ctx *c, const std::string &dest, const std::vector<std::string> &srcs) {
    std::lock_guard<std::recursive_mutex> g(c->ks.mu);
    RBX_TRY(set_device(c));
    ScratchOrder so_(c, c->stream);
    std::vector<std::shared_ptr<HllState>> keep;
    std::vector<uint8_t *> sp;
    for (const auto &s : srcs) {  // type-check every source first (isHLLObjectOrReply)
        std::shared_ptr<HllState> h;
        RBX_TRY(hll_get(c, s, false, c->stream, &h, nullptr));
        if (h) {
            sp.push_back(h->d_regs);
            keep.push_back(h);
        }
    }
    std::shared_ptr<HllState> d;
    RBX_TRY(hll_get(c, dest, true, c->stream, &d, nullptr));
    RBX_TRY(resolve_dense(c, d.get()));
    for (auto &h : keep) {
        RBX_TRY(resolve_dense(c, h.get()));
        d->dense = d->dense || h->dense;  // pfmergeCommand: use_dense if any input is
    }
    if (!sp.empty()) {
        RBX_TRY(c->ptrs.reserve(sp.size() * sizeof(uint8_t *)));
        HIP_TRY(hipMemcpyAsync(c->ptrs.p, sp.data(), sp.size() * sizeof(uint8_t *), hipMemcpyHostToDevice, c->stream));
        launch_hll_merge(d->d_regs, c->ptrs.as<uint8_t *>(), (uint32_t)sp.size(), c->stream);
        HIP_TRY(hipGetLastError());
        RBX_TRY(replay_merge(c, {d.get()}, c->stream));
    }
    HIP_TRY(hipStreamSynchronize(c->stream));
    d->card |= 1ULL << 63;  // HLL_INVALIDATE_CACHE
    return RBX_OK;
}

int rbx_hll_merge(rbx_ctx *c, const char *dest, const char *const *srcs, uint32_t nsrc) {
    if (!c || !dest || (nsrc && !srcs)) return fail(RBX_E_ILLEGAL_ARGUMENT, "NULL argument");
    std::vector<std::string> v;
    RBX_TRY(cstr_names(srcs, nsrc, &v));
    return hll_merge(c, dest, v);
}

int rbx_hll_merge_n(rbx_ctx *c, rbx_name dest, const rbx_name *srcs, uint32_t nsrc) {
    if (!c || (!dest.bytes && dest.len) || (nsrc && !srcs)) return fail(RBX_E_ILLEGAL_ARGUMENT, "NULL argument");
    std::vector<std::string> v;
    RBX_TRY(names_of(srcs, nsrc, &v));
    return hll_merge(c, name_of(dest), v);
}

// Redis HLL strings: 16-byte header ("HYLL", encoding, 3 unused, 8 cached-cardinality bytes)
// + dense registers (HLL_DENSE_SET_REGISTER layout, 6 bits each, LSB-first) or sparse opcodes.
constexpr uint64_t kHllDenseLen = 16 + 12288;

static void hll_header(uint8_t *s, int sparse, uint64_t card) {
    memcpy(s, "HYLL", 4);
    s[4] = (uint8_t)sparse;  // HLL_DENSE 0 / HLL_SPARSE 1
    s[5] = s[6] = s[7] = 0;
    for (int i = 0; i < 8; ++i) s[8 + i] = (uint8_t)(card >> (8 * i));
}

static void hll_encode_dense(const uint8_t *regs, uint8_t *p) {
    memset(p, 0, 12288);
    for (unsigned long r = 0; r < 16384; ++r) {
        const unsigned long byte = r * 6 / 8, fb = r * 6 & 7, fb8 = 8 - fb, v = regs[r];
        p[byte] |= (uint8_t)(v << fb);
        if (byte + 1 < 12288) p[byte + 1] |= (uint8_t)(v >> fb8);
    }
}

// Sparse opcodes with the fewest bytes: zero runs as ZERO (<= 64) or XZERO (65..16384), equal
// values as VAL runs of <= 4 (value 1..32).  Returns false when a register exceeds 32 (the
// sparse format cannot hold it).  Used for RBX_HLL_SPARSE exports of keys Redis holds dense
// (a sparse key exports the string it was built as, see hll_sparse_string).
static bool hll_encode_sparse(const uint8_t *regs, std::vector<uint8_t> &out) {
    out.clear();
    for (uint32_t i = 0; i < 16384;) {
        const uint8_t v = regs[i];
        uint32_t j = i + 1;
        while (j < 16384 && regs[j] == v) ++j;
        uint32_t run = j - i;
        if (v == 0) {
            if (run > 64) {
                out.push_back((uint8_t)(0x40 | ((run - 1) >> 8)));
                out.push_back((uint8_t)((run - 1) & 0xff));
            } else {
                out.push_back((uint8_t)(run - 1));
            }
        } else {
            if (v > 32) return false;
            for (; run; run -= std::min<uint32_t>(run, 4))
                out.push_back((uint8_t)(0x80 | ((v - 1) << 2) | (std::min<uint32_t>(run, 4) - 1)));
        }
        i = j;
    }
    return true;
}

// The sparse string of a key Redis holds sparse, as it was built (k_hll_sparse_replay's list):
// an XZERO opcode is two bytes, ZERO / VAL one.  The caller holds a ScratchOrder on c->stream.
static int hll_sparse_string(rbx_ctx *c, HllState *h, std::vector<uint8_t> &out) {
    uint32_t st[kHllStateWords];
    HIP_TRY(hipMemcpyAsync(st, h->d_promoted, sizeof(st), hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    out.clear();
    if (st[1] == 0) {  // createHLLObject
        out = {0x7f, 0xff};
        return RBX_OK;
    }
    std::vector<uint16_t> ops(st[1]);
    HIP_TRY(hipMemcpy(ops.data(), h->d_sp_ops, ops.size() * 2, hipMemcpyDeviceToHost));
    for (uint16_t op : ops) {
        if (op >= 0x100) out.push_back((uint8_t)(op >> 8));
        out.push_back((uint8_t)op);
    }
    if (out.size() != st[2]) return fail(RBX_E_DEVICE, "sparse HLL string length mismatch");
    return RBX_OK;
}

static int hll_export_enc(rbx_ctx *c, const std::string &name, int encoding, uint8_t *out, uint64_t cap,
                          uint64_t *len) {
    if (encoding < RBX_HLL_DENSE || encoding > RBX_HLL_AS_STORED)
        return fail(RBX_E_ILLEGAL_ARGUMENT, "encoding must be RBX_HLL_DENSE, RBX_HLL_SPARSE or RBX_HLL_AS_STORED");
    std::lock_guard<std::recursive_mutex> g(c->ks.mu);
    RBX_TRY(set_device(c));
    ScratchOrder so_(c, c->stream);
    std::shared_ptr<HllState> h;
    RBX_TRY(hll_get(c, name, false, c->stream, &h, nullptr));
    if (!h) {
        if (len) *len = 0;
        return RBX_OK;
    }
    if (encoding != RBX_HLL_DENSE) RBX_TRY(resolve_dense(c, h.get()));
    std::vector<uint8_t> s;
    bool sparse = false;
    if (encoding != RBX_HLL_DENSE && !h->dense) {
        std::vector<uint8_t> ops;
        RBX_TRY(hll_sparse_string(c, h.get(), ops));
        s.resize(16 + ops.size());
        memcpy(s.data() + 16, ops.data(), ops.size());
        sparse = true;
    } else {
        std::vector<uint8_t> regs(kHllBytes);
        HIP_TRY(hipMemcpyAsync(regs.data(), h->d_regs, kHllBytes, hipMemcpyDeviceToHost, c->stream));
        HIP_TRY(hipStreamSynchronize(c->stream));
        if (encoding == RBX_HLL_SPARSE) {
            std::vector<uint8_t> ops;
            if (!hll_encode_sparse(regs.data(), ops))
                return fail(RBX_E_ILLEGAL_ARGUMENT, "a register exceeds 32: not representable in the sparse encoding");
            s.resize(16 + ops.size());
            memcpy(s.data() + 16, ops.data(), ops.size());
            sparse = true;
        } else {
            s.resize(kHllDenseLen);
            hll_encode_dense(regs.data(), s.data() + 16);
        }
    }
    hll_header(s.data(), sparse, h->card);
    if (len) *len = s.size();
    if (out) memcpy(out, s.data(), std::min<uint64_t>(cap, s.size()));
    return RBX_OK;
}

int rbx_hll_export_enc(rbx_ctx *c, const char *name, int encoding, uint8_t *out, uint64_t cap, uint64_t *len) {
    if (!c || !name) return fail(RBX_E_ILLEGAL_ARGUMENT, "NULL argument");
    return hll_export_enc(c, name, encoding, out, cap, len);
}

int rbx_hll_export_enc_n(rbx_ctx *c, rbx_name name, int encoding, uint8_t *out, uint64_t cap, uint64_t *len) {
    if (!c || (!name.bytes && name.len)) return fail(RBX_E_ILLEGAL_ARGUMENT, "NULL argument");
    return hll_export_enc(c, name_of(name), encoding, out, cap, len);
}

int rbx_hll_export(rbx_ctx *c, const char *name, uint8_t *out, uint64_t cap, uint64_t *len) {
    return rbx_hll_export_enc(c, name, RBX_HLL_DENSE, out, cap, len);
}

// accepts the Redis dense and sparse encodings (isHLLObjectOrReply validation)
static int hll_import(rbx_ctx *c, const std::string &name, const uint8_t *bytes, uint64_t len) {
    if (len < 16 || memcmp(bytes, "HYLL", 4) != 0 || bytes[4] > 1) return fail(RBX_E_WRONGTYPE, kHllWrongType);
    std::vector<uint8_t> regs(kHllBytes, 0);
    std::vector<uint16_t> ops;  // sparse: the opcodes as stored (SET keeps the string)
    if (bytes[4] == 0) {
        if (len != kHllDenseLen) return fail(RBX_E_WRONGTYPE, kHllWrongType);
        const uint8_t *p = bytes + 16;
        for (unsigned long r = 0; r < 16384; ++r) {
            unsigned long byte = r * 6 / 8, fb = r * 6 & 7, fb8 = 8 - fb;
            unsigned long b0 = p[byte], b1 = byte + 1 < 12288 ? p[byte + 1] : 0;
            regs[r] = (uint8_t)(((b0 >> fb) | (b1 << fb8)) & 63);
        }
    } else {
        const uint8_t *p = bytes + 16, *end = bytes + len;
        uint64_t idx = 0;
        while (p < end) {
            uint8_t b = *p;
            uint64_t run;
            if ((b & 0xc0) == 0) {  // ZERO
                run = (b & 0x3f) + 1;
                ops.push_back(b);
                p++;
            } else if ((b & 0xc0) == 0x40) {  // XZERO
                if (p + 1 >= end) return fail(RBX_E_WRONGTYPE, kHllWrongType);
                run = (((uint64_t)(b & 0x3f) << 8) | p[1]) + 1;
                ops.push_back((uint16_t)(b << 8 | p[1]));
                p += 2;
            } else {  // VAL
                ops.push_back(b);
                run = (b & 3) + 1;
                uint8_t v = ((b >> 2) & 0x1f) + 1;
                if (idx + run > 16384) return fail(RBX_E_WRONGTYPE, kHllWrongType);
                for (uint64_t j = 0; j < run; ++j) regs[idx + j] = v;
                p++;
            }
            idx += run;
            if (idx > 16384) return fail(RBX_E_WRONGTYPE, kHllWrongType);
        }
        if (idx != 16384) return fail(RBX_E_WRONGTYPE, kHllWrongType);
    }
    std::lock_guard<std::recursive_mutex> g(c->ks.mu);
    RBX_TRY(set_device(c));
    ScratchOrder so_(c, c->stream);
    Entry *ex = c->ks.find(name);
    std::shared_ptr<HllState> h;
    if (ex && ex->type == KType::Hll) {
        h = ex->hll;
        ex->expire_at = -1;  // SET discards the timeout
    } else {
        c->ks.generation++;
        RBX_TRY(hll_alloc(c, c->stream, &h));
        c->ks.put(name, Entry{KType::Hll, nullptr, nullptr, h});
    }
    uint64_t card = 0;
    for (int i = 0; i < 8; ++i) card |= (uint64_t)bytes[8 + i] << (8 * i);
    h->card = card;
    h->dense = bytes[4] == 0;  // SET keeps the string's encoding
    RBX_TRY(hll_ops_reserve(h.get(), ops.size()));
    // state: not promoted, the stored opcodes (a sparse string covers 16384 registers: >= 1)
    const uint32_t st[kHllStateWords] = {0u, (uint32_t)ops.size(), (uint32_t)(len - 16), 0u};
    HIP_TRY(hipMemcpyAsync(h->d_promoted, st, sizeof(st), hipMemcpyHostToDevice, c->stream));
    if (!ops.empty())
        HIP_TRY(hipMemcpyAsync(h->d_sp_ops, ops.data(), ops.size() * 2, hipMemcpyHostToDevice, c->stream));
    HIP_TRY(hipMemcpyAsync(h->d_regs, regs.data(), kHllBytes, hipMemcpyHostToDevice, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    return RBX_OK;
}

int rbx_hll_import(rbx_ctx *c, const char *name, const uint8_t *bytes, uint64_t len) {
    if (!c || !name || !bytes) return fail(RBX_E_ILLEGAL_ARGUMENT, "NULL argument");
    return hll_import(c, name, bytes, len);
}

int rbx_hll_import_n(rbx_ctx *c, rbx_name name, const uint8_t *bytes, uint64_t len) {
    if (!c || (!name.bytes && name.len) || !bytes) return fail(RBX_E_ILLEGAL_ARGUMENT, "NULL argument");
    return hll_import(c, name_of(name), bytes, len);
}

int rbx_hll_delete(rbx_ctx *c, const char *name, int *deleted) {
    if (!c || !name) return fail(RBX_E_ILLEGAL_ARGUMENT, "NULL argument");
    return ks_del(c->ks, {std::string(name)}, deleted);
}

int rbx_hll_exists(rbx_ctx *c, const char *name, int *exists) {
    if (!c || !name || !exists) return fail(RBX_E_ILLEGAL_ARGUMENT, "NULL argument");
    return ks_exists(c->ks, {std::string(name)}, exists);
}

static int hll_open(rbx_ctx *c, const std::string &name, int create, rbx_hll **out) {
    std::lock_guard<std::recursive_mutex> g(c->ks.mu);
    RBX_TRY(set_device(c));
    ScratchOrder so_(c, c->stream);
    std::shared_ptr<HllState> h;
    RBX_TRY(hll_get(c, name, create != 0, c->stream, &h, nullptr));
    if (!h) return fail(RBX_E_NO_SUCH_KEY, "ERR no such key");
    HIP_TRY(hipStreamSynchronize(c->stream));
    *out = new rbx_hll{c, name, h, c->ks.generation};
    c->refs.fetch_add(1);
    return RBX_OK;
}

int rbx_hll_open(rbx_ctx *c, const char *name, int create, rbx_hll **out) {
    if (!c || !name || !out) return fail(RBX_E_ILLEGAL_ARGUMENT, "NULL argument");
    return hll_open(c, name, create, out);
}

int rbx_hll_open_n(rbx_ctx *c, rbx_name name, int create, rbx_hll **out) {
    if (!c || (!name.bytes && name.len) || !out) return fail(RBX_E_ILLEGAL_ARGUMENT, "NULL argument");
    return hll_open(c, name_of(name), create, out);
}

int rbx_hll_close(rbx_hll *h) {
    if (!h) return RBX_OK;
    rbx_ctx *c = h->ctx;
    {
        std::lock_guard<std::recursive_mutex> g(c->ks.mu);
        delete h;
    }
    ctx_release(c);
    return RBX_OK;
}

int rbx_hll_registers_dev(rbx_hll *h, void **d_regs) {
    if (!h || !d_regs) return fail(RBX_E_ILLEGAL_ARGUMENT, "NULL argument");
    rbx_ctx *c = h->ctx;
    std::lock_guard<std::recursive_mutex> g(c->ks.mu);
    RBX_TRY(set_device(c));
    ScratchOrder so_(c, c->stream);
    RBX_TRY(hll_bind(c, h, true, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));  // a re-created HLL's zero fill lands first
    *d_regs = h->st->d_regs;
    return RBX_OK;
}

int rbx_hll_add_multi_dev(rbx_ctx *c, rbx_hll *const *hlls, uint32_t nseg, const uint64_t *d_seg_offsets,
                          const uint64_t *h_seg_offsets, const rbx_keys *d_elements, uint32_t *d_changed,
                          void *stream) {
    (void)d_seg_offsets;
    if (!c || !hlls || !h_seg_offsets || !d_changed) return fail(RBX_E_ILLEGAL_ARGUMENT, "NULL argument");
    RBX_TRY(validate_keys(d_elements));
    std::lock_guard<std::recursive_mutex> g(c->ks.mu);
    RBX_TRY(set_device(c));
    hipStream_t st = pick_stream(c, stream);
    ScratchOrder so_(c, st);
    std::vector<HllState *> hl(nseg);
    for (uint32_t s = 0; s < nseg; ++s) {
        if (!hlls[s]) return fail(RBX_E_ILLEGAL_ARGUMENT, "NULL hll handle");
        RBX_TRY(hll_bind(c, hlls[s], true, st));
        hl[s] = hlls[s]->st.get();
        hl[s]->card |= 1ULL << 63;  // conservatively invalidate (the flags are device-side)
    }
    return pfadd_run(c, hl, h_seg_offsets, keys_dev(d_elements), d_changed, st);
}

int rbx_hll_count_each_handles(rbx_ctx *c, rbx_hll *const *hlls, uint32_t n, uint64_t *out) {
    if (!c || (n && (!hlls || !out))) return fail(RBX_E_ILLEGAL_ARGUMENT, "NULL argument");
    std::lock_guard<std::recursive_mutex> g(c->ks.mu);
    RBX_TRY(set_device(c));
    ScratchOrder so_(c, c->stream);
    std::vector<HllState *> hl(n);
    for (uint32_t i = 0; i < n; ++i) {
        if (hlls[i]) RBX_TRY(hll_bind(c, hlls[i], false, c->stream));
        hl[i] = hlls[i] ? hlls[i]->st.get() : nullptr;
    }
    return pfcount_each(c, hl, out);
}

// ---- register packing (the exchange step of an element-partitioned HLL set) ------------------
// hlls[i]'s 16384 registers <-> d_buf[i*16384, (i+1)*16384), on `st` (both enqueue only).
static int hll_handles_regs(rbx_ctx *c, rbx_hll *const *hlls, uint32_t n, hipStream_t st,
                            std::vector<uint8_t *> *regs) {
    regs->resize(n);
    for (uint32_t i = 0; i < n; ++i) {
        if (!hlls[i]) return fail(RBX_E_ILLEGAL_ARGUMENT, "NULL hll handle");
        RBX_TRY(hll_bind(c, hlls[i], true, st));
        (*regs)[i] = hlls[i]->st->d_regs;
    }
    return RBX_OK;
}

static int hll_pack_locked(rbx_ctx *c, rbx_hll *const *hlls, uint32_t n, uint8_t *d_buf, bool unpack_max,
                           hipStream_t st) {
    std::vector<uint8_t *> regs;
    RBX_TRY(hll_handles_regs(c, hlls, n, st, &regs));
    if (!n) return RBX_OK;
    RBX_TRY(c->ptrs.reserve(n * sizeof(uint8_t *)));
    HIP_TRY(hipMemcpyAsync(c->ptrs.p, regs.data(), n * sizeof(uint8_t *), hipMemcpyHostToDevice, st));
    launch_hll_pack(c->ptrs.as<uint8_t *>(), n, d_buf, unpack_max, st);
    HIP_TRY(hipGetLastError());
    if (unpack_max) {
        // the exchange merges the other ranks' registers in: a sparse HLL's string takes them
        // as PFMERGE's write-back would (ascending registers, promotion by the same rules)
        std::vector<HllState *> hs(n);
        for (uint32_t i = 0; i < n; ++i) {
            hlls[i]->st->card |= 1ULL << 63;  // HLL_INVALIDATE_CACHE
            hs[i] = hlls[i]->st.get();
        }
        RBX_TRY(replay_merge(c, hs, st));
    }
    // `regs` is a pageable host vector: the runtime has staged it when hipMemcpyAsync returns
    return RBX_OK;
}

int rbx_hll_pack_registers(rbx_ctx *c, rbx_hll *const *hlls, uint32_t n, void *d_buf, void *stream) {
    if (!c || (n && (!hlls || !d_buf))) return fail(RBX_E_ILLEGAL_ARGUMENT, "NULL argument");
    std::lock_guard<std::recursive_mutex> g(c->ks.mu);
    RBX_TRY(set_device(c));
    hipStream_t st = pick_stream(c, stream);
    ScratchOrder so_(c, st);
    return hll_pack_locked(c, hlls, n, (uint8_t *)d_buf, false, st);
}

int rbx_hll_unpack_max_registers(rbx_ctx *c, rbx_hll *const *hlls, uint32_t n, const void *d_buf, void *stream) {
    if (!c || (n && (!hlls || !d_buf))) return fail(RBX_E_ILLEGAL_ARGUMENT, "NULL argument");
    std::lock_guard<std::recursive_mutex> g(c->ks.mu);
    RBX_TRY(set_device(c));
    hipStream_t st = pick_stream(c, stream);
    ScratchOrder so_(c, st);
    return hll_pack_locked(c, hlls, n, (uint8_t *)d_buf, true, st);
}

// ---- RCCL -----------------------------------------------------------------------------------
int rbx_rccl_unique_id(uint8_t out[128]) {
    if (!out) return fail(RBX_E_ILLEGAL_ARGUMENT, "NULL argument");
    ncclUniqueId id;
    ncclResult_t r = ncclGetUniqueId(&id);
    if (r != ncclSuccess) return fail(RBX_E_DEVICE, ncclGetErrorString(r));
    memcpy(out, id.internal, 128);
    return RBX_OK;
}

int rbx_rccl_init(rbx_ctx *c, const uint8_t id[128], int nranks, int rank) {
    if (!c || !id || nranks < 1 || rank < 0 || rank >= nranks) return fail(RBX_E_ILLEGAL_ARGUMENT, "bad argument");
    std::lock_guard<std::recursive_mutex> g(c->ks.mu);
    RBX_TRY(set_device(c));
    if (c->comm) return fail(RBX_E_ILLEGAL_STATE, "rbx_rccl_init has already been called");
    ncclUniqueId u;
    memcpy(u.internal, id, 128);
    ncclResult_t r = ncclCommInitRank(&c->comm, nranks, u, rank);
    if (r != ncclSuccess) return fail(RBX_E_DEVICE, ncclGetErrorString(r));
    c->nranks = nranks;
    c->rank = rank;
    return RBX_OK;
}

// the communicator as RCCL sees it (ncclCommCount / ncclCommUserRank)
int rbx_rccl_info(rbx_ctx *c, int *nranks, int *rank) {
    if (!c) return fail(RBX_E_ILLEGAL_ARGUMENT, "NULL argument");
    std::lock_guard<std::recursive_mutex> g(c->ks.mu);
    if (!c->comm) return fail(RBX_E_ILLEGAL_STATE, "rbx_rccl_init has not been called");
    int n = 0, r = 0;
    ncclResult_t e = ncclCommCount(c->comm, &n);
    if (e == ncclSuccess) e = ncclCommUserRank(c->comm, &r);
    if (e != ncclSuccess) return fail(RBX_E_DEVICE, ncclGetErrorString(e));
    if (nranks) *nranks = n;
    if (rank) *rank = r;
    return RBX_OK;
}

// Every rank issues exactly ONE ncclAllReduce of n x 16384 bytes whatever its register pool
// layout: the registers are packed in the caller's (name) order into one contiguous buffer,
// max-reduced in place, and max-merged back.  (Coalescing "adjacent" pool blocks would make the
// number and sizes of the collectives depend on each rank's allocation history, and RCCL would
// pair mismatched calls.)  The pack/unpack kernels move 2 x 2 x n x 16 KiB of HBM (~0.1 ms for
// the 163.84 MB of C4), next to the all-reduce itself.
int rbx_hll_allreduce_max(rbx_ctx *c, rbx_hll *const *hlls, uint32_t n) {
    if (!c || (n && !hlls)) return fail(RBX_E_ILLEGAL_ARGUMENT, "NULL argument");
    std::lock_guard<std::recursive_mutex> g(c->ks.mu);
    RBX_TRY(set_device(c));
    if (!c->comm) return fail(RBX_E_ILLEGAL_STATE, "rbx_rccl_init has not been called");
    ScratchOrder so_(c, c->stream);
    const size_t bytes = (size_t)n * kHllBytes;
    RBX_TRY(c->hll_pack.reserve(std::max<size_t>(bytes, 16)));
    uint8_t *buf = c->hll_pack.as<uint8_t>();
    RBX_TRY(hll_pack_locked(c, hlls, n, buf, false, c->stream));
    ncclResult_t r = ncclAllReduce(buf, buf, bytes, ncclUint8, ncclMax, c->comm, c->stream);
    if (r != ncclSuccess) return fail(RBX_E_DEVICE, ncclGetErrorString(r));
    return hll_pack_locked(c, hlls, n, buf, true, c->stream);
}

// ---- asynchronous forms (RHyperLogLogAsync, M/api/RHyperLogLogAsync.java:37-70) ---------------
// The call is queued on the context's serial executor (host_exec.h) and runs after every call
// queued before it; names, segment offsets and the rbx_keys descriptor are copied at submit time,
// key bytes and output buffers are read / written when the call runs (valid until completion).
static int submit_async(rbx_ctx *c, std::function<int()> fn, rbx_callback cb, void *user, rbx_future **out) {
    if (!c || !out) return fail(RBX_E_ILLEGAL_ARGUMENT, "NULL argument");
    // exec_mu is held through the submit, so rbx_shutdown cannot free the executor under it; the
    // queued call holds a context reference until it has run (the context outlives a shutdown
    // issued from a completion callback while calls are still queued).
    std::lock_guard<std::mutex> g(c->exec_mu);
    if (!c->exec) return fail(RBX_E_ILLEGAL_STATE, "the context has been shut down");
    c->refs.fetch_add(1);
    auto f = c->exec->submit(
        [c, fn = std::move(fn)]() {
            const int rc = fn();
            ctx_release(c);
            return rc;
        },
        cb, user);
    if (!f) {
        ctx_release(c);
        return fail(RBX_E_ILLEGAL_STATE, "the context has been shut down");
    }
    *out = new rbx_future{std::move(f)};
    return RBX_OK;
}

int rbx_future_wait(rbx_future *f, int64_t timeout_ms, int *call_rc) {
    if (!f) return fail(RBX_E_ILLEGAL_ARGUMENT, "NULL future");
    if (!f->f->wait(timeout_ms)) return fail(RBX_E_TIMEOUT, "the call has not completed");
    std::lock_guard<std::mutex> g(f->f->mu);
    if (call_rc) *call_rc = f->f->rc;
    if (f->f->rc) fail(f->f->rc, f->f->msg);  // rbx_last_error() on this thread = the call's message
    return RBX_OK;
}

int rbx_future_done(rbx_future *f, int *done) {
    if (!f || !done) return fail(RBX_E_ILLEGAL_ARGUMENT, "NULL argument");
    std::lock_guard<std::mutex> g(f->f->mu);
    *done = f->f->done;
    return RBX_OK;
}

int rbx_future_free(rbx_future *f) {
    delete f;  // the executor keeps its own reference until the call completes
    return RBX_OK;
}

int rbx_bloom_add_async(rbx_ctx *c, const char *name, uint64_t size, uint32_t k, const rbx_keys *keys,
                        uint8_t *out_new, uint64_t *out_count, rbx_callback cb, void *user, rbx_future **out) {
    if (!c || !name || !keys) return fail(RBX_E_ILLEGAL_ARGUMENT, "NULL argument");
    std::string nm(name);
    rbx_keys kc = *keys;
    return submit_async(c, [=]() { return rbx_bloom_add(c, nm.c_str(), size, k, &kc, out_new, out_count); }, cb,
                        user, out);
}

int rbx_bloom_contains_async(rbx_ctx *c, const char *name, uint64_t size, uint32_t k, const rbx_keys *keys,
                             uint8_t *out_present, uint64_t *out_count, rbx_callback cb, void *user,
                             rbx_future **out) {
    if (!c || !name || !keys) return fail(RBX_E_ILLEGAL_ARGUMENT, "NULL argument");
    std::string nm(name);
    rbx_keys kc = *keys;
    return submit_async(c, [=]() { return rbx_bloom_contains(c, nm.c_str(), size, k, &kc, out_present, out_count); },
                        cb, user, out);
}

// addAsync / addAllAsync (:71-81)
int rbx_hll_add_async(rbx_ctx *c, const char *name, const rbx_keys *elements, int *changed, rbx_callback cb,
                      void *user, rbx_future **out) {
    if (!c || !name || !elements) return fail(RBX_E_ILLEGAL_ARGUMENT, "NULL argument");
    std::string nm(name);
    rbx_keys kc = *elements;
    return submit_async(c, [=]() { return rbx_hll_add(c, nm.c_str(), &kc, changed); }, cb, user, out);
}

int rbx_hll_add_multi_async(rbx_ctx *c, const char *const *names, uint32_t nseg, const uint64_t *seg_offsets,
                            const rbx_keys *elements, uint8_t *out_changed, rbx_callback cb, void *user,
                            rbx_future **out) {
    if (!c || !names || !seg_offsets || !elements) return fail(RBX_E_ILLEGAL_ARGUMENT, "NULL argument");
    std::vector<std::string> v;
    RBX_TRY(cstr_names(names, nseg, &v));
    std::vector<uint64_t> seg(seg_offsets, seg_offsets + nseg + 1);
    rbx_keys kc = *elements;
    return submit_async(c, [=]() { return hll_add_multi(c, v, seg.data(), &kc, out_changed); }, cb, user, out);
}

// countAsync / countWithAsync (:84-94)
int rbx_hll_count_async(rbx_ctx *c, const char *const *names, uint32_t n, uint64_t *result, rbx_callback cb,
                        void *user, rbx_future **out) {
    if (!c || !names || !result || n == 0) return fail(RBX_E_ILLEGAL_ARGUMENT, "NULL/empty argument");
    std::vector<std::string> v;
    RBX_TRY(cstr_names(names, n, &v));
    return submit_async(c, [=]() { return hll_count(c, v, result); }, cb, user, out);
}

// mergeWithAsync (:97-102)
int rbx_hll_merge_async(rbx_ctx *c, const char *dest, const char *const *srcs, uint32_t nsrc, rbx_callback cb,
                        void *user, rbx_future **out) {
    if (!c || !dest || (nsrc && !srcs)) return fail(RBX_E_ILLEGAL_ARGUMENT, "NULL argument");
    std::vector<std::string> v;
    RBX_TRY(cstr_names(srcs, nsrc, &v));
    std::string d(dest);
    return submit_async(c, [=]() { return hll_merge(c, d, v); }, cb, user, out);
}

// ---- self test of the host-compiled device primitives (CPU tests call this) ------------
// Returns the number of mismatches of mod63 against '%' over `n` pseudo-random pairs.
uint64_t rbx_selftest_mod(uint64_t n, uint64_t seed) {
    uint64_t bad = 0, s = seed;
    auto next = [&]() {
        uint64_t z = (s += 0x9e3779b97f4a7c15ULL);
        z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
        z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
        return z ^ (z >> 31);
    };
    for (uint64_t i = 0; i < n; ++i) {
        uint64_t d;
        uint64_t r = next();
        switch (r & 7) {
        case 0: d = 1 + (next() & 0xff); break;
        case 1: d = (1ULL << 32) - (next() & 0xff); break;
        case 2: d = (1ULL << (1 + (next() % 32))); break;
        case 3: d = (1ULL << 31) + (next() & 0xffff) - 0x8000; break;
        default: d = 1 + (next() % (1ULL << 32)); break;
        }
        if (d == 0 || d > (1ULL << 32)) d = 1;
        ModParams p = make_mod_params(d);
        for (int t = 0; t < 16; ++t) {
            uint64_t h = next() & 0x7fffffffffffffffULL;
            if (t == 0) h = 0x7fffffffffffffffULL;
            if (t == 1) h = d - 1;
            if (t == 2) h = d;
            if (mod63(h, p) != (uint32_t)(h % d)) ++bad;
        }
    }
    return bad;
}

// HighwayHash128 / MurmurHash64A of the host-compiled device code (CPU cross-check).
void rbx_selftest_hash128(const uint8_t *data, uint64_t len, uint64_t out[2]) {
    HH s;
    hh_reset(s);
    uint64_t i = 0;
    for (; i + 32 <= len; i += 32) {
        uint32_t w[8];
        memcpy(w, data + i, 32);
        hh_packet(s, w);
    }
    uint32_t r = (uint32_t)(len & 31);
    if (r) {
        uint32_t t[8] = {0}, p[8];
        memcpy(t, data + i, r);
        for (int j = (int)r; j < 32; ++j) ((uint8_t *)t)[j] = 0xA5;  // garbage past the tail
        hh_tail_packet(t, r, p);
        hh_remainder_prologue(s, r);
        hh_packet(s, p);
    }
    hh_finalize128(s, out[0], out[1]);
}

// ---- measurement helpers (include/rbx_bench.h) -----------------------------------------------
int rbx_bench_gather(rbx_ctx *c, const void *d_table, uint64_t table_bytes, uint64_t nkeys, uint32_t k,
                     void *d_sink, void *stream) {
    if (!c || !d_table || !d_sink || table_bytes < 4) return fail(RBX_E_ILLEGAL_ARGUMENT, "bad argument");
    RBX_TRY(set_device(c));
    launch_gather_probe((const uint32_t *)d_table, table_bytes / 4, nkeys, k, (uint32_t *)d_sink,
                        pick_stream(c, stream));
    HIP_TRY(hipGetLastError());
    return RBX_OK;
}

int rbx_bench_slice_probe(rbx_ctx *c, const void *d_entries, uint64_t per_bucket, uint32_t nbuckets,
                          const void *d_bitmap, uint64_t slice_bytes, unsigned grid, void *d_sink, void *stream) {
    if (!c || !d_entries || !d_bitmap || !d_sink || grid < 8 || slice_bytes < 4 || (slice_bytes & (slice_bytes - 1)))
        return fail(RBX_E_ILLEGAL_ARGUMENT, "bad argument");
    RBX_TRY(set_device(c));
    uint32_t lg = 0;
    while ((4ULL << lg) < slice_bytes) ++lg;
    launch_bench_slice_probe(d_entries, per_bucket, nbuckets, (const uint32_t *)d_bitmap, lg, grid & ~7u,
                             (uint32_t *)d_sink, pick_stream(c, stream));
    HIP_TRY(hipGetLastError());
    return RBX_OK;
}

static int quiesce(rbx_ctx *c);
int rbx_bench_add_stamps(rbx_ctx *c, unsigned long long *out, uint32_t n) {
    if (!c || !out || n > 16) return fail(RBX_E_ILLEGAL_ARGUMENT, "rbx_bench_add_stamps: n <= 16");
    // the context's lock and device, and only this context's work drained
    std::lock_guard<std::recursive_mutex> g(c->ks.mu);
    RBX_TRY(set_device(c));  // fails on a shut context (pa_stamps freed)
    if (c->pa_stamps.cap == 0) {
        memset(out, 0, n * 8);
        return RBX_OK;
    }
    RBX_TRY(quiesce(c));
    HIP_TRY(hipMemcpyAsync(out, c->pa_stamps.p, n * 8, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipMemsetAsync(c->pa_stamps.p, 0, 16 * 8, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    return RBX_OK;
}

int rbx_bench_stream_read(rbx_ctx *c, const void *d_buf, uint64_t bytes, void *d_sink, void *stream) {
    if (!c || !d_buf || !d_sink || ((uintptr_t)d_buf & 15)) return fail(RBX_E_ILLEGAL_ARGUMENT, "bad argument");
    RBX_TRY(set_device(c));
    launch_stream_read(d_buf, bytes, (uint32_t *)d_sink, pick_stream(c, stream));
    HIP_TRY(hipGetLastError());
    return RBX_OK;
}

int rbx_bench_stream_write(rbx_ctx *c, void *d_buf, uint64_t bytes, void *stream) {
    if (!c || !d_buf || ((uintptr_t)d_buf & 15)) return fail(RBX_E_ILLEGAL_ARGUMENT, "bad argument");
    RBX_TRY(set_device(c));
    launch_stream_write(d_buf, bytes, pick_stream(c, stream));
    HIP_TRY(hipGetLastError());
    return RBX_OK;
}

int rbx_bench_gather_segments(rbx_ctx *c, const void *d_table, uint64_t table_bytes, uint64_t segment_bytes,
                              uint64_t keys_per_segment, uint64_t nkeys, void *d_sink, void *stream) {
    if (!c || !d_table || !d_sink || segment_bytes < 4 || table_bytes < segment_bytes || !keys_per_segment)
        return fail(RBX_E_ILLEGAL_ARGUMENT, "bad argument");
    RBX_TRY(set_device(c));
    launch_gather_segments((const uint32_t *)d_table, table_bytes / 4, segment_bytes / 4, keys_per_segment, nkeys,
                           (uint32_t *)d_sink, pick_stream(c, stream));
    HIP_TRY(hipGetLastError());
    return RBX_OK;
}

int rbx_bench_gather_regions(rbx_ctx *c, const void *d_table, uint64_t table_bytes, uint64_t region_bytes,
                             uint64_t nlanes, unsigned grid, void *d_sink, void *stream) {
    if (!c || !d_table || !d_sink || region_bytes < 4 || table_bytes < region_bytes || grid < 8)
        return fail(RBX_E_ILLEGAL_ARGUMENT, "bad argument");
    RBX_TRY(set_device(c));
    launch_gather_regions((const uint32_t *)d_table, table_bytes / 4, region_bytes / 4, nlanes, (uint32_t *)d_sink,
                          pick_stream(c, stream), grid & ~7u);
    HIP_TRY(hipGetLastError());
    return RBX_OK;
}

int rbx_host_alloc(uint64_t bytes, void **out) {
    if (!out) return fail(RBX_E_ILLEGAL_ARGUMENT, "NULL out");
    HIP_TRY(hipHostMalloc(out, bytes ? bytes : 1, hipHostMallocDefault));
    return RBX_OK;
}

int rbx_host_free(void *p) {
    if (p) HIP_TRY(hipHostFree(p));
    return RBX_OK;
}

int rbx_set_staging(rbx_ctx *c, uint64_t bytes) {
    if (!c || bytes < 4096) return fail(RBX_E_ILLEGAL_ARGUMENT, "staging must be >= 4 KiB");
    std::lock_guard<std::recursive_mutex> g(c->ks.mu);
    c->staging_bytes = bytes;
    return RBX_OK;
}

// ---- sizeInMemory (M/RedissonObject.java:124-130, Bloom: both keys, M/RedissonBloomFilter.java:234-238)
// Bytes the engine holds for each existing key: a bitmap's device allocation (+ its 256-byte
// length-word tail), an HLL's 16384 register bytes, a config hash's fields; plus the key name.
// Redis' MEMORY USAGE reports its own allocator's figures, which no engine reproduces.
static int memory_usage(rbx_ctx *c, const std::vector<std::string> &names, uint64_t *bytes) {
    std::lock_guard<std::recursive_mutex> g(c->ks.mu);
    uint64_t total = 0;
    for (const auto &nm : names) {
        Entry *e = c->ks.find(nm);
        if (!e) continue;
        total += nm.size();
        if (e->type == KType::Bitmap) total += e->bm->cap_bytes + 256;
        else if (e->type == KType::Hll) total += kHllBytes;
        else total += sizeof(BloomConfig) + e->cfg->fpp_str.size();
    }
    *bytes = total;
    return RBX_OK;
}

int rbx_memory_usage_n(rbx_ctx *c, const rbx_name *names, uint32_t n, uint64_t *bytes) {
    if (!c || !bytes) return fail(RBX_E_ILLEGAL_ARGUMENT, "NULL argument");
    std::vector<std::string> v;
    RBX_TRY(names_of(names, n, &v));
    return memory_usage(c, v, bytes);
}

int rbx_bloom_size_in_memory(rbx_ctx *c, const char *name, uint64_t *bytes) {
    if (!c || !name || !bytes) return fail(RBX_E_ILLEGAL_ARGUMENT, "NULL argument");
    return memory_usage(c, {std::string(name), config_name(name)}, bytes);
}

// ---- key timeouts (RedissonExpirable, M/RedissonExpirable.java:53-251; keyspace.cpp) ----------
int rbx_pexpire(rbx_ctx *c, const char *const *names, uint32_t n, int64_t when_ms, int absolute, int cond,
                int *result) {
    if (!c || (n && !names)) return fail(RBX_E_ILLEGAL_ARGUMENT, "bad argument");
    std::vector<std::string> v;
    RBX_TRY(cstr_names(names, n, &v));
    return ks_pexpire(c->ks, v, when_ms, absolute, cond, result);
}

int rbx_pexpire_n(rbx_ctx *c, const rbx_name *names, uint32_t n, int64_t when_ms, int absolute, int cond,
                  int *result) {
    if (!c) return fail(RBX_E_ILLEGAL_ARGUMENT, "bad argument");
    std::vector<std::string> v;
    RBX_TRY(names_of(names, n, &v));
    return ks_pexpire(c->ks, v, when_ms, absolute, cond, result);
}

int rbx_persist(rbx_ctx *c, const char *const *names, uint32_t n, int *result) {
    if (!c || (n && !names)) return fail(RBX_E_ILLEGAL_ARGUMENT, "bad argument");
    std::vector<std::string> v;
    RBX_TRY(cstr_names(names, n, &v));
    return ks_persist(c->ks, v, result);
}

int rbx_pttl(rbx_ctx *c, const char *name, int64_t *out) {
    if (!c || !name || !out) return fail(RBX_E_ILLEGAL_ARGUMENT, "NULL argument");
    return ks_pttl(c->ks, name, out);
}

int rbx_pexpiretime(rbx_ctx *c, const char *name, int64_t *out) {
    if (!c || !name || !out) return fail(RBX_E_ILLEGAL_ARGUMENT, "NULL argument");
    return ks_pexpiretime(c->ks, name, out);
}

// ---- replicas: digest and device-to-device copies between contexts ---------------------------
// Waits until every engine call issued on `c` so far has finished on the device (the scratch
// event chain orders them all, whatever stream each used), so its objects can be read elsewhere.
static int quiesce(rbx_ctx *c) {
    if (c->ev_scratch && c->scratch_stream) HIP_TRY(hipEventSynchronize(c->ev_scratch));
    HIP_TRY(hipStreamSynchronize(c->stream));
    return RBX_OK;
}

static uint64_t mix64_host(uint64_t x) {
    x ^= x >> 31;
    x *= 0x7fb5d329728ea185ULL;
    x ^= x >> 27;
    x *= 0x81dadef4bc2dd44dULL;
    x ^= x >> 33;
    return x;
}

int rbx_bloom_digest_n(rbx_ctx *c, rbx_name name, uint64_t *out) {
    if (!c || (!name.bytes && name.len) || !out) return fail(RBX_E_ILLEGAL_ARGUMENT, "NULL argument");
    std::lock_guard<std::recursive_mutex> g(c->ks.mu);
    RBX_TRY(set_device(c));
    ScratchOrder so_(c, c->stream);
    Entry *e = c->ks.find(name_of(name));
    if (!e) {
        *out = 0;  // a missing key (GET = nil)
        return RBX_OK;
    }
    if (e->type != KType::Bitmap) return fail(RBX_E_WRONGTYPE, kWrongTypeMsg);
    int rc;
    const uint64_t len = read_dev_u64(c, e->bm->d_len, &rc);
    RBX_TRY(rc);
    RBX_TRY(c->counters.reserve(64));
    auto *d = c->counters.as<unsigned long long>() + 4;
    HIP_TRY(hipMemsetAsync(d, 0, 8, c->stream));
    if (len) launch_digest((const uint8_t *)e->bm->d_words, len, d, c->stream);
    HIP_TRY(hipGetLastError());
    const uint64_t v = read_dev_u64(c, d, &rc);
    RBX_TRY(rc);
    *out = v + mix64_host(len ^ 0xD1B54A32D192ED03ULL) + 1;  // never 0 for an existing key
    return RBX_OK;
}

int rbx_bloom_digest(rbx_ctx *c, const char *name, uint64_t *out) {
    if (!name) return fail(RBX_E_ILLEGAL_ARGUMENT, "NULL argument");
    return rbx_bloom_digest_n(c, rbx_name{(const uint8_t *)name, strlen(name)}, out);
}

// Replica sync of one Bloom filter: dst's {name}:config := src's (all four fields) and dst's
// bitmap string := src's, copied device to device (hipMemcpyPeerAsync: xGMI between the GPUs of
// a node, a plain device copy on one GPU).  The replica's key timeouts are not copied.
int rbx_bloom_copy_to(rbx_ctx *src, rbx_ctx *dst, rbx_name name) {
    if (!src || !dst || (!name.bytes && name.len)) return fail(RBX_E_ILLEGAL_ARGUMENT, "NULL argument");
    if (src == dst) return fail(RBX_E_ILLEGAL_ARGUMENT, "source and destination are the same context");
    std::scoped_lock lk(src->ks.mu, dst->ks.mu);
    const std::string nm = name_of(name);
    RBX_TRY(set_device(src));
    if (dst->shut) return fail(RBX_E_ILLEGAL_STATE, "the context has been shut down");
    BloomConfig cfg;
    RBX_TRY(ks_get_config(src->ks, nm, &cfg));
    RBX_TRY(check_offsets(cfg.size));
    Entry *e = src->ks.find(nm);
    if (e && e->type != KType::Bitmap) return fail(RBX_E_WRONGTYPE, kWrongTypeMsg);
    std::shared_ptr<Bitmap> sb = e ? e->bm : nullptr;
    uint64_t len = 0;
    if (sb) {
        RBX_TRY(quiesce(src));
        int rc;
        len = read_dev_u64(src, sb->d_len, &rc);
        RBX_TRY(rc);
    }
    RBX_TRY(set_device(dst));
    ScratchOrder so_(dst, dst->stream);
    dst->ks.put(config_name(nm), Entry{KType::Config, std::make_shared<BloomConfig>(cfg), nullptr, nullptr});
    dst->ks.generation++;
    if (!sb) {  // the source has no bitmap yet: neither has the replica
        dst->ks.erase(nm);
        return RBX_OK;
    }
    const uint64_t bits = std::max<uint64_t>(size_bits(cfg.size), len * 8);
    std::shared_ptr<Bitmap> b;
    Entry *de = dst->ks.find(nm);
    if (de && de->type == KType::Bitmap && de->bm->cap_bytes >= (bits + 7) / 8) {
        b = de->bm;  // in place: the replica's open handles keep seeing it
        HIP_TRY(hipMemsetAsync(b->d_words, 0, b->cap_bytes, dst->stream));
    } else {
        RBX_TRY(new_bitmap(dst, bits, dst->stream, &b));
    }
    if (len) HIP_TRY(hipMemcpyPeerAsync(b->d_words, dst->device, sb->d_words, src->device, len, dst->stream));
    static thread_local unsigned long long L;
    L = len;
    HIP_TRY(hipMemcpyAsync(b->d_len, &L, 8, hipMemcpyHostToDevice, dst->stream));
    HIP_TRY(hipStreamSynchronize(dst->stream));
    dst->ks.put(nm, Entry{KType::Bitmap, nullptr, b, nullptr});
    dst->ks.generation++;
    return RBX_OK;
}

// PFMERGE's input from another GPU: dst_name on dst := src_name on src (registers, encoding,
// cached cardinality and promotion word), device to device.  A missing source deletes dst_name.
int rbx_hll_copy_to(rbx_ctx *src, rbx_name src_name, rbx_ctx *dst, rbx_name dst_name) {
    if (!src || !dst || (!src_name.bytes && src_name.len) || (!dst_name.bytes && dst_name.len))
        return fail(RBX_E_ILLEGAL_ARGUMENT, "NULL argument");
    const std::string sn = name_of(src_name), dn = name_of(dst_name);
    if (src == dst && sn == dn) return RBX_OK;
    std::unique_lock<std::recursive_mutex> l1(src->ks.mu, std::defer_lock), l2(dst->ks.mu, std::defer_lock);
    if (src == dst) l1.lock();
    else std::lock(l1, l2);
    RBX_TRY(set_device(src));
    if (dst->shut) return fail(RBX_E_ILLEGAL_STATE, "the context has been shut down");
    Entry *e = src->ks.find(sn);
    if (e && e->type != KType::Hll) return fail(RBX_E_WRONGTYPE, kHllWrongType);
    if (!e) {
        dst->ks.erase(dn);
        return RBX_OK;
    }
    std::shared_ptr<HllState> sh = e->hll;
    RBX_TRY(quiesce(src));
    RBX_TRY(set_device(dst));
    ScratchOrder so_(dst, dst->stream);
    Entry *de = dst->ks.find(dn);
    if (de && de->type != KType::Hll) {
        dst->ks.erase(dn);
        de = nullptr;
    }
    std::shared_ptr<HllState> h;
    if (de) {
        h = de->hll;
        de->expire_at = -1;  // SET semantics
    } else {
        RBX_TRY(hll_alloc(dst, dst->stream, &h));
        dst->ks.put(dn, Entry{KType::Hll, nullptr, nullptr, h});
        dst->ks.generation++;
    }
    h->card = sh->card;
    h->dense = sh->dense;
    // the source's opcode count (its state word [1]) sizes the copy and the destination's list
    uint32_t sst[kHllStateWords];
    HIP_TRY(hipSetDevice(src->device));
    HIP_TRY(hipMemcpy(sst, sh->d_promoted, sizeof(sst), hipMemcpyDeviceToHost));
    HIP_TRY(hipSetDevice(dst->device));
    RBX_TRY(hll_ops_reserve(h.get(), sst[1]));
    HIP_TRY(hipMemcpyPeerAsync(h->d_regs, dst->device, sh->d_regs, src->device, kHllBytes, dst->stream));
    HIP_TRY(hipMemcpyPeerAsync(h->d_promoted, dst->device, sh->d_promoted, src->device, kHllStateWords * 4, dst->stream));
    if (sst[1])
        HIP_TRY(hipMemcpyPeerAsync(h->d_sp_ops, dst->device, sh->d_sp_ops, src->device, (size_t)sst[1] * 2, dst->stream));
    HIP_TRY(hipStreamSynchronize(dst->stream));
    return RBX_OK;
}

// Peer access between the GPUs of a node (best effort: copies work without it, staged).
int rbx_enable_peer_access(int device, int peer) {
    if (device == peer) return RBX_OK;
    int can = 0;
    HIP_TRY(hipDeviceCanAccessPeer(&can, device, peer));
    if (!can) return RBX_OK;
    HIP_TRY(hipSetDevice(device));
    const hipError_t e = hipDeviceEnablePeerAccess(peer, 0);
    if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled) return fail(RBX_E_DEVICE, hipGetErrorString(e));
    (void)hipGetLastError();
    return RBX_OK;
}

// Tuning knobs (process-wide).  "contains_stage1": early-exit width of contains (0 = off).
int rbx_bench_stream_geometry(rbx_ctx *c, uint64_t *out) {
    if (!c || !out) return fail(RBX_E_ILLEGAL_ARGUMENT, "NULL argument");
    std::lock_guard<std::recursive_mutex> g(c->ks.mu);
    for (int i = 0; i < 4; ++i) out[i] = c->st_geom[i];
    return RBX_OK;
}

int rbx_tune(const char *key, int value) {
    if (!key) return fail(RBX_E_ILLEGAL_ARGUMENT, "NULL key");
    if (!strcmp(key, "contains_partition")) {
        if (value < 0 || value > 2) return fail(RBX_E_ILLEGAL_ARGUMENT, "contains_partition in [0, 2]");
        g_partition_mode = value;
        return RBX_OK;
    }
    // DIAGNOSTICS ONLY, profiling build (kDiag; tools/microbench.py pflags / padiag through RBX_LIB_PATH):
    // contains_partition_flags 4 = stage 1 emits no pairs, 8 = the probe records no misses, 16 = one
    // atomicOr per clear bit, 32 = no bit-0 gather, 64 = phase stamps; add_partition_diag 4 = the region
    // kernel emits no records, 8 = it loads only its first two regions' pairs, 16 = it only loads, 64 =
    // phase stamps (rbx_bench_add_stamps).  librbx.so rejects them: no knob there changes an answer.
    if (!strcmp(key, "contains_partition_flags") || !strcmp(key, "add_partition_diag") || !strcmp(key, "stream_diag")) {
        if (!kDiag) return fail(RBX_E_ILLEGAL_ARGUMENT, std::string(key) + ": diagnostics exist only in librbx_diag.so");
        if (!strcmp(key, "contains_partition_flags")) {
            if (value != 0 && value != 4 && value != 8 && value != 12 && value != 16 && value != 32 && value != 64)
                return fail(RBX_E_ILLEGAL_ARGUMENT, "contains_partition_flags in {0, 4, 8, 12, 16, 32, 64}");
            g_partition_flags = value;
        } else if (!strcmp(key, "add_partition_diag")) {
            if (value < 0 || (value & ~92) != 0) return fail(RBX_E_ILLEGAL_ARGUMENT, "add_partition_diag: bits of 4|8|16|64");
            g_add_partition_diag = value;
        } else {
            if (value < 0 || (value & ~9) != 0) return fail(RBX_E_ILLEGAL_ARGUMENT, "stream_diag: bits of 1|8");
            set_stream_diag(value);
        }
        return RBX_OK;
    }
    // How the add's region kernel reports which keys are new (add_partitioned.hip k_ba_mode):
    // 0 owner bits, 1 non-owner counters, 3 owner records, 2 (default) chosen from the sampled
    // fill.  Exact either way.
    if (!strcmp(key, "add_records")) {
        if (value < 0 || value > 3) return fail(RBX_E_ILLEGAL_ARGUMENT, "add_records in [0, 3]");
        g_add_record_policy = value;
        return RBX_OK;
    }
    if (!strcmp(key, "add_partition")) {
        if (value < 0 || value > 2) return fail(RBX_E_ILLEGAL_ARGUMENT, "add_partition in [0, 2]");
        g_add_partition_mode = value;
        return RBX_OK;
    }
    if (!strcmp(key, "contains_multi_slots")) {
        if (value < 0 || value > 2) return fail(RBX_E_ILLEGAL_ARGUMENT, "contains_multi_slots in [0, 2]");
        g_multi_slots = value;
        return RBX_OK;
    }
    // EXPERIMENTS (tools/microbench.py): shape and grid of the slot contains kernel (stage 5)
    if (!strcmp(key, "stream_table8")) {
        if (value != 0 && value != 1) return fail(RBX_E_ILLEGAL_ARGUMENT, "stream_table8 is 0 or 1");
        g_stream_table8 = value;
        return RBX_OK;
    }
    if (!strcmp(key, "stream_chunk")) {
        if (value < 0) return fail(RBX_E_ILLEGAL_ARGUMENT, "stream_chunk >= 0 (0: 2^26 / k commands)");
        g_stream_chunk = (uint64_t)value;
        return RBX_OK;
    }
    if (!strcmp(key, "wide_subchunk")) {
        if (value < 0) return fail(RBX_E_ILLEGAL_ARGUMENT, "wide_subchunk >= 0 (0: 2^29 / k keys)");
        g_wide_subchunk = (uint64_t)value;
        return RBX_OK;
    }
    if (!strcmp(key, "contains_qgrid")) {
        if (value < 256 || value > 8192) return fail(RBX_E_ILLEGAL_ARGUMENT, "contains_qgrid in [256, 8192]");
        set_contains_qgrid(value);
        return RBX_OK;
    }
    if (!strcmp(key, "stream_qgrid")) {
        if (value < 256 || value > 8192) return fail(RBX_E_ILLEGAL_ARGUMENT, "stream_qgrid in [256, 8192]");
        set_stream_qgrid(value);
        return RBX_OK;
    }
    if (!strcmp(key, "add_multi_table8")) {
        if (value != 0 && value != 2) return fail(RBX_E_ILLEGAL_ARGUMENT, "add_multi_table8: 0 or 2");
        g_add_multi_t8 = value;
        return RBX_OK;
    }
    if (!strcmp(key, "add_multi_segment")) {
        if (value < 0 || value > 1) return fail(RBX_E_ILLEGAL_ARGUMENT, "add_multi_segment: 0 or 1");
        g_madd_seg = value;
        return RBX_OK;
    }
    if (!strcmp(key, "add_multi_segmax")) {
        if (value < 1 || value > (int)kSegMaxKeys) return fail(RBX_E_ILLEGAL_ARGUMENT, "add_multi_segmax in [1, 16384]");
        g_madd_segmax = (uint64_t)value;
        return RBX_OK;
    }
    if (!strcmp(key, "add_multi_conflict_log2")) {
        if (value < 6 || value > 24) return fail(RBX_E_ILLEGAL_ARGUMENT, "add_multi_conflict_log2 in [6, 24]");
        g_maddx_lgc = (uint32_t)value;
        return RBX_OK;
    }
    if (!strcmp(key, "add_region_grid")) {
        if (value < 256 || value > 65536) return fail(RBX_E_ILLEGAL_ARGUMENT, "add_region_grid in [256, 65536]");
        set_add_region_grid(value);
        return RBX_OK;
    }
    if (!strcmp(key, "add_multi_seg_grid")) {
        if (value < 64 || value > 65536) return fail(RBX_E_ILLEGAL_ARGUMENT, "add_multi_seg_grid in [64, 65536]");
        g_madd_seg_grid = (uint32_t)value;
        return RBX_OK;
    }
    if (!strcmp(key, "stream_final_grid")) {
        if (value < 32 || value > 2048) return fail(RBX_E_ILLEGAL_ARGUMENT, "stream_final_grid in [32, 2048]");
        set_stream_final_grid(value);
        return RBX_OK;
    }
    if (!strcmp(key, "host_small_bytes")) {
        if (value < 4096 || value > (64 << 20)) return fail(RBX_E_ILLEGAL_ARGUMENT, "host_small_bytes in [4 KiB, 64 MiB]");
        g_small_bytes = (uint64_t)value;
        return RBX_OK;
    }
    if (!strcmp(key, "host_tiny_spin")) {
        if (value != 0 && value != 1) return fail(RBX_E_ILLEGAL_ARGUMENT, "host_tiny_spin in {0, 1}");
        g_tiny_spin = value;
        return RBX_OK;
    }
    if (!strcmp(key, "add_one_key")) {
        if (value != 0 && value != 1) return fail(RBX_E_ILLEGAL_ARGUMENT, "add_one_key in {0, 1}");
        g_add_one = value;
        return RBX_OK;
    }
    if (!strcmp(key, "add_single_seg_keys")) {
        if (value < 0 || value > (int64_t)kSegMaxKeys) return fail(RBX_E_ILLEGAL_ARGUMENT, "add_single_seg_keys in [0, 16384]");
        g_seg_single_keys = (uint64_t)value;
        return RBX_OK;
    }
    if (!strcmp(key, "host_tiny_keys")) {
        if (value < 0 || value > (int64_t)kSegMaxKeys) return fail(RBX_E_ILLEGAL_ARGUMENT, "host_tiny_keys in [0, 16384]");
        g_tiny_keys = (uint64_t)value;
        return RBX_OK;
    }
    if (!strcmp(key, "host_small_batches")) {
        if (value != 0 && value != 1) return fail(RBX_E_ILLEGAL_ARGUMENT, "host_small_batches in {0, 1}");
        g_small_host = value;
        return RBX_OK;
    }
    if (!strcmp(key, "add_rec_lds_limit")) {
        if (value < 0 || value > 7168) return fail(RBX_E_ILLEGAL_ARGUMENT, "add_rec_lds_limit in [0, 7168]");
        set_add_rec_lds_limit(value);
        return RBX_OK;
    }
    if (!strcmp(key, "contains_stage1")) {
        if (value < 0 || value > 5) return fail(RBX_E_ILLEGAL_ARGUMENT, "contains_stage1 in [0, 5]");
        set_contains_stage1(value);
        return RBX_OK;
    }
    return fail(RBX_E_ILLEGAL_ARGUMENT, std::string("unknown tuning key ") + key);
}

// Java BigDecimal.valueOf(d).toPlainString() as stored in the config hash.
int rbx_selftest_plain_string(double d, char *out, int cap) {
    std::string s = java_plain_string(d);
    if (!out || cap <= 0) return (int)s.size();
    snprintf(out, (size_t)cap, "%s", s.c_str());
    return (int)s.size();
}

}  // extern "C"
