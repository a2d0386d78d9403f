// node_fake_rbx.cpp -- TEST INFRASTRUCTURE: a host-memory stand-in for the per-GPU half of the C ABI
// (include/rbx.h) that redisson_amd/csrc/rbx_node.cpp is written against, so the node router
// (slot routing, the GPU worker pool, replication barrier, failure semantics, handle cache) builds
// with plain g++ under TSan / ASan and runs on the CPU (tests/test_sanitizers.py).
//
// Keys live in the real keyspace (keyspace.cpp: config rules, DEL / EXISTS, generations); only
// the device objects are replaced by host vectors:
//   - a Bloom bitmap is its Redis string (MSB-first bytes, grown to the highest SETBIT), with the
//     reference's in-order add semantics (a key is new iff one of its k SETBITs returned 0,
//     M/RedissonBloomFilter.java:104-137); bit indexes come from FNV-1a, NOT HighwayHash -- the
//     hashing is the GPU library's business and is parity-tested against the oracle elsewhere;
//   - an HLL is 16384 raw registers; its "count" here is the number of nonzero registers of the
//     union, a stand-in that keeps PFCOUNT's union semantics, not redis' estimator.
// Every call takes the context's keyspace lock, as librbx.so does, and yields inside it so the
// router's concurrency is exercised with realistic critical sections.
#include <algorithm>
#include <atomic>
#include <cstring>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/rbx.h"
#include "../../redisson_amd/csrc/keyspace.h"

namespace rbx {
struct Bitmap {
    std::vector<uint8_t> bytes;
};
struct HllState {
    std::vector<uint8_t> regs = std::vector<uint8_t>(16384, 0);
};
}  // namespace rbx

using namespace rbx;

struct rbx_ctx {
    Keyspace ks;
    int device = 0;
    std::atomic<int> refs{1};
};
struct rbx_bloom {
    rbx_ctx *ctx;
    std::string name;
    int64_t size;
    uint32_t k;
};

static const char *kWrong = "WRONGTYPE Operation against a key holding the wrong kind of value";

static void release(rbx_ctx *c) {
    if (c->refs.fetch_sub(1) == 1) delete c;
}

static std::string name_of(rbx_name n) { return std::string((const char *)n.bytes, (size_t)n.len); }

static void key_span(const rbx_keys *k, uint64_t i, const uint8_t **p, uint64_t *len) {
    if (k->offsets) {
        *p = k->bytes + k->offsets[i];
        *len = k->offsets[i + 1] - k->offsets[i];
    } else {
        *p = k->bytes + i * k->stride;
        *len = k->stride;
    }
}

static uint64_t fnv(const uint8_t *p, uint64_t n, uint64_t seed) {
    uint64_t h = 0xcbf29ce484222325ULL ^ seed;
    for (uint64_t i = 0; i < n; ++i) h = (h ^ p[i]) * 0x100000001b3ULL;
    return h;
}

static bool get_bit(const Bitmap &b, uint64_t i) {
    return (i >> 3) < b.bytes.size() && (b.bytes[i >> 3] >> (7 - (i & 7)) & 1);
}
static bool set_bit(Bitmap &b, uint64_t i) {  // SETBIT i 1, returns the old bit
    if ((i >> 3) >= b.bytes.size()) b.bytes.resize((i >> 3) + 1, 0);
    const uint8_t m = (uint8_t)(1u << (7 - (i & 7)));
    const bool old = b.bytes[i >> 3] & m;
    b.bytes[i >> 3] |= m;
    return old;
}

// one add(Collection) / contains(Collection) on an existing config, keys [i0, i1); lock held
static int bloom_apply(rbx_ctx *c, const std::string &name, int64_t size, uint32_t k, const rbx_keys *keys,
                       uint64_t i0, uint64_t i1, uint8_t *out, uint64_t *count, bool is_add) {
    std::this_thread::yield();
    Entry *e = c->ks.find(name);
    if (e && e->type != KType::Bitmap) return fail(RBX_E_WRONGTYPE, kWrong);
    if (!e && is_add) {
        c->ks.put(name, Entry{KType::Bitmap, nullptr, std::make_shared<Bitmap>(), nullptr});
        c->ks.generation++;
        e = c->ks.find(name);
    }
    const uint64_t m = size_bits(size);
    uint64_t cnt = 0;
    for (uint64_t i = i0; i < i1; ++i) {
        const uint8_t *p;
        uint64_t len;
        key_span(keys, i, &p, &len);
        const uint64_t h1 = fnv(p, len, 0), h2 = fnv(p, len, 0x9e3779b97f4a7c15ULL) | 1;
        bool flag = is_add ? false : true;
        for (uint32_t j = 0; j < k; ++j) {
            const uint64_t idx = (h1 + j * h2) % m;
            if (is_add) flag |= !set_bit(*e->bm, idx);
            else flag &= e ? get_bit(*e->bm, idx) : false;
        }
        cnt += flag;
        if (out) out[i] = flag;
    }
    if (count) *count = cnt;
    return RBX_OK;
}

static int bloom_op(rbx_ctx *c, rbx_name name, uint64_t size, uint32_t k, const rbx_keys *keys, uint8_t *out,
                    uint64_t *count, bool is_add) {
    if (!c || !keys) return fail(RBX_E_ILLEGAL_ARGUMENT, "NULL argument");
    const std::string nm = name_of(name);
    std::lock_guard<std::recursive_mutex> g(c->ks.mu);
    int64_t sz = (int64_t)size;
    if (sz == 0) {
        BloomConfig cfg;
        const int rc = ks_get_config(c->ks, nm, &cfg);
        if (rc) return rc;
        sz = cfg.size;
        k = cfg.k;
    }
    const int rc = ks_config_check(c->ks, nm, sz, k);
    if (rc) return rc;
    if (keys->n == 0) return fail(RBX_E_ARITHMETIC, "/ by zero");
    return bloom_apply(c, nm, sz, k, keys, 0, keys->n, out, count, is_add);
}

extern "C" {

const char *rbx_last_error(void) { return last_error_message(); }

int rbx_init(int device, rbx_ctx **out) {
    if (!out) return fail(RBX_E_ILLEGAL_ARGUMENT, "NULL argument");
    *out = new rbx_ctx();
    (*out)->device = device;
    return RBX_OK;
}

int rbx_shutdown(rbx_ctx *c) {
    if (c) release(c);
    return RBX_OK;
}

int rbx_enable_peer_access(int, int) { return RBX_OK; }

int rbx_bloom_try_init_n(rbx_ctx *c, rbx_name name, int64_t n, double p, int *created) {
    return ks_bloom_try_init(c->ks, name_of(name), n, p, created);
}

int rbx_bloom_read_config_n(rbx_ctx *c, rbx_name name, rbx_bloom_config *out) {
    BloomConfig cfg;
    const int rc = ks_get_config(c->ks, name_of(name), &cfg);
    if (rc) return rc;
    memset(out, 0, sizeof(*out));
    out->size = cfg.size;
    out->hash_iterations = cfg.k;
    out->expected_insertions = cfg.expected;
    out->false_probability = cfg.fpp;
    snprintf(out->false_probability_str, sizeof(out->false_probability_str), "%s", cfg.fpp_str.c_str());
    return RBX_OK;
}

int rbx_bloom_add_n(rbx_ctx *c, rbx_name name, uint64_t size, uint32_t k, const rbx_keys *keys, uint8_t *out_new,
                    uint64_t *out_count) {
    return bloom_op(c, name, size, k, keys, out_new, out_count, true);
}

int rbx_bloom_contains_n(rbx_ctx *c, rbx_name name, uint64_t size, uint32_t k, const rbx_keys *keys,
                         uint8_t *out_present, uint64_t *out_count) {
    return bloom_op(c, name, size, k, keys, out_present, out_count, false);
}

int rbx_bloom_count_n(rbx_ctx *c, rbx_name name, int64_t *out) {
    const std::string nm = name_of(name);
    std::lock_guard<std::recursive_mutex> g(c->ks.mu);
    BloomConfig cfg;
    const int rc = ks_get_config(c->ks, nm, &cfg);
    if (rc) return rc;
    uint64_t bits = 0;
    if (Entry *e = c->ks.find(nm)) {
        if (e->type != KType::Bitmap) return fail(RBX_E_WRONGTYPE, kWrong);
        for (uint8_t b : e->bm->bytes) bits += (uint64_t)__builtin_popcount(b);
    }
    *out = (int64_t)bits;  // the popcount stands in for the estimator
    return RBX_OK;
}

int rbx_del_n(rbx_ctx *c, const rbx_name *names, uint32_t n, int *deleted) {
    std::vector<std::string> v;
    for (uint32_t i = 0; i < n; ++i) v.push_back(name_of(names[i]));
    std::lock_guard<std::recursive_mutex> g(c->ks.mu);
    std::this_thread::yield();
    return ks_del(c->ks, v, deleted);
}

int rbx_exists_n(rbx_ctx *c, const rbx_name *names, uint32_t n, int *count) {
    std::vector<std::string> v;
    for (uint32_t i = 0; i < n; ++i) v.push_back(name_of(names[i]));
    return ks_exists(c->ks, v, count);
}

// replica sync: dst's config and bitmap := src's (read under src's lock, written under dst's)
int rbx_bloom_copy_to(rbx_ctx *src, rbx_ctx *dst, rbx_name name) {
    const std::string nm = name_of(name), cn = config_name(nm);
    BloomConfig cfg;
    std::shared_ptr<Bitmap> copy;
    {
        std::lock_guard<std::recursive_mutex> g(src->ks.mu);
        const int rc = ks_get_config(src->ks, nm, &cfg);
        if (rc) return rc;
        if (Entry *e = src->ks.find(nm)) {
            if (e->type != KType::Bitmap) return fail(RBX_E_WRONGTYPE, kWrong);
            copy = std::make_shared<Bitmap>(*e->bm);
        }
    }
    std::this_thread::yield();
    std::lock_guard<std::recursive_mutex> g(dst->ks.mu);
    dst->ks.put(cn, Entry{KType::Config, std::make_shared<BloomConfig>(cfg), nullptr, nullptr});
    if (copy) dst->ks.put(nm, Entry{KType::Bitmap, nullptr, copy, nullptr});
    else dst->ks.erase(nm);
    dst->ks.generation++;
    return RBX_OK;
}

int rbx_hll_copy_to(rbx_ctx *src, rbx_name src_name, rbx_ctx *dst, rbx_name dst_name) {
    std::shared_ptr<HllState> copy;
    {
        std::lock_guard<std::recursive_mutex> g(src->ks.mu);
        if (Entry *e = src->ks.find(name_of(src_name))) {
            if (e->type != KType::Hll) return fail(RBX_E_WRONGTYPE, kWrong);
            copy = std::make_shared<HllState>(*e->hll);
        }
    }
    std::lock_guard<std::recursive_mutex> g(dst->ks.mu);
    if (copy) dst->ks.put(name_of(dst_name), Entry{KType::Hll, nullptr, nullptr, copy});
    else dst->ks.erase(name_of(dst_name));
    dst->ks.generation++;
    return RBX_OK;
}

int rbx_bloom_open_n(rbx_ctx *c, rbx_name name, rbx_bloom **out) {
    const std::string nm = name_of(name);
    std::lock_guard<std::recursive_mutex> g(c->ks.mu);
    BloomConfig cfg;
    const int rc = ks_get_config(c->ks, nm, &cfg);
    if (rc) return rc;
    *out = new rbx_bloom{c, nm, cfg.size, cfg.k};
    c->refs.fetch_add(1);
    return RBX_OK;
}

int rbx_bloom_close(rbx_bloom *b) {
    if (!b) return RBX_OK;
    rbx_ctx *c = b->ctx;
    {
        std::lock_guard<std::recursive_mutex> g(c->ks.mu);
        delete b;
    }
    release(c);
    return RBX_OK;
}

static int bloom_multi(rbx_ctx *c, rbx_bloom *const *f, uint32_t nseg, const uint64_t *seg, const rbx_keys *keys,
                       uint8_t *out, uint64_t *counts, bool is_add) {
    std::lock_guard<std::recursive_mutex> g(c->ks.mu);
    for (uint32_t s = 0; s < nseg; ++s) {  // every handle's cached config must still hold (addConfigCheck)
        if (f[s]->ctx != c) return fail(RBX_E_ILLEGAL_ARGUMENT, "handle of another context");
        const int rc = ks_config_check(c->ks, f[s]->name, f[s]->size, f[s]->k);
        if (rc) return rc;
    }
    for (uint32_t s = 0; s < nseg; ++s) {
        uint64_t cnt = 0;
        const int rc = bloom_apply(c, f[s]->name, f[s]->size, f[s]->k, keys, seg[s], seg[s + 1], out, &cnt, is_add);
        if (rc) return rc;
        counts[s] = cnt;
    }
    return RBX_OK;
}

int rbx_bloom_contains_multi(rbx_ctx *c, rbx_bloom *const *filters, uint32_t nseg, const uint64_t *seg_offsets,
                             const rbx_keys *keys, uint8_t *out_present, uint64_t *out_counts) {
    return bloom_multi(c, filters, nseg, seg_offsets, keys, out_present, out_counts, false);
}

int rbx_bloom_add_multi(rbx_ctx *c, rbx_bloom *const *filters, uint32_t nseg, const uint64_t *seg_offsets,
                        const rbx_keys *keys, uint8_t *out_new, uint64_t *out_counts) {
    return bloom_multi(c, filters, nseg, seg_offsets, keys, out_new, out_counts, true);
}

// PFADD per segment: register = max(register, rank), MurmurHash replaced by FNV (see the header)
int rbx_hll_add_multi_n(rbx_ctx *c, const rbx_name *names, uint32_t nseg, const uint64_t *seg,
                        const rbx_keys *el, uint8_t *out_changed) {
    std::lock_guard<std::recursive_mutex> g(c->ks.mu);
    std::this_thread::yield();
    for (uint32_t s = 0; s < nseg; ++s) {
        const std::string nm = name_of(names[s]);
        Entry *e = c->ks.find(nm);
        bool changed = false;
        if (e && e->type != KType::Hll) return fail(RBX_E_WRONGTYPE, kWrong);
        if (!e) {
            c->ks.put(nm, Entry{KType::Hll, nullptr, nullptr, std::make_shared<HllState>()});
            c->ks.generation++;
            e = c->ks.find(nm);
            changed = true;
        }
        for (uint64_t i = seg[s]; i < seg[s + 1]; ++i) {
            const uint8_t *p;
            uint64_t len;
            key_span(el, i, &p, &len);
            const uint64_t h = fnv(p, len, 0xadc83b19ULL);
            const uint8_t rank = (uint8_t)(1 + __builtin_ctzll((h >> 14) | (1ULL << 50)));
            uint8_t &r = e->hll->regs[h & 16383];
            if (rank > r) {
                r = rank;
                changed = true;
            }
        }
        if (out_changed) out_changed[s] = changed;
    }
    return RBX_OK;
}

int rbx_hll_count_n(rbx_ctx *c, const rbx_name *names, uint32_t n, uint64_t *out) {
    std::lock_guard<std::recursive_mutex> g(c->ks.mu);
    std::vector<uint8_t> u(16384, 0);
    for (uint32_t i = 0; i < n; ++i) {
        Entry *e = c->ks.find(name_of(names[i]));
        if (!e) continue;
        if (e->type != KType::Hll) return fail(RBX_E_WRONGTYPE, kWrong);
        for (int j = 0; j < 16384; ++j) u[j] = std::max(u[j], e->hll->regs[j]);
    }
    uint64_t nz = 0;
    for (uint8_t r : u) nz += r != 0;
    *out = nz;
    return RBX_OK;
}

int rbx_hll_merge_n(rbx_ctx *c, rbx_name dest, const rbx_name *srcs, uint32_t nsrc) {
    std::lock_guard<std::recursive_mutex> g(c->ks.mu);
    std::vector<uint8_t> u(16384, 0);
    const std::string dn = name_of(dest);
    for (uint32_t i = 0; i <= nsrc; ++i) {
        Entry *e = c->ks.find(i == nsrc ? dn : name_of(srcs[i]));
        if (!e) continue;
        if (e->type != KType::Hll) return fail(RBX_E_WRONGTYPE, kWrong);
        for (int j = 0; j < 16384; ++j) u[j] = std::max(u[j], e->hll->regs[j]);
    }
    auto st = std::make_shared<HllState>();
    st->regs = u;
    c->ks.put(dn, Entry{KType::Hll, nullptr, nullptr, st});
    c->ks.generation++;
    return RBX_OK;
}

}  // extern "C"

// inspection for node_test.cpp: the bitmap string of `name` on context c (false: no bitmap key)
bool fake_bitmap_bytes(rbx_ctx *c, const std::string &name, std::vector<uint8_t> *out) {
    std::lock_guard<std::recursive_mutex> g(c->ks.mu);
    Entry *e = c->ks.find(name);
    if (!e || e->type != KType::Bitmap) return false;
    *out = e->bm->bytes;
    return true;
}
