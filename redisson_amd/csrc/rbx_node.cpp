// rbx_node.cpp -- one process over the GPUs of a node (include/rbx.h, "one process over the GPUs
// of a node").  A pure host-side router written against the public per-GPU C ABI: a node holds
// one rbx_ctx per GPU and sends every name to GPU = calc_slot(name) * n_gpus / 16384, the slot
// routing the reference's client applies per command
// (M/cluster/ClusterConnectionManager.java:777-830) and per batch, where each node's commands
// are grouped and sent together (M/command/CommandBatchService.java:569-604).
//
// Multi-tenant batches are scattered by slot into per-GPU host arenas, run concurrently (one host
// thread per GPU with work; each GPU has its own context, stream and copy stream, so the PCIe
// uploads and kernels of different GPUs overlap) and gathered back in segment order.
#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <cstring>
#include <deque>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <set>
#include <shared_mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/rbx.h"
#include "../../include/rbx_bench.h"
#include "keyspace.h"

using namespace rbx;

// A cached Bloom handle, closed when the last holder lets go: the cache holds one reference and
// every in-flight batch holds its own, so a handle evicted (DEL) or replaced (config re-created)
// while another thread still runs a batch on it is closed when that batch ends.
struct NodeHandle {
    rbx_bloom *h = nullptr;
    ~NodeHandle() {
        if (h) rbx_bloom_close(h);
    }
};
using HandleRef = std::shared_ptr<NodeHandle>;

// Above this many cached handles the cache is emptied (handles are re-opened on demand): a
// long-lived node with tenant churn does not keep one handle per name it ever served.
constexpr size_t kMaxCachedHandles = 1u << 20;

// One worker thread per GPU of the node: a call's per-GPU parts run on the GPUs' workers
// concurrently (r03 started a std::thread per GPU per call).  Worker g runs GPU g's parts in the
// order they are submitted.
class GpuWorkers {
  public:
    explicit GpuWorkers(int n) : ws_(n) {
        for (auto &w : ws_) {
            w = std::make_unique<W>();
            W *p = w.get();
            p->th = std::thread([p] { p->loop(); });
        }
    }
    ~GpuWorkers() {
        for (auto &w : ws_) {
            {
                std::lock_guard<std::mutex> lk(w->mu);
                w->stop = true;
            }
            w->cv.notify_one();
            w->th.join();
        }
    }
    void submit(int g, std::function<void()> f) {
        W &w = *ws_[g];
        {
            std::lock_guard<std::mutex> lk(w.mu);
            w.q.push_back(std::move(f));
        }
        w.cv.notify_one();
    }

  private:
    struct W {
        std::thread th;
        std::mutex mu;
        std::condition_variable cv;
        std::deque<std::function<void()>> q;
        bool stop = false;
        void loop() {
            for (;;) {
                std::function<void()> f;
                {
                    std::unique_lock<std::mutex> lk(mu);
                    cv.wait(lk, [&] { return stop || !q.empty(); });
                    if (q.empty()) return;  // stop, and nothing left
                    f = std::move(q.front());
                    q.pop_front();
                }
                f();
            }
        }
    };
    std::vector<std::unique_ptr<W>> ws_;
};

// Writer-preferring shared mutex for the replication barrier: std::shared_mutex is
// glibc's reader-preferring rwlock, so under sustained overlapping batches (shared holders) a
// replicate / DEL of a replicated name (exclusive) could wait forever.  Here a waiting writer stops
// new shared holders; the batches already inside drain, the writer runs, then they resume.  No
// holder takes it twice.
class ReplBarrier {
  public:
    void lock() {
        std::unique_lock<std::mutex> l(m_);
        ++writers_waiting_;
        cv_.wait(l, [&] { return !writer_ && readers_ == 0; });
        --writers_waiting_;
        writer_ = true;
    }
    void unlock() {
        {
            std::lock_guard<std::mutex> l(m_);
            writer_ = false;
        }
        cv_.notify_all();
    }
    void lock_shared() {
        std::unique_lock<std::mutex> l(m_);
        cv_.wait(l, [&] { return !writer_ && writers_waiting_ == 0; });
        ++readers_;
    }
    void unlock_shared() {
        bool last;
        {
            std::lock_guard<std::mutex> l(m_);
            last = --readers_ == 0;
        }
        if (last) cv_.notify_all();
    }

  private:
    std::mutex m_;
    std::condition_variable cv_;
    int readers_ = 0, writers_waiting_ = 0;
    bool writer_ = false;
};

struct rbx_node {
    std::vector<rbx_ctx *> ctx;
    std::unique_ptr<GpuWorkers> workers;
    std::mutex mu;                                           // the handle cache and the replica set
    std::map<std::pair<int, std::string>, HandleRef> blooms;  // open handles per (GPU, name)
    // Bloom filters replicated on every GPU (rbx_node_bloom_replicate): adds go to every replica,
    // contains are spread over them (Redisson's ReadMode.SLAVE reads,
    // M/config/BaseMasterSlaveServersConfig.java:60; GETBIT is a read, M/RedissonBitSet.java:277-279)
    std::set<std::string> replicated;
    // Replication barrier: a batch holds it shared from the moment it reads `replicated` until its
    // kernels are done; replicate(on / off), DEL, and dropping the copies after a failed replicated
    // add hold it exclusively.  So a replica copy never misses an add that ran during the copy, and
    // copies are never deleted under a contains already routed to them.
    ReplBarrier repl_mu;
    // test hook (rbx_node_test_fail_adds): the next fail_adds[g] Bloom adds on GPU g fail
    std::unique_ptr<std::atomic<int>[]> fail_adds;
};

static bool is_replicated(rbx_node *nd, const std::string &name) {
    std::lock_guard<std::mutex> lk(nd->mu);
    return nd->replicated.count(name) != 0;
}

static std::atomic<uint64_t> g_tmp_serial{1};

static std::string str_of(const rbx_name &n) { return std::string((const char *)n.bytes, (size_t)n.len); }
static rbx_name name_ref(const std::string &s) { return rbx_name{(const uint8_t *)s.data(), (uint64_t)s.size()}; }

static int gpu_of(const rbx_node *nd, const std::string &name) {
    return slot_to_gpu(calc_slot((const uint8_t *)name.data(), name.size()), (int)nd->ctx.size());
}

static int check_name(const rbx_name &n) {
    if (!n.bytes && n.len) return fail(RBX_E_ILLEGAL_ARGUMENT, "NULL key name");
    return RBX_OK;
}

#define NODE_TRY(expr)                 \
    do {                               \
        const int r_ = (expr);         \
        if (r_ != RBX_OK) return r_;   \
    } while (0)

// Runs fn(g) for every GPU g with work, concurrently (on the GPUs' workers) when more than one;
// the first failure (in GPU order) becomes this thread's error.  fn must not call per_gpu.
template <class Fn>
static int per_gpu(rbx_node *nd, const std::vector<int> &gpus, Fn &&fn) {
    struct Res {
        int rc = RBX_OK;
        std::string msg;
    };
    std::vector<Res> res(gpus.size());
    auto run = [&](size_t i) {
        res[i].rc = fn(gpus[i]);
        if (res[i].rc != RBX_OK) res[i].msg = rbx_last_error();  // the worker's thread-local message
    };
    if (gpus.size() == 1) {
        run(0);
    } else {
        std::mutex mu;
        std::condition_variable cv;
        size_t left = gpus.size();
        for (size_t i = 0; i < gpus.size(); ++i)
            nd->workers->submit(gpus[i], [&, i] {
                run(i);
                std::lock_guard<std::mutex> lk(mu);
                if (--left == 0) cv.notify_one();
            });
        std::unique_lock<std::mutex> lk(mu);
        cv.wait(lk, [&] { return left == 0; });
    }
    for (auto &r : res)
        if (r.rc != RBX_OK) return fail(r.rc, r.msg);
    return RBX_OK;
}

extern "C" {

int rbx_node_init(int n_gpus, const int *devices, rbx_node **out) {
    if (!out || n_gpus < 1 || n_gpus > 16384) return fail(RBX_E_ILLEGAL_ARGUMENT, "n_gpus must be in [1, 16384]");
    // replica syncs and cross-GPU HLL inputs are peer copies over xGMI
    for (int i = 0; i < n_gpus; ++i)
        for (int j = 0; j < n_gpus; ++j)
            (void)rbx_enable_peer_access(devices ? devices[i] : i, devices ? devices[j] : j);
    auto *nd = new rbx_node();
    nd->fail_adds.reset(new std::atomic<int>[n_gpus]);
    for (int i = 0; i < n_gpus; ++i) nd->fail_adds[i] = 0;
    for (int i = 0; i < n_gpus; ++i) {
        rbx_ctx *c = nullptr;
        const int rc = rbx_init(devices ? devices[i] : i, &c);
        if (rc != RBX_OK) {
            const std::string msg = rbx_last_error();
            for (rbx_ctx *p : nd->ctx) rbx_shutdown(p);
            delete nd;
            return fail(rc, msg);
        }
        nd->ctx.push_back(c);
    }
    nd->workers = std::make_unique<GpuWorkers>(n_gpus);
    *out = nd;
    return RBX_OK;
}

int rbx_node_shutdown(rbx_node *nd) {
    if (!nd) return RBX_OK;
    nd->blooms.clear();  // closes every cached handle (no batch may run during shutdown)
    nd->workers.reset();  // idle: joined
    int rc = RBX_OK;
    for (rbx_ctx *c : nd->ctx) {
        const int r = rbx_shutdown(c);
        if (rc == RBX_OK) rc = r;
    }
    delete nd;
    return rc;
}

int rbx_node_size(const rbx_node *nd, int *n) {
    if (!nd || !n) return fail(RBX_E_ILLEGAL_ARGUMENT, "NULL argument");
    *n = (int)nd->ctx.size();
    return RBX_OK;
}

int rbx_node_gpu_of(const rbx_node *nd, rbx_name name, int *gpu) {
    if (!nd || !gpu) return fail(RBX_E_ILLEGAL_ARGUMENT, "NULL argument");
    NODE_TRY(check_name(name));
    *gpu = gpu_of(nd, str_of(name));
    return RBX_OK;
}

int rbx_node_ctx(rbx_node *nd, int gpu, rbx_ctx **out) {
    if (!nd || !out || gpu < 0 || gpu >= (int)nd->ctx.size()) return fail(RBX_E_ILLEGAL_ARGUMENT, "bad argument");
    *out = nd->ctx[gpu];
    return RBX_OK;
}

// ---- single objects: routed by slot -------------------------------------------------------------
int rbx_node_bloom_try_init(rbx_node *nd, rbx_name name, int64_t n, double p, int *created) {
    if (!nd) return fail(RBX_E_ILLEGAL_ARGUMENT, "NULL node");
    NODE_TRY(check_name(name));
    return rbx_bloom_try_init_n(nd->ctx[gpu_of(nd, str_of(name))], name, n, p, created);
}

int rbx_node_bloom_read_config(rbx_node *nd, rbx_name name, rbx_bloom_config *out) {
    if (!nd) return fail(RBX_E_ILLEGAL_ARGUMENT, "NULL node");
    NODE_TRY(check_name(name));
    return rbx_bloom_read_config_n(nd->ctx[gpu_of(nd, str_of(name))], name, out);
}

static std::vector<int> all_gpus(const rbx_node *nd) {
    std::vector<int> g(nd->ctx.size());
    for (size_t i = 0; i < g.size(); ++i) g[i] = (int)i;
    return g;
}

// the test hook: true (and one injected failure used up) when GPU g's next add must fail
static bool injected_add_fault(rbx_node *nd, int g) {
    int v = nd->fail_adds[g].load();
    while (v > 0)
        if (nd->fail_adds[g].compare_exchange_weak(v, v - 1)) return true;
    return false;
}

static int node_add_on(rbx_node *nd, int g, rbx_name name, uint64_t size, uint32_t k, const rbx_keys *keys,
                       uint8_t *out_new, uint64_t *out_count) {
    if (injected_add_fault(nd, g)) return fail(RBX_E_DEVICE, "injected add fault (rbx_node_test_fail_adds)");
    return rbx_bloom_add_n(nd->ctx[g], name, size, k, keys, out_new, out_count);
}

// Failure semantics of a replicated add: when the add failed on any replica, the replicas may
// differ (a replica that succeeded holds bits another lacks), so the filter stops being
// replicated.  The caller has already taken the names out of `replicated` (under nd->mu, while
// it still held the barrier shared, so no later batch is routed to a copy); here, with the
// barrier exclusive (no batch still running on a copy), the copies on the non-home GPUs are
// deleted and their cached handles evicted.  The home GPU keeps the filter as its own add left
// it, and the caller returns the add's error.  A name replicated again meanwhile is left alone.
static void drop_copies_locked(rbx_node *nd, const std::string &nm) {
    const int home = gpu_of(nd, nm);
    const std::string cn = config_name(nm);
    const rbx_name both[2] = {name_ref(nm), name_ref(cn)};
    std::vector<HandleRef> evicted;
    {
        std::lock_guard<std::mutex> lk(nd->mu);
        for (int g = 0; g < (int)nd->ctx.size(); ++g) {
            if (g == home) continue;
            auto it = nd->blooms.find(std::make_pair(g, nm));
            if (it != nd->blooms.end()) {
                evicted.push_back(std::move(it->second));
                nd->blooms.erase(it);
            }
        }
    }
    evicted.clear();  // outside the cache lock: closing takes the context lock
    for (int g = 0; g < (int)nd->ctx.size(); ++g) {
        if (g == home) continue;
        int d;
        (void)rbx_del_n(nd->ctx[g], both, 2, &d);
    }
}

static void drop_replicas_after_failure(rbx_node *nd, const std::vector<std::string> &names) {
    std::unique_lock<ReplBarrier> ex(nd->repl_mu);
    for (const std::string &nm : names) {
        {
            std::lock_guard<std::mutex> lk(nd->mu);
            if (nd->replicated.count(nm)) continue;  // replicated again since: its copies are fresh
        }
        drop_copies_locked(nd, nm);
    }
}

// A replicated filter's add is applied to every replica (the same batch in the same order on
// each, so they stay identical); the reply is the home GPU's.  If any replica fails, the filter
// is unreplicated (drop_replicas_after_failure) and the first error (in GPU order) is returned.
int rbx_node_bloom_add(rbx_node *nd, rbx_name name, uint64_t size, uint32_t k, const rbx_keys *keys,
                       uint8_t *out_new, uint64_t *out_count) {
    if (!nd) return fail(RBX_E_ILLEGAL_ARGUMENT, "NULL node");
    NODE_TRY(check_name(name));
    const std::string nm = str_of(name);
    const int home = gpu_of(nd, nm);
    int rc;
    {
        std::shared_lock<ReplBarrier> barrier(nd->repl_mu);
        if (!is_replicated(nd, nm) || nd->ctx.size() == 1)
            return node_add_on(nd, home, name, size, k, keys, out_new, out_count);
        rc = per_gpu(nd, all_gpus(nd), [&](int g) -> int {
            uint64_t cnt = 0;
            return node_add_on(nd, g, name, size, k, keys, g == home ? out_new : nullptr,
                               g == home ? out_count : &cnt);
        });
        if (rc == RBX_OK) return RBX_OK;
        std::lock_guard<std::mutex> lk(nd->mu);
        nd->replicated.erase(nm);
    }
    const std::string msg = rbx_last_error();
    drop_replicas_after_failure(nd, {nm});
    return fail(rc, msg);
}

// A replicated filter's contains is split into one contiguous key range per replica, run
// concurrently; flags land in key order and the count is the sum.
int rbx_node_bloom_contains(rbx_node *nd, rbx_name name, uint64_t size, uint32_t k, const rbx_keys *keys,
                            uint8_t *out_present, uint64_t *out_count) {
    if (!nd) return fail(RBX_E_ILLEGAL_ARGUMENT, "NULL node");
    NODE_TRY(check_name(name));
    const std::string nm = str_of(name);
    const int home = gpu_of(nd, nm);
    const uint64_t N = nd->ctx.size();
    std::shared_lock<ReplBarrier> barrier(nd->repl_mu);
    if (!keys || keys->n < N || !is_replicated(nd, nm) || N == 1)
        return rbx_bloom_contains_n(nd->ctx[home], name, size, k, keys, out_present, out_count);
    if (keys->n && !keys->bytes) return fail(RBX_E_ILLEGAL_ARGUMENT, "keys->bytes is NULL");
    std::vector<uint64_t> cnt(N, 0);
    NODE_TRY(per_gpu(nd, all_gpus(nd), [&](int g) -> int {
        const uint64_t i0 = keys->n * (uint64_t)g / N, i1 = keys->n * (uint64_t)(g + 1) / N;
        rbx_keys sub = keys->offsets ? rbx_keys{keys->bytes, keys->offsets + i0, 0, i1 - i0}
                                     : rbx_keys{keys->bytes + i0 * keys->stride, nullptr, keys->stride, i1 - i0};
        return rbx_bloom_contains_n(nd->ctx[g], name, size, k, &sub, out_present ? out_present + i0 : nullptr,
                                    &cnt[g]);
    }));
    if (out_count) {
        uint64_t t = 0;
        for (uint64_t c : cnt) t += c;
        *out_count = t;
    }
    return RBX_OK;
}

// on != 0: copies the filter (config hash + bitmap) from its home GPU to every other GPU, device
// to device, and from then on routes adds to all replicas and spreads contains over them.
// on == 0: drops the copies (the home GPU keeps the filter).
int rbx_node_bloom_replicate(rbx_node *nd, rbx_name name, int on) {
    if (!nd) return fail(RBX_E_ILLEGAL_ARGUMENT, "NULL node");
    NODE_TRY(check_name(name));
    const std::string nm = str_of(name), cn = config_name(nm);
    const int home = gpu_of(nd, nm);
    std::vector<int> others;
    for (int g = 0; g < (int)nd->ctx.size(); ++g)
        if (g != home) others.push_back(g);
    // exclusive: no add runs between the copy and the routing change, and no contains still runs on
    // a copy when it is deleted
    std::unique_lock<ReplBarrier> ex(nd->repl_mu);
    if (on) {
        rbx_bloom_config cfg;
        NODE_TRY(rbx_bloom_read_config_n(nd->ctx[home], name, &cfg));  // not initialized: ISE
        const int rc = per_gpu(nd, others, [&](int g) -> int { return rbx_bloom_copy_to(nd->ctx[home], nd->ctx[g], name); });
        if (rc != RBX_OK) {  // a partial copy (or re-sync) is not a replica: drop whatever landed
            const std::string msg = rbx_last_error();
            {
                std::lock_guard<std::mutex> lk(nd->mu);
                nd->replicated.erase(nm);
            }
            drop_copies_locked(nd, nm);
            return fail(rc, msg);
        }
        std::lock_guard<std::mutex> lk(nd->mu);
        nd->replicated.insert(nm);
        return RBX_OK;
    }
    {
        std::lock_guard<std::mutex> lk(nd->mu);
        nd->replicated.erase(nm);
    }
    const rbx_name both[2] = {name, name_ref(cn)};
    std::vector<HandleRef> evicted;
    {
        std::lock_guard<std::mutex> lk(nd->mu);
        for (int g : others) {
            auto it = nd->blooms.find(std::make_pair(g, nm));
            if (it != nd->blooms.end()) {
                evicted.push_back(std::move(it->second));
                nd->blooms.erase(it);
            }
        }
    }
    evicted.clear();
    return per_gpu(nd, others, [&](int g) -> int {
        int d;
        return rbx_del_n(nd->ctx[g], both, 2, &d);
    });
}

int rbx_node_test_fail_adds(rbx_node *nd, int gpu, int n) {
    if (!nd || gpu < 0 || gpu >= (int)nd->ctx.size() || n < 0) return fail(RBX_E_ILLEGAL_ARGUMENT, "bad argument");
    nd->fail_adds[gpu] = n;
    return RBX_OK;
}

int rbx_node_bloom_is_replicated(rbx_node *nd, rbx_name name, int *out) {
    if (!nd || !out) return fail(RBX_E_ILLEGAL_ARGUMENT, "NULL argument");
    NODE_TRY(check_name(name));
    *out = is_replicated(nd, str_of(name)) ? 1 : 0;
    return RBX_OK;
}

int rbx_node_bloom_count(rbx_node *nd, rbx_name name, int64_t *out) {
    if (!nd) return fail(RBX_E_ILLEGAL_ARGUMENT, "NULL node");
    NODE_TRY(check_name(name));
    return rbx_bloom_count_n(nd->ctx[gpu_of(nd, str_of(name))], name, out);
}

// the filters a key name can belong to: `key` itself, or every `name` with
// suffixName(name, "config") == key -- "{name}:config", or "name:config" for a name holding a '{'
// (M/RedissonObject.java:77-82; "X" and "{X}" share the config key "{X}:config")
static std::vector<std::string> filters_of(const std::string &key) {
    std::vector<std::string> out{key};
    const std::string sfx = ":config";
    if (key.size() <= sfx.size() || key.compare(key.size() - sfx.size(), sfx.size(), sfx) != 0) return out;
    const std::string plain = key.substr(0, key.size() - sfx.size());
    if (config_name(plain) == key) out.push_back(plain);
    if (plain.size() >= 2 && plain.front() == '{' && plain.back() == '}') {
        const std::string inner = plain.substr(1, plain.size() - 2);
        if (config_name(inner) == key) out.push_back(inner);
    }
    return out;
}

int rbx_node_del(rbx_node *nd, const rbx_name *names, uint32_t n, int *deleted) {
    if (!nd || (n && !names)) return fail(RBX_E_ILLEGAL_ARGUMENT, "NULL argument");
    for (uint32_t i = 0; i < n; ++i) NODE_TRY(check_name(names[i]));
    // Exclusive only when a name (or the filter of a config name) is replicated: then no batch may
    // still run on a copy being deleted.  Otherwise the barrier is held shared, like a batch's, so a
    // DEL of plain names neither waits for the node's in-flight batches nor blocks new ones (ADVICE
    // r04); holding it shared also keeps a replicate() of these names from starting meanwhile.
    std::shared_lock<ReplBarrier> sh(nd->repl_mu);
    bool any = false;
    {
        std::lock_guard<std::mutex> lk(nd->mu);
        if (!nd->replicated.empty())
            for (uint32_t i = 0; i < n && !any; ++i)
                for (const std::string &f : filters_of(str_of(names[i]))) any = any || nd->replicated.count(f) != 0;
    }
    std::unique_lock<ReplBarrier> ex;
    if (any) {  // (the names are re-checked below under nd->mu, one by one)
        sh.unlock();
        ex = std::unique_lock<ReplBarrier>(nd->repl_mu);
    }
    std::vector<std::vector<rbx_name>> by(nd->ctx.size());
    std::vector<std::vector<rbx_name>> replica_keys(nd->ctx.size());  // copies: not counted
    std::deque<std::string> held;  // names the replica deletions add (a config's filter bitmap)
    std::vector<std::string> evict;
    for (uint32_t i = 0; i < n; ++i) {
        const std::string key = str_of(names[i]);
        const int home = gpu_of(nd, key);
        by[home].push_back(names[i]);
        evict.push_back(key);
        std::lock_guard<std::mutex> lk(nd->mu);
        bool repl = false;
        for (const std::string &f : filters_of(key)) {
            if (!nd->replicated.count(f)) continue;
            repl = true;
            if (f == key) continue;
            // the config is gone: the filter is gone, and so are its copies -- the bitmap copies too,
            // whatever the order of the names (a config-only DEL left 512 MiB orphans)
            nd->replicated.erase(f);
            held.push_back(f);
            evict.push_back(f);
            for (size_t g = 0; g < nd->ctx.size(); ++g)
                if ((int)g != home) replica_keys[g].push_back(name_ref(held.back()));
        }
        if (repl)
            for (size_t g = 0; g < nd->ctx.size(); ++g)
                if ((int)g != home) replica_keys[g].push_back(names[i]);
    }
    // the deleted names' cached handles go too (each holds its bitmap until its next call)
    std::vector<HandleRef> evicted;
    {
        std::lock_guard<std::mutex> lk(nd->mu);
        for (const std::string &nm : evict) {
            for (int g = 0; g < (int)nd->ctx.size(); ++g) {  // replicas are cached on every GPU
                auto it = nd->blooms.find(std::make_pair(g, nm));
                if (it != nd->blooms.end()) {
                    evicted.push_back(std::move(it->second));
                    nd->blooms.erase(it);
                }
            }
        }
    }
    evicted.clear();  // outside the cache lock: closing takes the context lock
    int total = 0;
    for (size_t g = 0; g < by.size(); ++g) {
        if (by[g].empty()) continue;
        int d = 0;
        NODE_TRY(rbx_del_n(nd->ctx[g], by[g].data(), (uint32_t)by[g].size(), &d));
        total += d;
    }
    for (size_t g = 0; g < replica_keys.size(); ++g) {
        if (replica_keys[g].empty()) continue;
        int d = 0;
        NODE_TRY(rbx_del_n(nd->ctx[g], replica_keys[g].data(), (uint32_t)replica_keys[g].size(), &d));
    }
    if (deleted) *deleted = total;
    return RBX_OK;
}

// ---- multi-tenant batches -------------------------------------------------------------------------
// One GPU's share of a batch: its segments (in batch order) copied into a host arena.
struct Part {
    std::vector<uint32_t> segs;  // batch segment ids
    std::vector<uint8_t> primary;  // 1: this GPU's reply is the segment's (0: a replica's copy)
    std::vector<uint8_t> bytes;
    std::vector<uint64_t> offs;  // variable-length arenas
    std::vector<uint64_t> seg;   // local segment offsets
    std::vector<uint8_t> out;
    std::vector<uint64_t> cnt;
    rbx_keys keys{};
};

static int validate_batch(const rbx_name *names, uint32_t nseg, const uint64_t *seg, const rbx_keys *keys) {
    if (!names || !seg || !keys || nseg == 0) return fail(RBX_E_ILLEGAL_ARGUMENT, "NULL/empty argument");
    if (keys->n && !keys->bytes) return fail(RBX_E_ILLEGAL_ARGUMENT, "keys->bytes is NULL");
    if (seg[0] != 0 || seg[nseg] != keys->n) return fail(RBX_E_ILLEGAL_ARGUMENT, "segment offsets must span [0, n]");
    for (uint32_t s = 0; s < nseg; ++s) {
        if (seg[s + 1] < seg[s]) return fail(RBX_E_ILLEGAL_ARGUMENT, "segment offsets must be ascending");
        NODE_TRY(check_name(names[s]));
    }
    return RBX_OK;
}

// scatter: every GPU's part of the batch, keys copied in segment order.  Segment s runs on its
// name's home GPU; with `repl` (replicated names, Bloom only) an add segment also runs on every
// other GPU (its reply discarded) and a contains segment runs on GPU (home + s) % N instead.
static void build_parts(const rbx_node *nd, const std::vector<std::string> &sn, const uint64_t *seg,
                        const rbx_keys *keys, std::vector<Part> *parts, const std::vector<uint8_t> *repl = nullptr,
                        bool is_add = false) {
    const int N = (int)nd->ctx.size();
    parts->assign(N, Part{});
    for (uint32_t s = 0; s < sn.size(); ++s) {
        const int home = gpu_of(nd, sn[s]);
        if (!repl || !(*repl)[s]) {
            (*parts)[home].segs.push_back(s);
            (*parts)[home].primary.push_back(1);
        } else if (!is_add) {
            const int g = (home + (int)(s % (uint32_t)N)) % N;
            (*parts)[g].segs.push_back(s);
            (*parts)[g].primary.push_back(1);
        } else {
            for (int g = 0; g < N; ++g) {
                (*parts)[g].segs.push_back(s);
                (*parts)[g].primary.push_back(g == home);
            }
        }
    }
    for (Part &p : *parts) {
        if (p.segs.empty()) continue;
        p.seg.push_back(0);
        if (keys->offsets) p.offs.push_back(0);
        for (uint32_t s : p.segs) {
            const uint64_t i0 = seg[s], i1 = seg[s + 1];
            if (keys->offsets) {
                const uint64_t b0 = keys->offsets[i0], b1 = keys->offsets[i1];
                const uint64_t base = p.bytes.size();
                p.bytes.insert(p.bytes.end(), keys->bytes + b0, keys->bytes + b1);
                for (uint64_t i = i0; i < i1; ++i) p.offs.push_back(base + keys->offsets[i + 1] - b0);
            } else {
                p.bytes.insert(p.bytes.end(), keys->bytes + i0 * keys->stride, keys->bytes + i1 * keys->stride);
            }
            p.seg.push_back(p.seg.back() + (i1 - i0));
        }
        if (p.bytes.empty()) p.bytes.push_back(0);
        p.keys = rbx_keys{p.bytes.data(), keys->offsets ? p.offs.data() : nullptr, keys->stride, p.seg.back()};
        p.out.resize(std::max<uint64_t>(p.seg.back(), 1));
        p.cnt.resize(p.segs.size());
    }
}

static std::vector<int> gpus_with_work(const std::vector<Part> &parts) {
    std::vector<int> g;
    for (size_t i = 0; i < parts.size(); ++i)
        if (!parts[i].segs.empty()) g.push_back((int)i);
    return g;
}

// the cached handle of (gpu, name); refresh = replace it with a freshly opened one (the config was
// re-created with other parameters: a new RBloomFilter object would read the new config)
static int bloom_handle(rbx_node *nd, int g, const std::string &name, bool refresh, HandleRef *out) {
    auto key = std::make_pair(g, name);
    HandleRef old;  // a replaced handle is closed outside the cache lock (when its users are done)
    {
        std::lock_guard<std::mutex> lk(nd->mu);
        auto it = nd->blooms.find(key);
        if (it != nd->blooms.end() && !refresh) {
            *out = it->second;
            return RBX_OK;
        }
    }
    auto ref = std::make_shared<NodeHandle>();
    NODE_TRY(rbx_bloom_open_n(nd->ctx[g], name_ref(name), &ref->h));
    std::map<std::pair<int, std::string>, HandleRef> flushed;
    {
        std::lock_guard<std::mutex> lk(nd->mu);
        if (nd->blooms.size() >= kMaxCachedHandles) flushed.swap(nd->blooms);
        HandleRef &slot = nd->blooms[key];
        old = std::move(slot);
        slot = ref;
    }
    *out = ref;
    return RBX_OK;
}

static int bloom_multi(rbx_node *nd, const rbx_name *names, uint32_t nseg, const uint64_t *seg, const rbx_keys *keys,
                       uint8_t *out, uint64_t *counts, bool is_add) {
    if (!nd) return fail(RBX_E_ILLEGAL_ARGUMENT, "NULL node");
    NODE_TRY(validate_batch(names, nseg, seg, keys));
    std::vector<std::string> sn(nseg);
    for (uint32_t s = 0; s < nseg; ++s) sn[s] = str_of(names[s]);
    std::vector<uint8_t> repl(nseg, 0);
    std::vector<Part> parts;
    std::vector<int> gpus;
    std::vector<std::string> unreplicated;  // replicated names of a failed add
    int rc;
    {
        std::shared_lock<ReplBarrier> barrier(nd->repl_mu);
        {
            std::lock_guard<std::mutex> lk(nd->mu);
            if (!nd->replicated.empty())
                for (uint32_t s = 0; s < nseg; ++s) repl[s] = nd->replicated.count(sn[s]) != 0;
        }
        build_parts(nd, sn, seg, keys, &parts, &repl, is_add);
        gpus = gpus_with_work(parts);
        rc = per_gpu(nd, gpus, [&](int g) -> int {
            Part &p = parts[g];
            if (is_add && injected_add_fault(nd, g)) return fail(RBX_E_DEVICE, "injected add fault (rbx_node_test_fail_adds)");
            for (int attempt = 0;; ++attempt) {
                std::vector<HandleRef> refs(p.segs.size());  // held for the batch
                std::vector<rbx_bloom *> hs(p.segs.size());
                for (size_t j = 0; j < p.segs.size(); ++j) {
                    NODE_TRY(bloom_handle(nd, g, sn[p.segs[j]], attempt > 0, &refs[j]));
                    hs[j] = refs[j]->h;
                }
                const auto fn = is_add ? rbx_bloom_add_multi : rbx_bloom_contains_multi;
                const int r = fn(nd->ctx[g], hs.data(), (uint32_t)hs.size(), p.seg.data(), &p.keys,
                                 out ? p.out.data() : nullptr, p.cnt.data());
                if (r != RBX_E_CONFIG_CHANGED || attempt > 0) return r;
            }
        });
        // a failed add may have reached some replicas of a replicated filter and not others: every
        // replicated filter of the batch stops being replicated (see drop_replicas_after_failure)
        if (rc != RBX_OK && is_add) {
            std::lock_guard<std::mutex> lk(nd->mu);
            for (uint32_t s = 0; s < nseg; ++s)
                if (repl[s] && nd->replicated.erase(sn[s])) unreplicated.push_back(sn[s]);
        }
    }
    if (rc != RBX_OK) {
        const std::string msg = rbx_last_error();
        if (!unreplicated.empty()) drop_replicas_after_failure(nd, unreplicated);
        return fail(rc, msg);
    }
    // gather in segment order
    for (int g : gpus) {
        const Part &p = parts[g];
        for (size_t j = 0; j < p.segs.size(); ++j) {
            if (!p.primary[j]) continue;
            const uint32_t s = p.segs[j];
            if (counts) counts[s] = p.cnt[j];
            if (out) memcpy(out + seg[s], p.out.data() + p.seg[j], seg[s + 1] - seg[s]);
        }
    }
    return RBX_OK;
}

int rbx_node_bloom_contains_multi(rbx_node *nd, const rbx_name *names, uint32_t nseg, const uint64_t *seg_offsets,
                                  const rbx_keys *keys, uint8_t *out_present, uint64_t *out_counts) {
    return bloom_multi(nd, names, nseg, seg_offsets, keys, out_present, out_counts, false);
}

int rbx_node_bloom_add_multi(rbx_node *nd, const rbx_name *names, uint32_t nseg, const uint64_t *seg_offsets,
                             const rbx_keys *keys, uint8_t *out_new, uint64_t *out_counts) {
    return bloom_multi(nd, names, nseg, seg_offsets, keys, out_new, out_counts, true);
}

// ---- HyperLogLog ------------------------------------------------------------------------------
int rbx_node_hll_add_multi(rbx_node *nd, const rbx_name *names, uint32_t nseg, const uint64_t *seg_offsets,
                           const rbx_keys *elements, uint8_t *out_changed) {
    if (!nd) return fail(RBX_E_ILLEGAL_ARGUMENT, "NULL node");
    NODE_TRY(validate_batch(names, nseg, seg_offsets, elements));
    std::vector<std::string> sn(nseg);
    for (uint32_t s = 0; s < nseg; ++s) sn[s] = str_of(names[s]);
    std::vector<Part> parts;
    build_parts(nd, sn, seg_offsets, elements, &parts);
    const std::vector<int> gpus = gpus_with_work(parts);
    const int rc = per_gpu(nd, gpus, [&](int g) -> int {
        Part &p = parts[g];
        std::vector<rbx_name> nm(p.segs.size());
        for (size_t j = 0; j < p.segs.size(); ++j) nm[j] = name_ref(sn[p.segs[j]]);
        return rbx_hll_add_multi_n(nd->ctx[g], nm.data(), (uint32_t)nm.size(), p.seg.data(), &p.keys, p.out.data());
    });
    if (rc != RBX_OK) return rc;
    for (int g : gpus) {
        const Part &p = parts[g];
        for (size_t j = 0; j < p.segs.size(); ++j)
            if (out_changed) out_changed[p.segs[j]] = p.out[j];
    }
    return RBX_OK;
}

// Names of other GPUs' HLLs as temporary keys on GPU `dst`: their registers (with encoding and
// cached cardinality) copied device to device (rbx_hll_copy_to: a peer copy over xGMI, no host
// staging).  Missing keys are skipped (PFCOUNT / PFMERGE ignore them).
static int stage_on(rbx_node *nd, int dst, const std::vector<std::string> &remote, std::vector<std::string> *tmps) {
    for (const std::string &r : remote) {
        int ex = 0;
        const rbx_name rn = name_ref(r);
        const int g = gpu_of(nd, r);
        NODE_TRY(rbx_exists_n(nd->ctx[g], &rn, 1, &ex));
        if (!ex) continue;
        // a binary name no client key is expected to take: NUL-prefixed, unique per call
        std::string t = std::string("\0rbx-node-tmp:", 14) + std::to_string(g_tmp_serial++);
        tmps->push_back(t);
        NODE_TRY(rbx_hll_copy_to(nd->ctx[g], rn, nd->ctx[dst], name_ref(t)));
    }
    return RBX_OK;
}

static void drop(rbx_node *nd, int g, const std::vector<std::string> &tmps) {
    if (tmps.empty()) return;
    std::vector<rbx_name> v;
    for (const auto &t : tmps) v.push_back(name_ref(t));
    int d;
    (void)rbx_del_n(nd->ctx[g], v.data(), (uint32_t)v.size(), &d);
}

int rbx_node_hll_count(rbx_node *nd, const rbx_name *names, uint32_t n, uint64_t *out) {
    if (!nd || !names || !out || n == 0) return fail(RBX_E_ILLEGAL_ARGUMENT, "NULL/empty argument");
    std::vector<std::string> sn(n);
    for (uint32_t i = 0; i < n; ++i) {
        NODE_TRY(check_name(names[i]));
        sn[i] = str_of(names[i]);
    }
    const int g0 = gpu_of(nd, sn[0]);
    std::vector<rbx_name> local;
    std::vector<std::string> remote, tmps;
    for (const auto &s : sn) {
        if (gpu_of(nd, s) == g0) local.push_back(name_ref(s));
        else remote.push_back(s);
    }
    if (remote.empty()) return rbx_hll_count_n(nd->ctx[g0], local.data(), (uint32_t)local.size(), out);
    int rc = stage_on(nd, g0, remote, &tmps);
    if (rc == RBX_OK) {
        for (const auto &t : tmps) local.push_back(name_ref(t));
        // >= 2 names: the union count, never a single key's cached cardinality
        rc = rbx_hll_count_n(nd->ctx[g0], local.data(), (uint32_t)local.size(), out);
    }
    const std::string msg = rc ? rbx_last_error() : "";
    drop(nd, g0, tmps);
    return rc ? fail(rc, msg) : RBX_OK;
}

int rbx_node_hll_merge(rbx_node *nd, rbx_name dest, const rbx_name *srcs, uint32_t nsrc) {
    if (!nd || (nsrc && !srcs)) return fail(RBX_E_ILLEGAL_ARGUMENT, "NULL argument");
    NODE_TRY(check_name(dest));
    const std::string d = str_of(dest);
    const int gd = gpu_of(nd, d);
    std::vector<std::string> sn, remote, tmps;
    for (uint32_t i = 0; i < nsrc; ++i) {
        NODE_TRY(check_name(srcs[i]));
        sn.push_back(str_of(srcs[i]));
    }
    std::vector<rbx_name> local;
    for (const auto &s : sn) {
        if (gpu_of(nd, s) == gd) local.push_back(name_ref(s));
        else remote.push_back(s);
    }
    int rc = stage_on(nd, gd, remote, &tmps);
    if (rc == RBX_OK) {
        for (const auto &t : tmps) local.push_back(name_ref(t));
        rc = rbx_hll_merge_n(nd->ctx[gd], dest, local.data(), (uint32_t)local.size());
    }
    const std::string msg = rc ? rbx_last_error() : "";
    drop(nd, gd, tmps);
    return rc ? fail(rc, msg) : RBX_OK;
}

}  // extern "C"
