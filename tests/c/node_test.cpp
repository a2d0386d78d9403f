// node_test.cpp -- host-only test of the node router (redisson_amd/csrc/rbx_node.cpp) over the
// host-memory stand-in of the per-GPU ABI (node_fake_rbx.cpp), built with g++ under
// -fsanitize=address,undefined and -fsanitize=thread (tests/test_sanitizers.py).
//
//   1. Routing parity: multi-tenant Bloom add / contains batches and single-name calls through a
//      4-GPU node give the same per-key flags and per-segment counts as the same commands applied
//      one by one to a single context (segments run in batch order on each name's home GPU,
//      M/command/CommandBatchService.java:569-604); HLL PFADD batches, PFCOUNT over names on
//      different GPUs and PFMERGE across GPUs agree with the single context.
//   2. Replicas (rbx_node_bloom_replicate): after replicate(on), adds (single and multi-tenant)
//      leave every GPU's copy byte-identical and contains split over the replicas answer as the
//      home does; replicate(off) deletes the copies and keeps the home filter.
//   3. Failure semantics: an add that fails on one replica (rbx_node_test_fail_adds) returns the
//      error, unreplicates the filter and deletes its copies -- never divergent replicas.
//   4. Replica re-sync racing adds (unique keys): a filter still replicated at the end has identical
//      copies -- the replication barrier orders every add before the copy or after the routing change.
//   5. Concurrency: 8 threads mix adds / contains (single, multi-tenant, replicated), replicate
//      on/off, DEL + tryInit, injected add failures and HLL PFADD / PFCOUNT / PFMERGE over shared
//      names; afterwards every filter still marked replicated has identical copies on all GPUs.
// Exit code 0 and "node_test: ok" on stdout = every check passed.
#include <algorithm>
#include <atomic>
#include <cstdio>
#include <cstring>
#include <random>
#include <string>
#include <thread>
#include <vector>

#include "../../include/rbx.h"
#include "../../include/rbx_bench.h"

bool fake_bitmap_bytes(rbx_ctx *c, const std::string &name, std::vector<uint8_t> *out);

static std::atomic<int> g_fails{0};
#define CHECK(c)                                                                             \
    do {                                                                                     \
        if (!(c)) {                                                                          \
            fprintf(stderr, "FAIL %s:%d %s (%s)\n", __FILE__, __LINE__, #c, rbx_last_error()); \
            g_fails++;                                                                       \
        }                                                                                    \
    } while (0)

constexpr int kGpus = 4;
constexpr uint64_t kKeyLen = 16;

static rbx_name nm(const std::string &s) { return rbx_name{(const uint8_t *)s.data(), (uint64_t)s.size()}; }

struct Batch {  // a multi-tenant batch: segment s = keys [seg[s], seg[s+1]) on names[s]
    std::vector<std::string> names;
    std::vector<uint64_t> seg{0};
    std::vector<uint8_t> bytes;
    rbx_keys keys() const { return rbx_keys{bytes.data(), nullptr, kKeyLen, seg.back()}; }
    std::vector<rbx_name> refs() const {
        std::vector<rbx_name> v;
        for (const auto &s : names) v.push_back(nm(s));
        return v;
    }
};

// keys drawn from a small pool, so batches repeat keys (within and across segments)
static Batch make_batch(std::mt19937_64 &rng, const std::vector<std::string> &tenants, int nseg, int maxkeys) {
    Batch b;
    for (int s = 0; s < nseg; ++s) {
        b.names.push_back(tenants[rng() % tenants.size()]);
        const int n = 1 + (int)(rng() % maxkeys);
        for (int i = 0; i < n; ++i) {
            const uint64_t v = rng() % 5000;
            uint8_t key[kKeyLen] = {0};
            memcpy(key, &v, 8);
            b.bytes.insert(b.bytes.end(), key, key + kKeyLen);
        }
        b.seg.push_back(b.seg.back() + n);
    }
    return b;
}

static int home_of(rbx_node *nd, const std::string &s) {
    int g = -1;
    CHECK(rbx_node_gpu_of(nd, nm(s), &g) == RBX_OK);
    return g;
}

static rbx_ctx *ctx_of(rbx_node *nd, int g) {
    rbx_ctx *c = nullptr;
    CHECK(rbx_node_ctx(nd, g, &c) == RBX_OK);
    return c;
}

// the model: the batch's segments applied one by one, in order, to a single context
static void model_multi(rbx_ctx *m, const Batch &b, bool is_add, std::vector<uint8_t> *flags,
                        std::vector<uint64_t> *counts) {
    flags->assign(b.seg.back(), 0);
    counts->assign(b.names.size(), 0);
    for (size_t s = 0; s < b.names.size(); ++s) {
        const uint64_t i0 = b.seg[s], n = b.seg[s + 1] - i0;
        rbx_keys k{b.bytes.data() + i0 * kKeyLen, nullptr, kKeyLen, n};
        const int rc = is_add ? rbx_bloom_add_n(m, nm(b.names[s]), 0, 0, &k, flags->data() + i0, &(*counts)[s])
                              : rbx_bloom_contains_n(m, nm(b.names[s]), 0, 0, &k, flags->data() + i0, &(*counts)[s]);
        CHECK(rc == RBX_OK);
    }
}

static void test_routing_parity() {
    rbx_node *nd = nullptr;
    CHECK(rbx_node_init(kGpus, nullptr, &nd) == RBX_OK);
    rbx_ctx *m = nullptr;
    CHECK(rbx_init(0, &m) == RBX_OK);
    std::vector<std::string> tenants;
    for (int t = 0; t < 40; ++t) tenants.push_back("tenant:" + std::to_string(t));
    tenants.push_back("{user1}:a");
    tenants.push_back("{user1}:b");  // same hashtag: same slot, same GPU
    CHECK(home_of(nd, "{user1}:a") == home_of(nd, "{user1}:b"));
    std::vector<int> used(kGpus, 0);
    for (const auto &t : tenants) {
        int c1 = 0, c2 = 0;
        CHECK(rbx_node_bloom_try_init(nd, nm(t), 1000, 0.01, &c1) == RBX_OK && c1 == 1);
        CHECK(rbx_bloom_try_init_n(m, nm(t), 1000, 0.01, &c2) == RBX_OK && c2 == 1);
        used[home_of(nd, t)]++;
    }
    for (int g = 0; g < kGpus; ++g) CHECK(used[g] > 0);  // the tenants really spread over the GPUs
    std::mt19937_64 rng(7);
    for (int it = 0; it < 30; ++it) {
        const bool is_add = it % 3 != 2;
        const Batch b = make_batch(rng, tenants, 1 + (int)(rng() % 12), 64);
        const auto names = b.refs();
        const rbx_keys k = b.keys();
        std::vector<uint8_t> f(b.seg.back(), 7), mf;
        std::vector<uint64_t> c(b.names.size(), 99), mc;
        const int rc = is_add ? rbx_node_bloom_add_multi(nd, names.data(), (uint32_t)names.size(), b.seg.data(), &k,
                                                         f.data(), c.data())
                              : rbx_node_bloom_contains_multi(nd, names.data(), (uint32_t)names.size(), b.seg.data(),
                                                              &k, f.data(), c.data());
        CHECK(rc == RBX_OK);
        model_multi(m, b, is_add, &mf, &mc);
        CHECK(f == mf);
        CHECK(c == mc);
    }
    // single-name calls
    for (int it = 0; it < 10; ++it) {
        const Batch b = make_batch(rng, tenants, 1, 100);
        const rbx_keys k = b.keys();
        std::vector<uint8_t> f(b.seg.back()), mf;
        std::vector<uint64_t> mc;
        uint64_t c = 0;
        CHECK(rbx_node_bloom_add(nd, nm(b.names[0]), 0, 0, &k, f.data(), &c) == RBX_OK);
        model_multi(m, b, true, &mf, &mc);
        CHECK(f == mf && c == mc[0]);
        CHECK(rbx_node_bloom_contains(nd, nm(b.names[0]), 0, 0, &k, f.data(), &c) == RBX_OK);
        model_multi(m, b, false, &mf, &mc);
        CHECK(f == mf && c == mc[0]);
    }
    // every tenant's bitmap on its home GPU equals the model's
    for (const auto &t : tenants) {
        std::vector<uint8_t> a, b;
        const bool ha = fake_bitmap_bytes(ctx_of(nd, home_of(nd, t)), t, &a), hb = fake_bitmap_bytes(m, t, &b);
        CHECK(ha == hb && a == b);
    }
    // HLL: PFADD batches, PFCOUNT over names of several GPUs, PFMERGE across GPUs
    std::vector<std::string> hlls;
    for (int h = 0; h < 24; ++h) hlls.push_back("hll:" + std::to_string(h));
    for (int it = 0; it < 10; ++it) {
        const Batch b = make_batch(rng, hlls, 1 + (int)(rng() % 10), 200);
        const auto names = b.refs();
        const rbx_keys k = b.keys();
        std::vector<uint8_t> ch(b.names.size()), mch(b.names.size());
        CHECK(rbx_node_hll_add_multi(nd, names.data(), (uint32_t)names.size(), b.seg.data(), &k, ch.data()) == RBX_OK);
        CHECK(rbx_hll_add_multi_n(m, names.data(), (uint32_t)names.size(), b.seg.data(), &k, mch.data()) == RBX_OK);
        CHECK(ch == mch);
    }
    for (int it = 0; it < 10; ++it) {
        std::vector<rbx_name> set;
        for (int j = 0; j < 1 + it; ++j) set.push_back(nm(hlls[rng() % hlls.size()]));
        static const std::string missing = "hll:missing";
        set.push_back(nm(missing));  // PFCOUNT ignores missing keys
        uint64_t a = 1, b = 2;
        CHECK(rbx_node_hll_count(nd, set.data(), (uint32_t)set.size(), &a) == RBX_OK);
        CHECK(rbx_hll_count_n(m, set.data(), (uint32_t)set.size(), &b) == RBX_OK);
        CHECK(a == b);
    }
    {
        std::vector<rbx_name> srcs;
        for (int j = 0; j < 8; ++j) srcs.push_back(nm(hlls[j]));
        CHECK(rbx_node_hll_merge(nd, nm("hll:dest"), srcs.data(), (uint32_t)srcs.size()) == RBX_OK);
        CHECK(rbx_hll_merge_n(m, nm("hll:dest"), srcs.data(), (uint32_t)srcs.size()) == RBX_OK);
        static const std::string dest = "hll:dest";
        const rbx_name d = nm(dest);
        uint64_t a = 1, b = 2;
        CHECK(rbx_node_hll_count(nd, &d, 1, &a) == RBX_OK);
        CHECK(rbx_hll_count_n(m, &d, 1, &b) == RBX_OK);
        CHECK(a == b && a > 0);
        // no temporary key is left behind on any GPU
        for (int g = 0; g < kGpus; ++g) {
            int n = -1;
            CHECK(rbx_exists_n(ctx_of(nd, g), &d, 1, &n) == RBX_OK);
            CHECK(n == (g == home_of(nd, "hll:dest") ? 1 : 0));
        }
    }
    rbx_shutdown(m);
    CHECK(rbx_node_shutdown(nd) == RBX_OK);
}

// true iff `name` has a bitmap on every GPU, all equal to the home GPU's
static bool replicas_identical(rbx_node *nd, const std::string &name) {
    std::vector<uint8_t> home;
    const bool hh = fake_bitmap_bytes(ctx_of(nd, home_of(nd, name)), name, &home);
    for (int g = 0; g < kGpus; ++g) {
        std::vector<uint8_t> v;
        if (fake_bitmap_bytes(ctx_of(nd, g), name, &v) != hh || v != home) return false;
    }
    return true;
}

static int copies_present(rbx_node *nd, const std::string &name) {  // GPUs other than home holding the name
    int n = 0;
    const rbx_name r = nm(name);
    for (int g = 0; g < kGpus; ++g) {
        if (g == home_of(nd, name)) continue;
        int e = 0;
        CHECK(rbx_exists_n(ctx_of(nd, g), &r, 1, &e) == RBX_OK);
        n += e;
    }
    return n;
}

static void test_replicas_and_failures() {
    rbx_node *nd = nullptr;
    CHECK(rbx_node_init(kGpus, nullptr, &nd) == RBX_OK);
    rbx_ctx *m = nullptr;
    CHECK(rbx_init(0, &m) == RBX_OK);
    const std::string big = "big-filter";
    const std::vector<std::string> tenants = {big, "t:1", "t:2", "t:3", "t:4", "t:5"};
    for (const auto &t : tenants) {
        int c = 0;
        CHECK(rbx_node_bloom_try_init(nd, nm(t), 20000, 0.01, &c) == RBX_OK);
        CHECK(rbx_bloom_try_init_n(m, nm(t), 20000, 0.01, &c) == RBX_OK);
    }
    std::mt19937_64 rng(11);
    std::vector<uint8_t> f, mf;
    std::vector<uint64_t> mc;
    uint64_t c = 0;
    Batch b0 = make_batch(rng, {big}, 1, 500);
    rbx_keys k0 = b0.keys();
    f.resize(b0.seg.back());
    CHECK(rbx_node_bloom_add(nd, nm(big), 0, 0, &k0, f.data(), &c) == RBX_OK);
    model_multi(m, b0, true, &mf, &mc);
    int rep = -1;
    CHECK(rbx_node_bloom_replicate(nd, nm(big), 1) == RBX_OK);
    CHECK(rbx_node_bloom_is_replicated(nd, nm(big), &rep) == RBX_OK && rep == 1);
    CHECK(replicas_identical(nd, big));
    CHECK(copies_present(nd, big) == kGpus - 1);
    for (int it = 0; it < 12; ++it) {
        const Batch b = make_batch(rng, tenants, 1 + (int)(rng() % 6), 200);
        const auto names = b.refs();
        const rbx_keys k = b.keys();
        std::vector<uint8_t> fl(b.seg.back());
        std::vector<uint64_t> cn(b.names.size());
        const bool is_add = it % 2 == 0;
        CHECK((is_add ? rbx_node_bloom_add_multi : rbx_node_bloom_contains_multi)(
                  nd, names.data(), (uint32_t)names.size(), b.seg.data(), &k, fl.data(), cn.data()) == RBX_OK);
        model_multi(m, b, is_add, &mf, &mc);
        CHECK(fl == mf && cn == mc);
        CHECK(replicas_identical(nd, big));
    }
    // contains split over the replicas (>= kGpus keys) answers as the model
    const Batch bp = make_batch(rng, {big}, 1, 900);
    const rbx_keys kp = bp.keys();
    f.assign(bp.seg.back(), 9);
    CHECK(rbx_node_bloom_contains(nd, nm(big), 0, 0, &kp, f.data(), &c) == RBX_OK);
    model_multi(m, bp, false, &mf, &mc);
    CHECK(f == mf && c == mc[0]);
    // replicate(off): the copies go, the home filter stays
    CHECK(rbx_node_bloom_replicate(nd, nm(big), 0) == RBX_OK);
    CHECK(rbx_node_bloom_is_replicated(nd, nm(big), &rep) == RBX_OK && rep == 0);
    CHECK(copies_present(nd, big) == 0);
    {
        std::vector<uint8_t> a, b;
        CHECK(fake_bitmap_bytes(ctx_of(nd, home_of(nd, big)), big, &a) && fake_bitmap_bytes(m, big, &b) && a == b);
    }
    // a replicated add failing on one replica (a copy, then the home GPU): the error comes back, the
    // filter is unreplicated and its copies are deleted
    const int home = home_of(nd, big);
    for (int victim : {(home + 1) % kGpus, home}) {
        CHECK(rbx_node_bloom_replicate(nd, nm(big), 1) == RBX_OK);
        CHECK(copies_present(nd, big) == kGpus - 1);
        CHECK(rbx_node_test_fail_adds(nd, victim, 1) == RBX_OK);
        const Batch b = make_batch(rng, {big}, 1, 300);
        const rbx_keys k = b.keys();
        f.resize(b.seg.back());
        CHECK(rbx_node_bloom_add(nd, nm(big), 0, 0, &k, f.data(), &c) == RBX_E_DEVICE);
        CHECK(strstr(rbx_last_error(), "injected") != nullptr);
        CHECK(rbx_node_bloom_is_replicated(nd, nm(big), &rep) == RBX_OK && rep == 0);
        CHECK(copies_present(nd, big) == 0);
        // the home GPU keeps the filter as its own add left it
        rbx_bloom_config cfg;
        CHECK(rbx_node_bloom_read_config(nd, nm(big), &cfg) == RBX_OK);
        if (victim != home) model_multi(m, b, true, &mf, &mc);  // the home add ran
        std::vector<uint8_t> a, mb;
        CHECK(fake_bitmap_bytes(ctx_of(nd, home), big, &a) && fake_bitmap_bytes(m, big, &mb) && a == mb);
    }
    // the same through a multi-tenant batch holding the replicated name
    {
        CHECK(rbx_node_bloom_replicate(nd, nm(big), 1) == RBX_OK);
        CHECK(rbx_node_test_fail_adds(nd, (home + 2) % kGpus, 1) == RBX_OK);
        const Batch b = make_batch(rng, {big, "t:1", "t:2"}, 6, 50);
        const auto names = b.refs();
        const rbx_keys k = b.keys();
        std::vector<uint8_t> fl(b.seg.back());
        std::vector<uint64_t> cn(b.names.size());
        const bool has_big = std::find(b.names.begin(), b.names.end(), big) != b.names.end();
        const int rc = rbx_node_bloom_add_multi(nd, names.data(), (uint32_t)names.size(), b.seg.data(), &k, fl.data(),
                                                cn.data());
        CHECK(rc == RBX_E_DEVICE);  // a replicated add reaches every GPU, the failing one included
        CHECK(rbx_node_bloom_is_replicated(nd, nm(big), &rep) == RBX_OK && rep == (has_big ? 0 : 1));
        CHECK(copies_present(nd, big) == (has_big ? 0 : kGpus - 1));
        if (!has_big) CHECK(replicas_identical(nd, big));
        CHECK(rbx_node_test_fail_adds(nd, (home + 2) % kGpus, 0) == RBX_OK);
    }
    rbx_shutdown(m);
    CHECK(rbx_node_shutdown(nd) == RBX_OK);
}

// replicate(on) re-syncs the copies while adds keep arriving: with the barrier, an add either ran
// before the copy (the copy holds it) or after the routing change (it reaches every replica).  Keys
// are unique per add, so a missed add is never healed by a later one.
static void test_replicate_vs_adds() {
    rbx_node *nd = nullptr;
    CHECK(rbx_node_init(kGpus, nullptr, &nd) == RBX_OK);
    const std::vector<std::string> hot = {"rv:a", "rv:b"};
    for (const auto &t : hot) {
        int c = 0;
        CHECK(rbx_node_bloom_try_init(nd, nm(t), 200000, 0.01, &c) == RBX_OK);
        CHECK(rbx_node_bloom_replicate(nd, nm(t), 1) == RBX_OK);
    }
    std::atomic<int> adders_left{3};
    std::vector<std::thread> th;
    for (int w = 0; w < 3; ++w) {
        th.emplace_back([&, w] {
            for (uint64_t it = 0; it < 600; ++it) {
                uint8_t key[4 * kKeyLen] = {0};
                for (uint64_t j = 0; j < 4; ++j) {
                    const uint64_t v = (uint64_t)w << 40 | it << 4 | j;
                    memcpy(key + j * kKeyLen, &v, 8);
                }
                const rbx_keys k{key, nullptr, kKeyLen, 4};
                uint64_t c = 0;
                CHECK(rbx_node_bloom_add(nd, nm(hot[it % hot.size()]), 0, 0, &k, nullptr, &c) == RBX_OK);
            }
            adders_left--;
        });
    }
    th.emplace_back([&] {
        for (int it = 0; adders_left.load() > 0; ++it)
            CHECK(rbx_node_bloom_replicate(nd, nm(hot[it % hot.size()]), it % 4 != 3) == RBX_OK);
    });
    for (auto &t : th) t.join();
    for (const auto &t : hot) {
        int rep = 0;
        CHECK(rbx_node_bloom_is_replicated(nd, nm(t), &rep) == RBX_OK);
        if (rep) CHECK(replicas_identical(nd, t));
        CHECK(rbx_node_bloom_replicate(nd, nm(t), 1) == RBX_OK);  // a fresh sync is identical
        CHECK(replicas_identical(nd, t));
    }
    CHECK(rbx_node_shutdown(nd) == RBX_OK);
}

static void test_concurrency() {
    rbx_node *nd = nullptr;
    CHECK(rbx_node_init(kGpus, nullptr, &nd) == RBX_OK);
    std::vector<std::string> tenants, hot, hlls;
    for (int t = 0; t < 16; ++t) tenants.push_back("c:" + std::to_string(t));
    for (int t = 0; t < 4; ++t) hot.push_back(tenants[t]);  // replicated on / off as the threads go
    for (int h = 0; h < 8; ++h) hlls.push_back("ch:" + std::to_string(h));
    for (const auto &t : tenants) {
        int c = 0;
        CHECK(rbx_node_bloom_try_init(nd, nm(t), 5000, 0.01, &c) == RBX_OK);
    }
    std::atomic<long> ok{0}, errs{0};
    std::vector<std::thread> th;
    for (int w = 0; w < 8; ++w) {
        th.emplace_back([&, w] {
            std::mt19937_64 rng(100 + w);
            for (int it = 0; it < 250; ++it) {
                const int op = (int)(rng() % 10);
                int rc = RBX_OK;
                if (op <= 2) {  // multi-tenant add / contains
                    const Batch b = make_batch(rng, tenants, 1 + (int)(rng() % 6), 40);
                    const auto names = b.refs();
                    const rbx_keys k = b.keys();
                    std::vector<uint8_t> fl(b.seg.back());
                    std::vector<uint64_t> cn(b.names.size());
                    rc = (op < 2 ? rbx_node_bloom_add_multi : rbx_node_bloom_contains_multi)(
                        nd, names.data(), (uint32_t)names.size(), b.seg.data(), &k, fl.data(), cn.data());
                } else if (op <= 4) {  // single-name add / contains on a hot (maybe replicated) filter
                    const Batch b = make_batch(rng, hot, 1, 60);
                    const rbx_keys k = b.keys();
                    std::vector<uint8_t> fl(b.seg.back());
                    uint64_t c = 0;
                    rc = op == 3 ? rbx_node_bloom_add(nd, nm(b.names[0]), 0, 0, &k, fl.data(), &c)
                                 : rbx_node_bloom_contains(nd, nm(b.names[0]), 0, 0, &k, fl.data(), &c);
                } else if (op == 5) {
                    rc = rbx_node_bloom_replicate(nd, nm(hot[rng() % hot.size()]), (int)(rng() % 3 != 0));
                } else if (op == 6) {  // DEL (name, config or both), then tryInit again
                    const std::string t = tenants[rng() % tenants.size()];
                    const std::string cfg = "{" + t + "}:config";
                    std::vector<std::string> del;
                    const int which = (int)(rng() % 3);
                    if (which != 1) del.push_back(t);
                    if (which != 0) del.push_back(cfg);
                    std::vector<rbx_name> r;
                    for (const auto &s : del) r.push_back(nm(s));
                    int d = 0;
                    rc = rbx_node_del(nd, r.data(), (uint32_t)r.size(), &d);
                    int c = 0;
                    if (rc == RBX_OK) rc = rbx_node_bloom_try_init(nd, nm(t), 5000, 0.01, &c);
                } else if (op == 7) {
                    rc = rbx_node_test_fail_adds(nd, (int)(rng() % kGpus), (int)(rng() % 2));
                } else if (op == 8) {
                    const Batch b = make_batch(rng, hlls, 1 + (int)(rng() % 4), 50);
                    const auto names = b.refs();
                    const rbx_keys k = b.keys();
                    std::vector<uint8_t> ch(b.names.size());
                    rc = rbx_node_hll_add_multi(nd, names.data(), (uint32_t)names.size(), b.seg.data(), &k, ch.data());
                } else {
                    std::vector<rbx_name> set;
                    for (int j = 0; j < 3; ++j) set.push_back(nm(hlls[rng() % hlls.size()]));
                    uint64_t cnt = 0;
                    rc = (rng() & 1) ? rbx_node_hll_count(nd, set.data(), (uint32_t)set.size(), &cnt)
                                     : rbx_node_hll_merge(nd, nm(hlls[rng() % hlls.size()]), set.data(),
                                                          (uint32_t)set.size());
                }
                // injected failures and names caught between DEL and tryInit are expected errors
                if (rc == RBX_OK) ok++;
                else if (rc == RBX_E_DEVICE || rc == RBX_E_ILLEGAL_STATE || rc == RBX_E_CONFIG_CHANGED) errs++;
                else {
                    fprintf(stderr, "FAIL op %d rc %d (%s)\n", op, rc, rbx_last_error());
                    g_fails++;
                }
            }
        });
    }
    for (auto &t : th) t.join();
    CHECK(ok > 1000);
    for (int g = 0; g < kGpus; ++g) CHECK(rbx_node_test_fail_adds(nd, g, 0) == RBX_OK);
    // quiescent: every filter still marked replicated has identical copies on every GPU (and a
    // config on every GPU); one more add through the node keeps them identical
    int nrep = 0;
    for (const auto &t : hot) {
        int rep = 0;
        CHECK(rbx_node_bloom_is_replicated(nd, nm(t), &rep) == RBX_OK);
        if (!rep) continue;
        nrep++;
        CHECK(replicas_identical(nd, t));
        const std::string cfg = "{" + t + "}:config";
        const rbx_name cr = nm(cfg);
        for (int g = 0; g < kGpus; ++g) {
            int e = 0;
            CHECK(rbx_exists_n(ctx_of(nd, g), &cr, 1, &e) == RBX_OK && e == 1);
        }
        std::mt19937_64 rng(5);
        const Batch b = make_batch(rng, {t}, 1, 100);
        const rbx_keys k = b.keys();
        uint64_t c = 0;
        CHECK(rbx_node_bloom_add(nd, nm(t), 0, 0, &k, nullptr, &c) == RBX_OK);
        CHECK(replicas_identical(nd, t));
    }
    printf("concurrency: %ld ok, %ld expected errors, %d filters replicated at the end\n", ok.load(), errs.load(),
           nrep);
    CHECK(rbx_node_shutdown(nd) == RBX_OK);
}

int main() {
    test_routing_parity();
    test_replicas_and_failures();
    test_replicate_vs_adds();
    test_concurrency();
    if (g_fails) {
        printf("node_test: %d failures\n", g_fails.load());
        return 1;
    }
    printf("node_test: ok\n");
    return 0;
}
