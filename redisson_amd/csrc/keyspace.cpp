// keyspace.cpp -- see keyspace.h.  Plain C++17, no HIP: built into librbx.so and, with the
// -fsanitize flags, into tests/c/keyspace_test (tests/test_sanitizers.py).
#include "keyspace.h"

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <ctime>

#include "../../include/rbx.h"

namespace rbx {

// =====================================================================================
// errors
// =====================================================================================
static thread_local std::string g_err;

int fail(int code, const std::string &msg) {
    g_err = msg;
    return code;
}

const char *last_error_message() { return g_err.c_str(); }

static const char *kWrongType = "WRONGTYPE Operation against a key holding the wrong kind of value";

// =====================================================================================
// Java semantics
// =====================================================================================
// Java Double.toString digit selection (shortest round-trip, JDK 19+) and
// BigDecimal.valueOf(d).toPlainString() (M/RedissonBloomFilter.java:288).
std::string java_plain_string(double d) {
    if (d == 0) return std::signbit(d) ? "-0.0" : "0.0";
    char buf[64];
    int prec = 1;
    for (; prec <= 17; ++prec) {
        snprintf(buf, sizeof buf, "%.*e", prec - 1, d);
        if (strtod(buf, nullptr) == d) break;
    }
    // buf = [-]D.DDDDe[+-]XX
    std::string s(buf);
    const bool neg = s[0] == '-';
    if (neg) s = s.substr(1);
    const size_t epos = s.find('e');
    const int exp10 = atoi(s.c_str() + epos + 1);
    std::string digits;
    for (size_t i = 0; i < epos; ++i)
        if (isdigit((unsigned char)s[i])) digits += s[i];
    while (digits.size() > 1 && digits.back() == '0') digits.pop_back();
    // Java: 1e-3 <= |d| < 1e7 -> plain decimal with >= 1 fraction digit; else d.dddE+-n
    std::string out;
    const double ad = std::fabs(d);
    if (ad >= 1e-3 && ad < 1e7) {
        const int ip = exp10 + 1;  // digits before the point
        std::string ipart, fpart;
        if (ip <= 0) {
            ipart = "0";
            fpart = std::string(-ip, '0') + digits;
        } else if ((size_t)ip >= digits.size()) {
            ipart = digits + std::string(ip - digits.size(), '0');
            fpart = "0";
        } else {
            ipart = digits.substr(0, ip);
            fpart = digits.substr(ip);
        }
        out = ipart + "." + fpart;
    } else {
        // BigDecimal("d.dddE+-n"): unscaled = all digits (>= 2 with the forced ".0"),
        // scale = fraction digits - n.  toPlainString writes it without exponent.
        const std::string frac = digits.size() > 1 ? digits.substr(1) : "0";
        const std::string unscaled = digits.substr(0, 1) + frac;
        const long scale = (long)frac.size() - exp10;
        if (scale <= 0) {
            out = unscaled + std::string(-scale, '0');
        } else if ((size_t)scale >= unscaled.size()) {
            out = "0." + std::string(scale - unscaled.size(), '0') + unscaled;
        } else {
            out = unscaled.substr(0, unscaled.size() - scale) + "." + unscaled.substr(unscaled.size() - scale);
        }
    }
    return neg ? "-" + out : out;
}

// java.lang.Math.round(double), JDK 8+ (round half up, saturating)
int64_t java_math_round(double a) {
    uint64_t bits;
    memcpy(&bits, &a, 8);
    const int64_t biased = (int64_t)((bits & 0x7ff0000000000000ULL) >> 52);
    const int64_t shift = (52 - 1 + 1023) - biased;
    if ((shift & -64) == 0) {
        int64_t r = (int64_t)((bits & 0x000fffffffffffffULL) | 0x0010000000000000ULL);
        if ((int64_t)bits < 0) r = -r;
        return ((r >> shift) + 1) >> 1;
    }
    return java_d2l(a);
}

int64_t java_d2l(double d) {
    if (d != d) return 0;
    if (d >= 9223372036854775807.0) return INT64_MAX;
    if (d <= -9223372036854775808.0) return INT64_MIN;
    return (int64_t)d;
}

// RedissonBloomFilter.optimalNumOfBits / optimalNumOfHashFunctions (:79-88) and the tryInit
// validation (:263-277).  `size > getMaxSize()` is the only upper check, so a negative size
// (negative expectedInsertions) passes exactly as in the reference.
int optimal_config(int64_t n, double p, uint64_t max_size, int64_t *size, uint32_t *k) {
    if (p > 1) return fail(RBX_E_ILLEGAL_ARGUMENT, "Bloom filter false probability can't be greater than 1");
    if (p < 0) return fail(RBX_E_ILLEGAL_ARGUMENT, "Bloom filter false probability can't be negative");
    const double pp = p == 0 ? 4.9e-324 : p;  // Double.MIN_VALUE
    volatile double ln2 = std::log(2.0);       // volatile: keep (ln2*ln2) a separate product
    const int64_t neg_n = (int64_t)(0 - (uint64_t)n);  // Java's wrapping -n
    const int64_t s = java_d2l((double)neg_n * std::log(pp) / (ln2 * ln2));
    if (s == 0) return fail(RBX_E_ILLEGAL_ARGUMENT, "Bloom filter calculated size is " + std::to_string(s));
    if (s > 0 && (uint64_t)s > max_size)
        return fail(RBX_E_ILLEGAL_ARGUMENT, "Bloom filter size can't be greater than " + std::to_string(max_size) +
                                                ". But calculated size is " + std::to_string(s));
    const int64_t r = java_math_round((double)s / (double)n * ln2);
    int32_t kk = (int32_t)(uint32_t)(uint64_t)r;  // (int) of a long: the low 32 bits
    if (kk < 1) kk = 1;
    *size = s;
    *k = (uint32_t)kk;
    return RBX_OK;
}

std::string config_name(const std::string &name) {
    if (name.find('{') != std::string::npos) return name + ":config";
    return "{" + name + "}:config";
}

// =====================================================================================
// Keyspace
// =====================================================================================
int64_t Keyspace::now() const {
    if (clock) return clock();
    struct timespec ts;
    clock_gettime(CLOCK_REALTIME, &ts);
    return (int64_t)ts.tv_sec * 1000 + ts.tv_nsec / 1000000;
}

Entry *Keyspace::find(const std::string &k) {
    auto it = map_.find(k);
    if (it == map_.end()) return nullptr;
    if (it->second.expire_at >= 0 && it->second.expire_at <= now()) {
        map_.erase(it);
        generation++;
        return nullptr;
    }
    return &it->second;
}

void Keyspace::sweep() {
    if (next_expiry == INT64_MAX) return;
    const int64_t t_now = now();
    if (t_now < next_expiry) return;
    int64_t next = INT64_MAX;
    for (auto it = map_.begin(); it != map_.end();) {
        const int64_t t = it->second.expire_at;
        if (t >= 0 && t <= t_now) {
            it = map_.erase(it);
            generation++;
            continue;
        }
        if (t >= 0) next = std::min(next, t);
        ++it;
    }
    next_expiry = next;
}

bool Keyspace::erase(const std::string &k) {
    if (!find(k)) return false;
    map_.erase(k);
    generation++;
    return true;
}

int Keyspace::rename(const std::string &from, const std::string &to) {
    Entry *src = find(from);
    if (!src) return fail(RBX_E_NO_SUCH_KEY, "ERR no such key");
    if (from == to) return RBX_OK;
    Entry e = *src;  // RENAME keeps the timeout
    map_.erase(from);
    map_[to] = std::move(e);
    generation++;
    return RBX_OK;
}

// =====================================================================================
// Bloom config (M/RedissonBloomFilter.java)
// =====================================================================================
static int bloom_init_common(Keyspace &ks, const std::string &name, int64_t size, uint32_t k, int64_t expected,
                             double fpp, const std::string &fpp_str, int *created) {
    const std::string cn = config_name(name);
    if (ks.find(cn)) {
        // Lua: assert(size == false and hashIterations == false) fails -> tryInit returns false
        if (created) *created = 0;
        return RBX_OK;
    }
    auto cfg = std::make_shared<BloomConfig>();
    cfg->size = size;
    cfg->k = k;
    cfg->expected = expected;
    cfg->fpp = fpp;
    cfg->fpp_str = fpp_str;
    ks.put(cn, Entry{KType::Config, cfg, nullptr, nullptr});
    if (created) *created = 1;
    return RBX_OK;
}

int ks_bloom_try_init(Keyspace &ks, const std::string &name, int64_t n, double p, int *created) {
    std::lock_guard<std::recursive_mutex> g(ks.mu);
    int64_t size;
    uint32_t k;
    int rc = optimal_config(n, p, kRedissonMaxSize, &size, &k);
    if (rc != RBX_OK) return rc;
    return bloom_init_common(ks, name, size, k, n, p, java_plain_string(p), created);
}

int ks_bloom_init_raw(Keyspace &ks, const std::string &name, uint64_t size, uint32_t k, int *created) {
    if (size == 0 || size > kEngineMaxSize) return fail(RBX_E_ILLEGAL_ARGUMENT, "size must be in [1, 2^32]");
    if (k == 0) return fail(RBX_E_ILLEGAL_ARGUMENT, "k must be >= 1");
    std::lock_guard<std::recursive_mutex> g(ks.mu);
    return bloom_init_common(ks, name, (int64_t)size, k, 0, 0.0, "0.0", created);
}

int ks_get_config(Keyspace &ks, const std::string &name, BloomConfig *out) {
    std::lock_guard<std::recursive_mutex> g(ks.mu);
    Entry *e = ks.find(config_name(name));
    if (!e) return fail(RBX_E_ILLEGAL_STATE, "Bloom filter is not initialized!");
    if (e->type != KType::Config) return fail(RBX_E_WRONGTYPE, kWrongType);
    *out = *e->cfg;
    return RBX_OK;
}

int ks_config_check(Keyspace &ks, const std::string &name, int64_t size, uint32_t k) {
    std::lock_guard<std::recursive_mutex> g(ks.mu);
    Entry *e = ks.find(config_name(name));
    if (!e || e->type != KType::Config || e->cfg->size != size || e->cfg->k != k)
        return fail(RBX_E_CONFIG_CHANGED, "Bloom filter config has been changed");
    return RBX_OK;
}

int ks_bloom_delete(Keyspace &ks, const std::string &name, int *deleted) {
    std::lock_guard<std::recursive_mutex> g(ks.mu);
    int n = (int)ks.erase(name);
    n += (int)ks.erase(config_name(name));
    if (deleted) *deleted = n;
    return RBX_OK;
}

int ks_bloom_is_exists(Keyspace &ks, const std::string &name, int *exists) {
    std::lock_guard<std::recursive_mutex> g(ks.mu);
    *exists = (ks.exists(name) + ks.exists(config_name(name))) > 0;
    return RBX_OK;
}

// renameAsync :349-364 (Lua: rename the bitmap if it exists, then the config)
int ks_bloom_rename(Keyspace &ks, const std::string &name, const std::string &new_name) {
    std::lock_guard<std::recursive_mutex> g(ks.mu);
    if (ks.exists(name)) {
        int rc = ks.rename(name, new_name);
        if (rc != RBX_OK) return rc;
    }
    return ks.rename(config_name(name), config_name(new_name));
}

// renamenxAsync :366-385 (Lua: renamenx bitmap; if 0 return 0; else renamenx config)
int ks_bloom_renamenx(Keyspace &ks, const std::string &name, const std::string &new_name, int *renamed) {
    std::lock_guard<std::recursive_mutex> g(ks.mu);
    if (!ks.exists(name)) return fail(RBX_E_NO_SUCH_KEY, "ERR no such key");
    if (ks.exists(new_name)) {
        if (renamed) *renamed = 0;
        return RBX_OK;
    }
    int rc = ks.rename(name, new_name);
    if (rc != RBX_OK) return rc;
    const std::string cf = config_name(name), ct = config_name(new_name);
    if (!ks.exists(cf)) return fail(RBX_E_NO_SUCH_KEY, "ERR no such key");
    if (ks.exists(ct)) {
        if (renamed) *renamed = 0;
        return RBX_OK;
    }
    rc = ks.rename(cf, ct);
    if (rc != RBX_OK) return rc;
    if (renamed) *renamed = 1;
    return RBX_OK;
}

int ks_del(Keyspace &ks, const std::vector<std::string> &names, int *deleted) {
    std::lock_guard<std::recursive_mutex> g(ks.mu);
    int n = 0;
    for (const auto &k : names) n += (int)ks.erase(k);
    if (deleted) *deleted = n;
    return RBX_OK;
}

int ks_exists(Keyspace &ks, const std::vector<std::string> &names, int *count) {
    std::lock_guard<std::recursive_mutex> g(ks.mu);
    int n = 0;
    for (const auto &k : names) n += (int)ks.exists(k);  // EXISTS counts repeated keys repeatedly
    if (count) *count = n;
    return RBX_OK;
}

// =====================================================================================
// key timeouts (RedissonExpirable, M/RedissonExpirable.java:53-251)
// =====================================================================================
// PEXPIRE / PEXPIREAT over several keys with the Lua fold of expireAsync / expireAtAsync
// (:207-239): result = 1 iff the timeout of any key was set.  Redis 7.2 rules per key: a
// missing key gives 0; cond NX = only without a timeout, XX = only with one, GT / LT = only if
// the new time is later / earlier (a key without a timeout counts as infinite); a time not in
// the future deletes the key (and counts as set).
int ks_pexpire(Keyspace &ks, const std::vector<std::string> &names, int64_t when_ms, int absolute, int cond,
               int *result) {
    if (cond < 0 || cond > 4) return fail(RBX_E_ILLEGAL_ARGUMENT, "bad argument");
    std::lock_guard<std::recursive_mutex> g(ks.mu);
    const int64_t t_now = ks.now();
    const int64_t at = absolute ? when_ms : t_now + when_ms;
    int any = 0;
    for (const auto &name : names) {
        Entry *e = ks.find(name);
        if (!e) continue;
        const int64_t cur = e->expire_at;  // -1: persistent (infinite for GT / LT)
        if (cond == 1 && cur >= 0) continue;
        if (cond == 2 && cur < 0) continue;
        if (cond == 3 && (cur < 0 || at <= cur)) continue;
        if (cond == 4 && cur >= 0 && at >= cur) continue;
        any = 1;
        if (at <= t_now) {
            ks.erase(name);
            continue;
        }
        e->expire_at = at;
        ks.next_expiry = std::min(ks.next_expiry, at);
    }
    if (result) *result = any;
    return RBX_OK;
}

// PERSIST over several keys (clearExpireAsync :241-251): result = 1 iff any timeout was removed
int ks_persist(Keyspace &ks, const std::vector<std::string> &names, int *result) {
    std::lock_guard<std::recursive_mutex> g(ks.mu);
    int any = 0;
    for (const auto &name : names) {
        Entry *e = ks.find(name);
        if (e && e->expire_at >= 0) {
            e->expire_at = -1;
            any = 1;
        }
    }
    if (result) *result = any;
    return RBX_OK;
}

// PTTL (remainTimeToLiveAsync :193-195) and PEXPIRETIME (getExpireTimeAsync :203-205) of one
// key: -2 when the key does not exist, -1 when it has no timeout
int ks_pttl(Keyspace &ks, const std::string &name, int64_t *out) {
    std::lock_guard<std::recursive_mutex> g(ks.mu);
    Entry *e = ks.find(name);
    *out = !e ? -2 : e->expire_at < 0 ? -1 : std::max<int64_t>(0, e->expire_at - ks.now());
    return RBX_OK;
}

int ks_pexpiretime(Keyspace &ks, const std::string &name, int64_t *out) {
    std::lock_guard<std::recursive_mutex> g(ks.mu);
    Entry *e = ks.find(name);
    *out = !e ? -2 : e->expire_at;
    return RBX_OK;
}

// =====================================================================================
// CRC16 / slots
// =====================================================================================
// XMODEM CRC16 (poly 0x1021, init 0): M/connection/CRC16.java:25-57, table built at load.
static uint16_t g_crc_table[256];
static std::once_flag g_crc_once;
static void build_crc_table() {
    for (int i = 0; i < 256; ++i) {
        uint32_t c = (uint32_t)i << 8;
        for (int b = 0; b < 8; ++b) c = (c & 0x8000) ? ((c << 1) ^ 0x1021) : (c << 1);
        g_crc_table[i] = (uint16_t)c;
    }
}

uint16_t crc16(const uint8_t *bytes, size_t len) {
    std::call_once(g_crc_once, build_crc_table);
    uint32_t crc = 0;
    for (size_t i = 0; i < len; ++i) crc = ((crc << 8) ^ g_crc_table[((crc >> 8) ^ bytes[i]) & 0xff]) & 0xffff;
    return (uint16_t)crc;
}

// calcSlot(byte[]) M/cluster/ClusterConnectionManager.java:777-792 (hashtag rules)
int calc_slot(const uint8_t *key, size_t len) {
    if (!key) return 0;
    const void *o = memchr(key, '{', len);
    if (o) {
        const size_t start = (const uint8_t *)o - key;
        const void *cl = memchr(key, '}', len);  // first '}' anywhere (indexOf from 0)
        if (cl) {
            const size_t end = (const uint8_t *)cl - key;
            if (start + 1 < end) return crc16(key + start + 1, end - start - 1) % 16384;
        }
    }
    return crc16(key, len) % 16384;
}

int slot_to_gpu(int slot, int n_gpus) {
    if (n_gpus <= 0 || slot < 0 || slot >= 16384) return 0;
    return (int)((int64_t)slot * n_gpus / 16384);
}

}  // namespace rbx
