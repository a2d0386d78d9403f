// keyspace.h -- the host half of librbx.so that never touches a device: the Redis-like keyspace
// the sketches live in (names, the {name}:config hash, key timeouts, DEL / EXISTS / RENAME), the
// Redisson Bloom config rules (tryInit sizing, addConfigCheck, readConfig, BigDecimal plain
// strings) and the error channel.  It includes no HIP header, so tests/c/keyspace_test.cpp builds
// it with plain g++ under ASan/UBSan and TSan (tests/test_sanitizers.py).
//
// Layout mirrors how Redisson keeps these objects in Redis:
//   name          -> bitmap string (Bloom) | HLL string
//   {name}:config -> Bloom config hash    (RedissonObject.suffixName, M/RedissonObject.java:77-82)
// M/ = /root/reference/redisson/src/main/java/org/redisson/
#pragma once

#include <cstdint>
#include <functional>
#include <memory>
#include <mutex>
#include <string>
#include <unordered_map>
#include <vector>

namespace rbx {

// ---- errors: thread-local message, int codes of include/rbx.h -------------------------------
int fail(int code, const std::string &msg);
const char *last_error_message();

// ---- Java semantics restated (M/RedissonBloomFilter.java) -------------------------------------
std::string java_plain_string(double d);  // BigDecimal.valueOf(d).toPlainString() (:288)
int64_t java_math_round(double a);        // java.lang.Math.round(double)
int64_t java_d2l(double d);               // (long) of a double
// optimalNumOfBits / optimalNumOfHashFunctions (:79-88) plus tryInit's checks (:263-277).  As in
// the reference a negative expectedInsertions yields a negative size, which tryInit accepts.
int optimal_config(int64_t n, double p, uint64_t max_size, int64_t *size, uint32_t *k);
// |size| as the bit count a bitmap index ranges over: Java's `x % size` for x >= 0 equals
// x % |size| when size < 0 (M/RedissonBloomFilter.java:139-151)
inline uint64_t size_bits(int64_t size) { return size < 0 ? 0 - (uint64_t)size : (uint64_t)size; }
constexpr uint64_t kRedissonMaxSize = 2147483647ULL * 2;  // getMaxSize() :257-259
constexpr uint64_t kEngineMaxSize = 1ULL << 32;           // Redis max bit offset + 1

std::string config_name(const std::string &name);  // suffixName(name, "config")

// ---- objects held by the keyspace ------------------------------------------------------------
struct Bitmap;    // a Redis string used with SETBIT/GETBIT (device memory; defined by rbx_api.cpp)
struct HllState;  // a Redis HLL string (device registers; defined by rbx_api.cpp)

struct BloomConfig {
    int64_t size = 0;  // "size" (Java long)
    uint32_t k = 0;    // "hashIterations"
    int64_t expected = 0;
    double fpp = 0;
    std::string fpp_str;
};

enum class KType { Config, Bitmap, Hll };

struct Entry {
    KType type;
    std::shared_ptr<BloomConfig> cfg;
    std::shared_ptr<Bitmap> bm;
    std::shared_ptr<HllState> hll;
    int64_t expire_at = -1;  // unix ms of the key's timeout (PEXPIREAT), -1 = persistent
};

// Every method expects `mu` held by the caller (the context lock of include/rbx.h: calls from
// several threads are serialized on it).  The ks_* functions below take it themselves.
class Keyspace {
public:
    std::recursive_mutex mu;
    uint64_t generation = 1;          // bumped whenever a key is created / removed or re-bound
    int64_t next_expiry = INT64_MAX;  // earliest expire_at in the keyspace (an upper bound)
    std::function<int64_t()> clock;   // unix ms; tests substitute a fake clock

    int64_t now() const;
    // exact-match lookup; a key past its timeout is removed on access (Redis lazy expiry)
    Entry *find(const std::string &k);
    // removes every key past its timeout once the earliest timeout has passed
    void sweep();
    void put(const std::string &k, Entry e) { map_[k] = std::move(e); }
    bool erase(const std::string &k);  // true iff the key existed (and was not expired)
    bool exists(const std::string &k) { return find(k) != nullptr; }
    // RENAME: overwrite the target, keep the timeout; RBX_E_NO_SUCH_KEY for a missing source
    int rename(const std::string &from, const std::string &to);
    void clear() { map_.clear(); }
    size_t size() const { return map_.size(); }

private:
    std::unordered_map<std::string, Entry> map_;
};

// ---- Redisson object semantics on the keyspace (each takes ks.mu) ------------------------
// tryInit(expectedInsertions, falseProbability)  M/RedissonBloomFilter.java:262-300
int ks_bloom_try_init(Keyspace &ks, const std::string &name, int64_t n, double p, int *created);
// engine-level init with a raw (size, k), size in [1, 2^32]
int ks_bloom_init_raw(Keyspace &ks, const std::string &name, uint64_t size, uint32_t k, int *created);
// readConfig() :240-255 (RBX_E_ILLEGAL_STATE when absent, RBX_E_WRONGTYPE for another type)
int ks_get_config(Keyspace &ks, const std::string &name, BloomConfig *out);
// addConfigCheck :207-213: the stored config must equal the caller's cached (size, k)
int ks_config_check(Keyspace &ks, const std::string &name, int64_t size, uint32_t k);
// delete() :230-232 = DEL name {name}:config; isExists :344-347; rename :349-364; renamenx :366-385
int ks_bloom_delete(Keyspace &ks, const std::string &name, int *deleted);
int ks_bloom_is_exists(Keyspace &ks, const std::string &name, int *exists);
int ks_bloom_rename(Keyspace &ks, const std::string &name, const std::string &new_name);
int ks_bloom_renamenx(Keyspace &ks, const std::string &name, const std::string &new_name, int *renamed);
// DEL / EXISTS over any keys (Redis semantics: counts)
int ks_del(Keyspace &ks, const std::vector<std::string> &names, int *deleted);
int ks_exists(Keyspace &ks, const std::vector<std::string> &names, int *count);
// RExpirable (M/RedissonExpirable.java:53-251): PEXPIRE/PEXPIREAT with NX/XX/GT/LT, PERSIST,
// PTTL, PEXPIRETIME
int ks_pexpire(Keyspace &ks, const std::vector<std::string> &names, int64_t when_ms, int absolute, int cond,
               int *result);
int ks_persist(Keyspace &ks, const std::vector<std::string> &names, int *result);
int ks_pttl(Keyspace &ks, const std::string &name, int64_t *out);
int ks_pexpiretime(Keyspace &ks, const std::string &name, int64_t *out);

// ---- cluster slots: M/connection/CRC16.java:25-57, M/cluster/ClusterConnectionManager.java:777-830
uint16_t crc16(const uint8_t *bytes, size_t len);
int calc_slot(const uint8_t *key, size_t len);
int slot_to_gpu(int slot, int n_gpus);

}  // namespace rbx
