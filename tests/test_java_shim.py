"""The Java drop-in (java/src/main/java/org/redisson/) against the C ABI, without a
JDK: every native symbol the shim binds is declared in include/rbx.h and exported by librbx.so; the
struct offsets it hard-codes (Rbx.java KEYS_* / CONFIG_* / NAME_*) equal the C compiler's (static
asserts compiled with gcc here; tests/c/ffm_replay.c checks the same macros at run time on the GPU);
every method of the reference interfaces is implemented.  CPU only."""
import glob
import os
import re
import subprocess
import sys

from redisson_amd import _lib as L

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
JAVA = os.path.join(ROOT, "java", "src", "main", "java", "org", "redisson")
sys.path.insert(0, os.path.join(ROOT, "tests", "c"))
import java_layout  # noqa: E402

from test_abi import declared_symbols  # noqa: E402


def java_sources():
    return {os.path.basename(p): open(p).read() for p in glob.glob(os.path.join(JAVA, "*.java"))}


def test_sources_present_in_package_org_redisson():
    src = java_sources()
    assert set(src) >= {"Rbx.java", "GpuExpirable.java", "GpuBloomFilter.java", "GpuHyperLogLog.java",
                        "GpuRedisson.java"}
    for name, text in src.items():
        # RedissonExpirable and its constructors are package-private (M/RedissonExpirable.java:37-45)
        assert text.startswith("package org.redisson;"), name
        cls = name[:-5]
        assert re.search(rf"\b(class|interface)\s+{cls}\b", text), name
    assert os.path.exists(os.path.join(ROOT, "java", "pom.xml"))


def test_every_bound_symbol_is_declared_and_exported():
    bound = set()
    for text in java_sources().values():
        bound |= set(re.findall(r'h\("(rbx_[a-z0-9_]+)"', text))
    assert len(bound) >= 25
    assert bound <= declared_symbols(), sorted(bound - declared_symbols())
    lib = L.lib()
    assert all(hasattr(lib, s) for s in bound)


def test_struct_offsets_match_the_c_declarations(tmp_path):
    c = java_layout.constants()
    assert {"KEYS_SIZE", "KEYS_N", "CONFIG_SIZE", "CONFIG_K", "CONFIG_FPP_STR", "NAME_SIZE", "NAME_LEN"} <= set(c)
    hdr = tmp_path / "rbx_java_layout.h"
    java_layout.main(str(hdr))
    src = tmp_path / "layout.c"
    src.write_text("""#include <stddef.h>
#include "rbx.h"
#include "rbx_java_layout.h"
_Static_assert(sizeof(rbx_keys) == RBX_JAVA_KEYS_SIZE, "keys");
_Static_assert(offsetof(rbx_keys, bytes) == RBX_JAVA_KEYS_BYTES, "keys.bytes");
_Static_assert(offsetof(rbx_keys, offsets) == RBX_JAVA_KEYS_OFFSETS, "keys.offsets");
_Static_assert(offsetof(rbx_keys, stride) == RBX_JAVA_KEYS_STRIDE, "keys.stride");
_Static_assert(offsetof(rbx_keys, n) == RBX_JAVA_KEYS_N, "keys.n");
_Static_assert(sizeof(rbx_bloom_config) == RBX_JAVA_CONFIG_SIZE, "config");
_Static_assert(offsetof(rbx_bloom_config, size) == RBX_JAVA_CONFIG_SIZE_BITS, "config.size");
_Static_assert(offsetof(rbx_bloom_config, hash_iterations) == RBX_JAVA_CONFIG_K, "config.k");
_Static_assert(offsetof(rbx_bloom_config, expected_insertions) == RBX_JAVA_CONFIG_EXPECTED, "config.expected");
_Static_assert(offsetof(rbx_bloom_config, false_probability) == RBX_JAVA_CONFIG_FPP, "config.fpp");
_Static_assert(offsetof(rbx_bloom_config, false_probability_str) == RBX_JAVA_CONFIG_FPP_STR, "config.fpp_str");
_Static_assert(sizeof(rbx_name) == RBX_JAVA_NAME_SIZE, "name");
_Static_assert(offsetof(rbx_name, bytes) == RBX_JAVA_NAME_BYTES, "name.bytes");
_Static_assert(offsetof(rbx_name, len) == RBX_JAVA_NAME_LEN, "name.len");
int main(void) { return 0; }
""")
    r = subprocess.run(["gcc", "-std=c11", "-fsyntax-only", "-I", os.path.join(ROOT, "include"), "-I", str(tmp_path),
                        str(src)], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr


# every abstract method of M/api/RBloomFilter.java:27-113, M/api/RHyperLogLog.java:27-68 and
# M/api/RHyperLogLogAsync.java:37-70
BLOOM = ["add(T object)", "add(Collection<T> objects)", "contains(T object)", "contains(Collection<T> objects)",
         "tryInit(long expectedInsertions, double falseProbability)", "getExpectedInsertions()",
         "getFalseProbability()", "getSize()", "getHashIterations()", "count()"]
HLL = ["add(V obj)", "addAll(Collection<V> objects)", "count()", "countWith(String... otherLogNames)",
       "mergeWith(String... otherLogNames)", "addAsync(V obj)", "addAllAsync(Collection<V> objects)", "countAsync()",
       "countWithAsync(String... otherLogNames)", "mergeWithAsync(String... otherLogNames)"]
# the RObject / RExpirable methods the reference's RedissonBloomFilter overrides (:230-385), shared by both
LIFECYCLE = ["deleteAsync()", "isExistsAsync()", "sizeInMemoryAsync()", "renameAsync(String newName)",
             "renamenxAsync(String newName)", "clearExpireAsync()", "remainTimeToLiveAsync()", "getExpireTimeAsync()",
             "expireAsync(long ttl, TimeUnit unit, String param, String... keys)",
             "expireAtAsync(long timestamp, String param, String... keys)"]


def test_interface_methods_implemented():
    src = java_sources()
    for cls, methods in (("GpuBloomFilter.java", BLOOM), ("GpuHyperLogLog.java", HLL),
                         ("GpuExpirable.java", LIFECYCLE)):
        text = re.sub(r"\s+", " ", src[cls])
        for m in methods:
            assert re.search(r"@Override (public|protected) [\w<>]+ " + re.escape(m), text), (cls, m)
    assert "extends GpuExpirable implements RBloomFilter<T>" in src["GpuBloomFilter.java"]
    assert "extends GpuExpirable implements RHyperLogLog<V>" in src["GpuHyperLogLog.java"]
    for f in ("getBloomFilter(String name)", "getBloomFilter(String name, Codec codec)", "getHyperLogLog(String name)",
              "getHyperLogLog(String name, Codec codec)"):
        assert f in src["GpuRedisson.java"], f
