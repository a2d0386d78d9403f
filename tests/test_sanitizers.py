"""Host-only sanitizer runs.  CPU only.

- the C oracle under ASan + UBSan;
- the HIP-free half of librbx.so (redisson_amd/csrc/keyspace.cpp: keyspace, Bloom config rules,
  key timeouts, DEL/EXISTS/RENAME) under ASan + UBSan, and under TSan with 8 threads issuing
  random tryInit / addConfigCheck / rename / renamenx / delete / pexpire / persist / pttl mixes
  on shared names (include/rbx.h: "calls from several threads are safe");
- the node router (redisson_amd/csrc/rbx_node.cpp: slot routing, the per-GPU worker pool, the
  replication barrier, failure semantics of replicated adds) over a host-memory stand-in of the
  per-GPU ABI (tests/c/node_fake_rbx.cpp), under ASan + UBSan and TSan: routing parity against a
  single context, replica identity, injected add failures, replica re-syncs racing adds, and an
  8-thread mix of every node call."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "redisson_amd", "csrc")


def test_oracle_under_asan_ubsan():
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "_build/oracle_asan"], check=True)
    r = subprocess.run([os.path.join(ROOT, "oracle", "_build", "oracle_asan")], capture_output=True, text=True,
                       timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "ok" in r.stdout


@pytest.mark.parametrize("flavor", ["asan", "tsan"])
def test_keyspace_under_sanitizers(flavor):
    target = f"../../tests/c/_build/keyspace_{flavor}"
    subprocess.run(["make", "-s", "-C", CSRC, target], check=True)
    env = dict(os.environ, TSAN_OPTIONS="halt_on_error=1", ASAN_OPTIONS="detect_leaks=1")
    r = subprocess.run([os.path.join(ROOT, "tests", "c", "_build", f"keyspace_{flavor}")], capture_output=True,
                       text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "keyspace_test: ok" in r.stdout
    assert "WARNING" not in r.stderr, r.stderr


@pytest.mark.parametrize("flavor", ["asan", "tsan"])
def test_node_router_under_sanitizers(flavor):
    target = f"../../tests/c/_build/node_{flavor}"
    subprocess.run(["make", "-s", "-C", CSRC, target], check=True)
    env = dict(os.environ, TSAN_OPTIONS="halt_on_error=1", ASAN_OPTIONS="detect_leaks=1")
    r = subprocess.run([os.path.join(ROOT, "tests", "c", "_build", f"node_{flavor}")], capture_output=True,
                       text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "node_test: ok" in r.stdout
    assert "WARNING" not in r.stderr, r.stderr
