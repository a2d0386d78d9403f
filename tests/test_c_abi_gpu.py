"""The C ABI driven from plain C (tests/c/abi_client.c, no Python or torch in the process)
and the RCCL entry points with a single-rank communicator."""
import ctypes as C
import os
import subprocess

import numpy as np
import pytest

from oracle import oracle as O
from redisson_amd import Arena
from redisson_amd import _lib as L

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_plain_c_client():
    exe = os.path.join(ROOT, "tests", "c", "_build", "abi_client")
    assert os.path.exists(exe), "built by __graft_entry__.build() (make -C redisson_amd/csrc)"
    r = subprocess.run([exe], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "all checks passed" in r.stdout


def test_rccl_single_rank_max_allreduce(client, fresh):
    rng = np.random.default_rng(3)
    names = [f"{fresh}-{i}" for i in range(5)]
    refs = []
    hs = []
    for nm in names:
        mat = rng.integers(0, 256, size=(3000, 16), dtype=np.uint8)
        client.getHyperLogLog(nm).addAll(Arena.fixed(mat))
        r = O.hll_new()
        O.hll_pfadd(r, *O.fixed_arena(mat))
        refs.append(r)
        h = C.c_void_p()
        assert L.lib().rbx_hll_open(client.ctx, nm.encode(), 0, C.byref(h)) == 0
        hs.append(h.value)
    uid = (C.c_uint8 * 128)()
    assert L.lib().rbx_rccl_unique_id(uid) == 0
    assert L.lib().rbx_rccl_init(client.ctx, uid, 1, 0) == 0, L.last_error()
    arr = (C.c_void_p * len(hs))(*hs)
    assert L.lib().rbx_hll_allreduce_max(client.ctx, arr, len(hs)) == 0, L.last_error()
    out = np.zeros(len(hs), np.uint64)
    assert L.lib().rbx_hll_count_each_handles(client.ctx, arr, len(hs), out.ctypes.data_as(L.u64p)) == 0
    assert out.tolist() == [O.hll_count(r) for r in refs]
    for nm, r in zip(names, refs):
        d = client.getHyperLogLog(nm).exportDense()
        assert np.array_equal(O.hll_dense_unpack(d[16:]), r)
    for h in hs:
        L.lib().rbx_hll_close(h)


def test_java_ffm_shim_replay():
    """INTEGRATION.md's Java FFM shim, replayed from C: struct offsets of rbx_keys /
    rbx_bloom_config / rbx_name as the Java StructLayouts declare them, and each shim method's
    downcall sequence (tryInit/readConfig/add/contains/count/sizeInMemory/expire/renamenx/delete,
    addAllAsync/mergeWithAsync/countWithAsync with the completion upcall)."""
    exe = os.path.join(ROOT, "tests", "c", "_build", "ffm_replay")
    assert os.path.exists(exe), "built by __graft_entry__.build() (make -C redisson_amd/csrc)"
    r = subprocess.run([exe], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "all checks passed" in r.stdout
