"""ctypes binding of librbx.so (include/rbx.h).

The product path runs only through this library: there is no CPU fallback.  If the
shared object is missing, importing any engine object raises immediately.
"""
from __future__ import annotations

import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("RBX_LIB_PATH") or os.path.join(_HERE, "librbx.so")  # override: A/B runs only

u8p = C.POINTER(C.c_uint8)
u64p = C.POINTER(C.c_uint64)
u32p = C.POINTER(C.c_uint32)
ullp = C.POINTER(C.c_ulonglong)
vp = C.c_void_p


class RbxKeys(C.Structure):
    """struct rbx_keys {bytes, offsets, stride, n}"""

    _fields_ = [("bytes", vp), ("offsets", vp), ("stride", C.c_uint64), ("n", C.c_uint64)]


class RbxName(C.Structure):
    """struct rbx_name {bytes, len}: a binary-safe key name"""

    _fields_ = [("bytes", vp), ("len", C.c_uint64)]


def names_array(names):
    """(rbx_name[], keep-alive buffers) for a list of bytes/str names."""
    bufs = [n.encode("utf-8") if isinstance(n, str) else bytes(n) for n in names]
    arr = (RbxName * max(len(bufs), 1))()
    keep = []
    for i, b in enumerate(bufs):
        cb = C.create_string_buffer(b, len(b) or 1)
        keep.append(cb)
        arr[i].bytes = C.cast(cb, vp)
        arr[i].len = len(b)
    return arr, keep


def name_struct(name):
    arr, keep = names_array([name])
    return arr[0], keep


class RbxBloomConfig(C.Structure):
    _fields_ = [
        ("size", C.c_int64),
        ("hash_iterations", C.c_uint32),
        ("expected_insertions", C.c_int64),
        ("false_probability", C.c_double),
        ("false_probability_str", C.c_char * 64),
    ]


RBX_OK = 0
RBX_E_ILLEGAL_ARGUMENT = -1
RBX_E_ILLEGAL_STATE = -2
RBX_E_CONFIG_CHANGED = -3
RBX_E_ARITHMETIC = -4
RBX_E_WRONGTYPE = -5
RBX_E_DEVICE = -6
RBX_E_OOM = -7
RBX_E_NO_SUCH_KEY = -8
RBX_E_REDIS = -9
RBX_E_TIMEOUT = -10

# name -> (restype, argtypes); every function declared in include/rbx.h
SIGNATURES = {
    "rbx_abi_version": (C.c_int, []),
    "rbx_last_error": (C.c_char_p, []),
    "rbx_device_count": (C.c_int, [C.POINTER(C.c_int)]),
    "rbx_init": (C.c_int, [C.c_int, C.POINTER(vp)]),
    "rbx_shutdown": (C.c_int, [vp]),
    "rbx_synchronize": (C.c_int, [vp]),
    "rbx_stream": (vp, [vp]),
    "rbx_host_alloc": (C.c_int, [C.c_uint64, C.POINTER(vp)]),
    "rbx_host_free": (C.c_int, [vp]),
    "rbx_set_staging": (C.c_int, [vp, C.c_uint64]),
    "rbx_crc16": (C.c_uint16, [u8p, C.c_size_t]),
    "rbx_calc_slot": (C.c_int, [u8p, C.c_size_t]),
    "rbx_slot_to_gpu": (C.c_int, [C.c_int, C.c_int]),
    "rbx_bloom_optimal_config": (C.c_int, [C.c_int64, C.c_double, C.POINTER(C.c_int64), u32p]),
    "rbx_bloom_try_init": (C.c_int, [vp, C.c_char_p, C.c_int64, C.c_double, C.POINTER(C.c_int)]),
    "rbx_bloom_init_raw": (C.c_int, [vp, C.c_char_p, C.c_uint64, C.c_uint32, C.POINTER(C.c_int)]),
    "rbx_bloom_read_config": (C.c_int, [vp, C.c_char_p, C.POINTER(RbxBloomConfig)]),
    "rbx_bloom_add": (C.c_int, [vp, C.c_char_p, C.c_uint64, C.c_uint32, C.POINTER(RbxKeys), u8p, u64p]),
    "rbx_bloom_contains": (C.c_int, [vp, C.c_char_p, C.c_uint64, C.c_uint32, C.POINTER(RbxKeys), u8p, u64p]),
    "rbx_bloom_count": (C.c_int, [vp, C.c_char_p, C.POINTER(C.c_int64)]),
    "rbx_bloom_bitcount": (C.c_int, [vp, C.c_char_p, u64p]),
    "rbx_bloom_delete": (C.c_int, [vp, C.c_char_p, C.POINTER(C.c_int)]),
    "rbx_bloom_is_exists": (C.c_int, [vp, C.c_char_p, C.POINTER(C.c_int)]),
    "rbx_bloom_rename": (C.c_int, [vp, C.c_char_p, C.c_char_p]),
    "rbx_bloom_renamenx": (C.c_int, [vp, C.c_char_p, C.c_char_p, C.POINTER(C.c_int)]),
    "rbx_pexpire": (C.c_int, [vp, C.POINTER(C.c_char_p), C.c_uint32, C.c_int64, C.c_int, C.c_int, C.POINTER(C.c_int)]),
    "rbx_persist": (C.c_int, [vp, C.POINTER(C.c_char_p), C.c_uint32, C.POINTER(C.c_int)]),
    "rbx_pttl": (C.c_int, [vp, C.c_char_p, C.POINTER(C.c_int64)]),
    "rbx_pexpiretime": (C.c_int, [vp, C.c_char_p, C.POINTER(C.c_int64)]),
    "rbx_bloom_export": (C.c_int, [vp, C.c_char_p, u8p, C.c_uint64, u64p]),
    "rbx_bloom_import": (C.c_int, [vp, C.c_char_p, u8p, C.c_uint64]),
    "rbx_bloom_import_dev": (C.c_int, [vp, C.c_char_p, vp, C.c_uint64, vp]),
    "rbx_bloom_open": (C.c_int, [vp, C.c_char_p, C.POINTER(vp)]),
    "rbx_bloom_close": (C.c_int, [vp]),
    "rbx_bloom_handle_config": (C.c_int, [vp, u64p, u32p]),
    "rbx_bloom_contains_dev": (C.c_int, [vp, vp, C.POINTER(RbxKeys), vp, vp, vp]),
    "rbx_bloom_add_dev": (C.c_int, [vp, vp, C.POINTER(RbxKeys), vp, vp, vp]),
    "rbx_bloom_contains_multi_dev": (C.c_int, [vp, C.POINTER(vp), C.c_uint32, vp, C.POINTER(RbxKeys), vp, vp, vp]),
    "rbx_bloom_add_multi_dev": (C.c_int, [vp, C.POINTER(vp), C.c_uint32, vp, C.POINTER(RbxKeys), vp, vp, vp]),
    "rbx_bloom_contains_multi": (C.c_int, [vp, C.POINTER(vp), C.c_uint32, u64p, C.POINTER(RbxKeys), u8p, u64p]),
    "rbx_bloom_add_multi": (C.c_int, [vp, C.POINTER(vp), C.c_uint32, u64p, C.POINTER(RbxKeys), u8p, u64p]),
    "rbx_bloom_stream_dev": (C.c_int, [vp, C.POINTER(vp), C.c_uint32, vp, vp, C.POINTER(RbxKeys), vp, vp, vp]),
    "rbx_bloom_stream": (C.c_int, [vp, C.POINTER(vp), C.c_uint32, u32p, u8p, C.POINTER(RbxKeys), u8p, u64p]),
    "rbx_hll_add": (C.c_int, [vp, C.c_char_p, C.POINTER(RbxKeys), C.POINTER(C.c_int)]),
    "rbx_hll_add_multi": (C.c_int, [vp, C.POINTER(C.c_char_p), C.c_uint32, u64p, C.POINTER(RbxKeys), u8p]),
    "rbx_hll_count": (C.c_int, [vp, C.POINTER(C.c_char_p), C.c_uint32, u64p]),
    "rbx_hll_count_each": (C.c_int, [vp, C.POINTER(C.c_char_p), C.c_uint32, u64p]),
    "rbx_hll_merge": (C.c_int, [vp, C.c_char_p, C.POINTER(C.c_char_p), C.c_uint32]),
    "rbx_hll_export": (C.c_int, [vp, C.c_char_p, u8p, C.c_uint64, u64p]),
    "rbx_hll_import": (C.c_int, [vp, C.c_char_p, u8p, C.c_uint64]),
    "rbx_hll_export_enc": (C.c_int, [vp, C.c_char_p, C.c_int, u8p, C.c_uint64, u64p]),
    "rbx_hll_delete": (C.c_int, [vp, C.c_char_p, C.POINTER(C.c_int)]),
    "rbx_hll_exists": (C.c_int, [vp, C.c_char_p, C.POINTER(C.c_int)]),
    "rbx_hll_open": (C.c_int, [vp, C.c_char_p, C.c_int, C.POINTER(vp)]),
    "rbx_hll_close": (C.c_int, [vp]),
    "rbx_hll_registers_dev": (C.c_int, [vp, C.POINTER(vp)]),
    "rbx_hll_add_multi_dev": (C.c_int, [vp, C.POINTER(vp), C.c_uint32, vp, u64p, C.POINTER(RbxKeys), vp, vp]),
    "rbx_hll_count_each_handles": (C.c_int, [vp, C.POINTER(vp), C.c_uint32, u64p]),
    "rbx_rccl_unique_id": (C.c_int, [u8p]),
    "rbx_rccl_init": (C.c_int, [vp, u8p, C.c_int, C.c_int]),
    "rbx_hll_allreduce_max": (C.c_int, [vp, C.POINTER(vp), C.c_uint32]),
    "rbx_rccl_info": (C.c_int, [vp, C.POINTER(C.c_int), C.POINTER(C.c_int)]),
    # asynchronous calls (rbx_future)
    "rbx_future_wait": (C.c_int, [vp, C.c_int64, C.POINTER(C.c_int)]),
    "rbx_future_done": (C.c_int, [vp, C.POINTER(C.c_int)]),
    "rbx_future_free": (C.c_int, [vp]),
    "rbx_bloom_add_async": (C.c_int, [vp, C.c_char_p, C.c_uint64, C.c_uint32, C.POINTER(RbxKeys), vp, vp, vp, vp,
                                      C.POINTER(vp)]),
    "rbx_bloom_contains_async": (C.c_int, [vp, C.c_char_p, C.c_uint64, C.c_uint32, C.POINTER(RbxKeys), vp, vp, vp,
                                           vp, C.POINTER(vp)]),
    "rbx_hll_add_async": (C.c_int, [vp, C.c_char_p, C.POINTER(RbxKeys), vp, vp, vp, C.POINTER(vp)]),
    "rbx_hll_add_multi_async": (C.c_int, [vp, C.POINTER(C.c_char_p), C.c_uint32, u64p, C.POINTER(RbxKeys), vp, vp,
                                          vp, C.POINTER(vp)]),
    "rbx_hll_count_async": (C.c_int, [vp, C.POINTER(C.c_char_p), C.c_uint32, vp, vp, vp, C.POINTER(vp)]),
    "rbx_hll_merge_async": (C.c_int, [vp, C.c_char_p, C.POINTER(C.c_char_p), C.c_uint32, vp, vp, C.POINTER(vp)]),
    # one process over the GPUs of a node (rbx_node)
    "rbx_node_init": (C.c_int, [C.c_int, C.POINTER(C.c_int), C.POINTER(vp)]),
    "rbx_node_shutdown": (C.c_int, [vp]),
    "rbx_node_size": (C.c_int, [vp, C.POINTER(C.c_int)]),
    "rbx_node_gpu_of": (C.c_int, [vp, RbxName, C.POINTER(C.c_int)]),
    "rbx_node_ctx": (C.c_int, [vp, C.c_int, C.POINTER(vp)]),
    "rbx_node_bloom_try_init": (C.c_int, [vp, RbxName, C.c_int64, C.c_double, C.POINTER(C.c_int)]),
    "rbx_node_bloom_read_config": (C.c_int, [vp, RbxName, C.POINTER(RbxBloomConfig)]),
    "rbx_node_bloom_add": (C.c_int, [vp, RbxName, C.c_uint64, C.c_uint32, C.POINTER(RbxKeys), u8p, u64p]),
    "rbx_node_bloom_contains": (C.c_int, [vp, RbxName, C.c_uint64, C.c_uint32, C.POINTER(RbxKeys), u8p, u64p]),
    "rbx_node_bloom_count": (C.c_int, [vp, RbxName, C.POINTER(C.c_int64)]),
    "rbx_node_del": (C.c_int, [vp, C.POINTER(RbxName), C.c_uint32, C.POINTER(C.c_int)]),
    "rbx_node_bloom_contains_multi": (C.c_int, [vp, C.POINTER(RbxName), C.c_uint32, u64p, C.POINTER(RbxKeys), u8p,
                                                u64p]),
    "rbx_node_bloom_add_multi": (C.c_int, [vp, C.POINTER(RbxName), C.c_uint32, u64p, C.POINTER(RbxKeys), u8p, u64p]),
    "rbx_node_hll_add_multi": (C.c_int, [vp, C.POINTER(RbxName), C.c_uint32, u64p, C.POINTER(RbxKeys), u8p]),
    "rbx_node_hll_count": (C.c_int, [vp, C.POINTER(RbxName), C.c_uint32, u64p]),
    "rbx_node_hll_merge": (C.c_int, [vp, RbxName, C.POINTER(RbxName), C.c_uint32]),
    "rbx_node_bloom_replicate": (C.c_int, [vp, RbxName, C.c_int]),
    "rbx_node_bloom_is_replicated": (C.c_int, [vp, RbxName, C.POINTER(C.c_int)]),
    "rbx_node_test_fail_adds": (C.c_int, [vp, C.c_int, C.c_int]),
    # replicas
    "rbx_bloom_digest": (C.c_int, [vp, C.c_char_p, u64p]),
    "rbx_bloom_digest_n": (C.c_int, [vp, RbxName, u64p]),
    "rbx_bloom_copy_to": (C.c_int, [vp, vp, RbxName]),
    "rbx_hll_copy_to": (C.c_int, [vp, RbxName, vp, RbxName]),
    "rbx_enable_peer_access": (C.c_int, [C.c_int, C.c_int]),
    "rbx_bench_slice_probe": (C.c_int, [vp, vp, C.c_uint64, C.c_uint32, vp, C.c_uint64, C.c_uint, vp, vp]),
    "rbx_bench_stream_read": (C.c_int, [vp, vp, C.c_uint64, vp, vp]),
    "rbx_bench_add_stamps": (C.c_int, [vp, vp, C.c_uint32]),
    "rbx_bench_stream_write": (C.c_int, [vp, vp, C.c_uint64, vp]),
    "rbx_bench_gather_segments": (C.c_int, [vp, vp, C.c_uint64, C.c_uint64, C.c_uint64, C.c_uint64, vp, vp]),
    # binary names (rbx_name)
    "rbx_bloom_try_init_n": (C.c_int, [vp, RbxName, C.c_int64, C.c_double, C.POINTER(C.c_int)]),
    "rbx_bloom_read_config_n": (C.c_int, [vp, RbxName, C.POINTER(RbxBloomConfig)]),
    "rbx_bloom_add_n": (C.c_int, [vp, RbxName, C.c_uint64, C.c_uint32, C.POINTER(RbxKeys), u8p, u64p]),
    "rbx_bloom_contains_n": (C.c_int, [vp, RbxName, C.c_uint64, C.c_uint32, C.POINTER(RbxKeys), u8p, u64p]),
    "rbx_bloom_count_n": (C.c_int, [vp, RbxName, C.POINTER(C.c_int64)]),
    "rbx_bloom_open_n": (C.c_int, [vp, RbxName, C.POINTER(vp)]),
    "rbx_del_n": (C.c_int, [vp, C.POINTER(RbxName), C.c_uint32, C.POINTER(C.c_int)]),
    "rbx_memory_usage_n": (C.c_int, [vp, C.POINTER(RbxName), C.c_uint32, u64p]),
    "rbx_bloom_size_in_memory": (C.c_int, [vp, C.c_char_p, u64p]),
    "rbx_exists_n": (C.c_int, [vp, C.POINTER(RbxName), C.c_uint32, C.POINTER(C.c_int)]),
    "rbx_pexpire_n": (C.c_int, [vp, C.POINTER(RbxName), C.c_uint32, C.c_int64, C.c_int, C.c_int, C.POINTER(C.c_int)]),
    "rbx_hll_add_multi_n": (C.c_int, [vp, C.POINTER(RbxName), C.c_uint32, u64p, C.POINTER(RbxKeys), u8p]),
    "rbx_hll_count_n": (C.c_int, [vp, C.POINTER(RbxName), C.c_uint32, u64p]),
    "rbx_hll_merge_n": (C.c_int, [vp, RbxName, C.POINTER(RbxName), C.c_uint32]),
    "rbx_hll_export_enc_n": (C.c_int, [vp, RbxName, C.c_int, u8p, C.c_uint64, u64p]),
    "rbx_hll_import_n": (C.c_int, [vp, RbxName, u8p, C.c_uint64]),
    "rbx_hll_open_n": (C.c_int, [vp, RbxName, C.c_int, C.POINTER(vp)]),
    "rbx_hll_pack_registers": (C.c_int, [vp, C.POINTER(vp), C.c_uint32, vp, vp]),
    "rbx_hll_unpack_max_registers": (C.c_int, [vp, C.POINTER(vp), C.c_uint32, vp, vp]),
    "rbx_bench_gather": (C.c_int, [vp, vp, C.c_uint64, C.c_uint64, C.c_uint32, vp, vp]),
    "rbx_tune": (C.c_int, [C.c_char_p, C.c_int]),
    "rbx_bench_stream_geometry": (C.c_int, [vp, u64p]),
    "rbx_bench_gather_regions": (C.c_int, [vp, vp, C.c_uint64, C.c_uint64, C.c_uint64, C.c_uint, vp, vp]),
    # include/rbx_selftest.h
    "rbx_selftest_mod": (C.c_uint64, [C.c_uint64, C.c_uint64]),
    "rbx_selftest_hash128": (None, [u8p, C.c_uint64, u64p]),
    "rbx_selftest_plain_string": (C.c_int, [C.c_double, C.c_char_p, C.c_int]),
}

_lib = None


def _adopt_torch_runtime() -> None:
    """One HIP runtime per process.  PyTorch ships its own libamdhip64.so.7 (same SONAME as
    /opt/rocm/lib's).  Whichever loads first is shared by both, and torch cannot run on a
    runtime other than its own, so when torch is installed it is loaded before librbx.so
    and librbx.so binds to torch's runtime.  (Without torch, /opt/rocm/lib is used.)"""
    import importlib.util

    if os.environ.get("RBX_NO_TORCH_RUNTIME") == "1":
        return
    if importlib.util.find_spec("torch") is not None:
        import torch  # noqa: F401


def lib() -> C.CDLL:
    """Loads librbx.so (built in-tree by __graft_entry__.build()).  Fails loudly."""
    global _lib
    if _lib is None:
        _adopt_torch_runtime()
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(
                f"{LIB_PATH} is missing: build the HIP engine first "
                "(python -c 'import __graft_entry__ as g; g.build()' or make -C redisson_amd/csrc)")
        L = C.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _lib = L
    return _lib


def last_error() -> str:
    m = lib().rbx_last_error()
    return m.decode("utf-8", "replace") if m else ""
