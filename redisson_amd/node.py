"""One process over the GPUs of a node (rbx_node_*, include/rbx.h).

Redisson configured for a Redis Cluster routes every command by slot and groups a batch per node
(M/command/CommandBatchService.java:569-604, M/cluster/ClusterConnectionManager.java:777-830).
RedissonNode does the same over GPUs: one engine context per GPU, names routed to
GPU = calc_slot(name) * n_gpus // 16384, multi-tenant batches scattered per GPU, run
concurrently and gathered back in segment order -- all inside librbx.so.

Names may be str (UTF-8) or bytes (binary-safe).
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _lib as L
from .client import _check, _is_collection
from .codec import DEFAULT_CODEC, Codec
from .keys import Arena, _OneKey


class RedissonNode:
    def __init__(self, n_gpus: int, devices: list[int] | None = None):
        self._node = C.c_void_p()
        devs = (C.c_int * n_gpus)(*devices) if devices is not None else None
        _check(L.lib().rbx_node_init(n_gpus, devs, C.byref(self._node)))
        self.n_gpus = n_gpus

    @property
    def node(self):
        if not self._node:
            raise RuntimeError("node has been shut down")
        return self._node

    def gpu_of(self, name) -> int:
        s, keep = L.name_struct(name)
        g = C.c_int()
        _check(L.lib().rbx_node_gpu_of(self.node, s, C.byref(g)))
        return g.value

    def getBloomFilter(self, name, codec: Codec | None = None) -> "NodeBloomFilter":
        return NodeBloomFilter(self, name, codec or DEFAULT_CODEC)

    def getHyperLogLog(self, name, codec: Codec | None = None) -> "NodeHyperLogLog":
        return NodeHyperLogLog(self, name, codec or DEFAULT_CODEC)

    def delete(self, *names) -> int:
        arr, keep = L.names_array(list(names))
        d = C.c_int()
        _check(L.lib().rbx_node_del(self.node, arr, len(names), C.byref(d)))
        return d.value

    def bloom_contains_multi(self, names, seg_offsets, arena: Arena, per_key: bool = False):
        return self._bloom_multi(L.lib().rbx_node_bloom_contains_multi, names, seg_offsets, arena, per_key)

    def bloom_add_multi(self, names, seg_offsets, arena: Arena, per_key: bool = False):
        return self._bloom_multi(L.lib().rbx_node_bloom_add_multi, names, seg_offsets, arena, per_key)

    def _bloom_multi(self, fn, names, seg_offsets, arena, per_key):
        arr, keep = L.names_array(list(names))
        seg = np.ascontiguousarray(seg_offsets, dtype=np.uint64)
        counts = np.zeros(len(names), np.uint64)
        out = np.zeros(max(arena.n, 1), np.uint8) if per_key else None
        _check(fn(self.node, arr, len(names), seg.ctypes.data_as(L.u64p), arena.ptr(),
                  out.ctypes.data_as(L.u8p) if per_key else None, counts.ctypes.data_as(L.u64p)))
        return (counts, out[: arena.n]) if per_key else counts

    def hll_add_multi(self, names, seg_offsets, arena: Arena) -> np.ndarray:
        arr, keep = L.names_array(list(names))
        seg = np.ascontiguousarray(seg_offsets, dtype=np.uint64)
        out = np.zeros(max(len(names), 1), np.uint8)
        _check(L.lib().rbx_node_hll_add_multi(self.node, arr, len(names), seg.ctypes.data_as(L.u64p), arena.ptr(),
                                              out.ctypes.data_as(L.u8p)))
        return out[: len(names)]

    def shutdown(self) -> None:
        if self._node:
            _check(L.lib().rbx_node_shutdown(self._node))
            self._node = C.c_void_p()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.shutdown()


class NodeBloomFilter:
    """RBloomFilter on the GPU that owns the name's slot."""

    def __init__(self, node: RedissonNode, name, codec: Codec):
        self._node, self._name, self._codec = node, name, codec
        self._size = self._k = 0

    def _n(self):
        return L.name_struct(self._name)

    def tryInit(self, expectedInsertions: int, falseProbability: float) -> bool:
        s, keep = self._n()
        created = C.c_int()
        _check(L.lib().rbx_node_bloom_try_init(self._node.node, s, int(expectedInsertions), float(falseProbability),
                                               C.byref(created)))
        self._read_config()
        return bool(created.value)

    def _read_config(self):
        s, keep = self._n()
        cfg = L.RbxBloomConfig()
        _check(L.lib().rbx_node_bloom_read_config(self._node.node, s, C.byref(cfg)))
        self._size, self._k = cfg.size, cfg.hash_iterations

    def getSize(self) -> int:
        self._read_config()
        return int(self._size)

    def getHashIterations(self) -> int:
        self._read_config()
        return int(self._k)

    def _batch(self, fn, objects, flags):
        if self._size == 0:
            self._read_config()
        a = objects if isinstance(objects, (Arena, _OneKey)) else Arena([self._codec.encode(o) for o in objects])
        s, keep = self._n()
        out = np.zeros(max(a.n, 1), np.uint8) if flags else None
        cnt = C.c_uint64()
        _check(fn(self._node.node, s, self._size, self._k, a.ptr(), out.ctypes.data_as(L.u8p) if flags else None,
                  C.byref(cnt)))
        return (int(cnt.value), out[: a.n]) if flags else int(cnt.value)

    def replicate(self, on: bool = True) -> None:
        """Copy the filter to every GPU of the node (adds go to all replicas, contains are spread
        over them) -- or drop the copies (rbx_node_bloom_replicate)."""
        s, keep = self._n()
        _check(L.lib().rbx_node_bloom_replicate(self._node.node, s, 1 if on else 0))

    def isReplicated(self) -> bool:
        s, keep = self._n()
        r = C.c_int()
        _check(L.lib().rbx_node_bloom_is_replicated(self._node.node, s, C.byref(r)))
        return bool(r.value)

    def addEach(self, objects):
        return self._batch(L.lib().rbx_node_bloom_add, objects, True)

    def add(self, objects):
        if isinstance(objects, Arena) or _is_collection(objects):
            return self._batch(L.lib().rbx_node_bloom_add, objects, False)
        return self._batch(L.lib().rbx_node_bloom_add, _OneKey(self._codec.encode(objects)), False) > 0

    def contains(self, objects):
        if isinstance(objects, Arena) or _is_collection(objects):
            return self._batch(L.lib().rbx_node_bloom_contains, objects, False)
        return self._batch(L.lib().rbx_node_bloom_contains, _OneKey(self._codec.encode(objects)), False) > 0

    def containsEach(self, objects):
        return self._batch(L.lib().rbx_node_bloom_contains, objects, True)

    def count(self) -> int:
        s, keep = self._n()
        out = C.c_int64()
        _check(L.lib().rbx_node_bloom_count(self._node.node, s, C.byref(out)))
        return int(out.value)


class NodeHyperLogLog:
    """RHyperLogLog on the GPU that owns the name's slot; countWith / mergeWith across GPUs."""

    def __init__(self, node: RedissonNode, name, codec: Codec):
        self._node, self._name, self._codec = node, name, codec

    def addAll(self, objects) -> bool:
        a = objects if isinstance(objects, Arena) else Arena([self._codec.encode(o) for o in objects])
        return bool(self._node.hll_add_multi([self._name], [0, a.n], a)[0])

    def add(self, obj) -> bool:
        return self.addAll([obj])

    def count(self) -> int:
        return self.countWith()

    def countWith(self, *others) -> int:
        arr, keep = L.names_array([self._name, *others])
        out = C.c_uint64()
        _check(L.lib().rbx_node_hll_count(self._node.node, arr, 1 + len(others), C.byref(out)))
        return int(out.value)

    def mergeWith(self, *others) -> None:
        d, keep_d = L.name_struct(self._name)
        arr, keep = L.names_array(list(others))
        _check(L.lib().rbx_node_hll_merge(self._node.node, d, arr, len(others)))
