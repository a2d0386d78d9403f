"""Node-level sharding of sketches across GPUs (one rank per GPU).

Redisson routes every command by Redis Cluster slot: slot = CRC16(hashtag or key) % 16384
(M/connection/CRC16.java:51-57, M/cluster/ClusterConnectionManager.java:777-830), and a
filter's bitmap `name` and config `{name}:config` share a slot (RedissonObject.suffixName,
M/RedissonObject.java:77-82).  Here the slot range of one node is split over its GPUs:
GPU = slot * n_gpus // 16384, so a tenant filter lives on exactly one GPU and a batch of
per-tenant commands scatters into per-GPU batches with no data-path collective.

HyperLogLog sets do the opposite: the ELEMENTS are partitioned over GPUs, every GPU holds
partial registers of every HLL, and one RCCL uint8 MAX all-reduce merges them
(rbx_hll_allreduce_max) -- max is associative and idempotent, so the union is exact.
"""
from __future__ import annotations

import numpy as np

from . import _lib as L


def slot_of(name: str | bytes) -> int:
    import ctypes as C

    b = name.encode("utf-8") if isinstance(name, str) else bytes(name)
    buf = (C.c_uint8 * max(1, len(b))).from_buffer_copy(b or b"\0")
    return int(L.lib().rbx_calc_slot(buf, len(b)))


def gpu_of(name: str | bytes, n_gpus: int) -> int:
    return slot_of(name) * n_gpus // 16384


def scatter_segments(names: list[str], seg_offsets: np.ndarray, n_gpus: int):
    """Splits a multi-tenant batch (segment s = keys [off[s], off[s+1]) of tenant names[s])
    into per-GPU batches.  Returns, per GPU: (segment ids, key index array, local segment
    offsets).  Segment order is preserved inside each GPU (per-tenant command order)."""
    seg_offsets = np.asarray(seg_offsets, dtype=np.int64)
    owner = np.array([gpu_of(n, n_gpus) for n in names], dtype=np.int64)
    out = []
    for g in range(n_gpus):
        segs = np.nonzero(owner == g)[0]
        lens = seg_offsets[segs + 1] - seg_offsets[segs]
        local = np.zeros(len(segs) + 1, dtype=np.int64)
        np.cumsum(lens, out=local[1:])
        idx = np.concatenate([np.arange(seg_offsets[s], seg_offsets[s + 1]) for s in segs]) if len(segs) else \
            np.zeros(0, np.int64)
        out.append((segs, idx, local))
    return out


def partition_elements(n: int, n_gpus: int, rank: int) -> tuple[int, int]:
    """Contiguous element range of `rank` for an element-partitioned HLL batch."""
    per = (n + n_gpus - 1) // n_gpus
    lo = min(n, rank * per)
    return lo, min(n, lo + per)
