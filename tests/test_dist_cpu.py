"""Multi-GPU logic rehearsed on CPU with gloo, world_size 2 (no GPU needed).

- Bloom tenants shard by CRC16 slot with no data-path collective: the per-rank results of a
  scattered multi-tenant batch equal the single-process results.
- HLL sets shard by element; the uint8 MAX all-reduce of the partial registers (what
  rbx_hll_allreduce_max does over RCCL) reproduces the single-process registers and counts.
- bench.py's max/sum-over-ranks aggregation.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import oracle as O
from redisson_amd.sharding import gpu_of, partition_elements, scatter_segments, slot_of


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run(fn, world=2):
    port = _free_port()
    mp.spawn(_entry, args=(world, port, fn), nprocs=world, join=True)


def _entry(rank, world, port, fn):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        fn(rank, world)
    finally:
        dist.destroy_process_group()


def test_slot_sharding_properties():
    names = [f"tenant:{t:06d}" for t in range(20000)]
    for n_gpus in (1, 2, 4, 8):
        owners = np.array([gpu_of(n, n_gpus) for n in names])
        assert owners.min() >= 0 and owners.max() < n_gpus
        counts = np.bincount(owners, minlength=n_gpus)
        assert counts.min() > 0.8 * len(names) / n_gpus
    # a filter's bitmap and its {name}:config share a slot, hence a GPU
    for n in names[:200]:
        assert slot_of(n) == slot_of("{" + n + "}:config")


def test_scatter_segments_is_a_partition():
    rng = np.random.default_rng(0)
    names = [f"t{i}" for i in range(50)]
    seg = np.concatenate([[0], np.cumsum(rng.integers(1, 20, size=50))])
    parts = scatter_segments(names, seg, 4)
    allidx = np.sort(np.concatenate([p[1] for p in parts]))
    assert np.array_equal(allidx, np.arange(seg[-1]))
    for g, (segs, idx, local) in enumerate(parts):
        assert all(gpu_of(names[s], 4) == g for s in segs)
        assert local[-1] == idx.size


def _bloom_sharded(rank, world):
    rng = np.random.default_rng(7)
    names = [f"tenant:{t:04d}" for t in range(40)]
    per = rng.integers(1, 30, size=len(names))
    seg = np.concatenate([[0], np.cumsum(per)])
    keys = [rng.bytes(16) for _ in range(int(seg[-1]))]
    # every tenant is pre-loaded with some keys (same on all ranks: deterministic)
    filt = {n: O.OracleBloom(9585, 7) for n in names}
    for n in names:
        filt[n].add(*O.arena([n.encode() + bytes([i]) for i in range(50)]))
    # single-process reference
    ref = []
    for s, n in enumerate(names):
        ref.append(filt[n].contains(*O.arena([n.encode() + bytes([i]) for i in range(3)] + keys[seg[s]:seg[s + 1]])))
    # this rank's shard only
    mine = np.zeros(len(names), np.int64)
    segs, idx, local = scatter_segments(names, seg, world)[rank]
    for j, s in enumerate(segs):
        n = names[s]
        sub = [keys[i] for i in idx[local[j]:local[j + 1]]]
        mine[s] = filt[n].contains(*O.arena([n.encode() + bytes([i]) for i in range(3)] + sub))
    t = torch.from_numpy(mine)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    assert t.tolist() == ref


def test_bloom_multitenant_sharded_gloo():
    _run(_bloom_sharded)


def _hll_partitioned(rank, world):
    rng = np.random.default_rng(8)
    nh, per = 6, 3000
    mats = [rng.integers(0, 256, size=(per, 16), dtype=np.uint8) for _ in range(nh)]
    regs = np.zeros((nh, 16384), np.uint8)
    for h in range(nh):
        lo, hi = partition_elements(per, world, rank)
        if hi > lo:
            O.hll_pfadd(regs[h], *O.fixed_arena(mats[h][lo:hi]))
    t = torch.from_numpy(regs)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)  # the RCCL ncclUint8/ncclMax step
    merged = t.numpy()
    for h in range(nh):
        ref = O.hll_new()
        O.hll_pfadd(ref, *O.fixed_arena(mats[h]))
        assert np.array_equal(merged[h], ref)
        assert O.hll_count(merged[h]) == O.hll_count(ref)


def test_hll_element_partitioned_max_allreduce_gloo():
    _run(_hll_partitioned)


def _bench_aggregation(rank, world):
    import bench

    assert bench.max_over_ranks(world, float(rank + 1)) == float(world)
    assert bench.sum_over_ranks(world, 10 * (rank + 1)) == 10 * world * (world + 1) // 2


def test_bench_rank_aggregation_gloo():
    _run(_bench_aggregation)


def test_bench_self_launches_n_ranks():
    """`bench.py --gpus N` with no launcher starts N ranks itself (torch.distributed.run child),
    each asserting WORLD_SIZE == N; --dry-run keeps it on the CPU (gloo)."""
    import json
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "3", "--dry-run"],
                       capture_output=True, text=True, timeout=240, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    line = [x for x in r.stdout.splitlines() if x.startswith("{")][-1]
    d = json.loads(line)
    assert d["n_gpus"] == 3 and d["ranks"] == 3 and len(set(d["pids"])) == 3


def test_bench_refuses_world_mismatch():
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--dry-run"],
                       capture_output=True, text=True, timeout=120, env=env)
    assert r.returncode == 2, (r.returncode, r.stderr[-2000:])


def _replica_digests(rank, world):
    """bench.py's C2 replica rule on the oracle: every rank adds the keys of ONE seed, so the
    replicas' Redis strings are identical and the digest all-gather agrees; rank-specific adds (the
    r02 bench) would not be one filter, and the same check catches it."""
    import hashlib

    import bench

    def digest(f):
        return int.from_bytes(hashlib.blake2b(f.redis_string(), digest_size=8).digest(), "little") >> 1

    keys = np.random.default_rng(0x5EED0002).integers(0, 256, size=(20_000, 32), dtype=np.uint8)
    f = O.OracleBloom(1 << 20, 7)
    f.add(*O.fixed_arena(keys))
    ds = bench.gather_over_ranks(world, digest(f))
    assert len(set(ds)) == 1
    own = np.random.default_rng(0x5EED0002 + 1000 * (rank + 1)).integers(0, 256, size=(20_000, 32), dtype=np.uint8)
    g = O.OracleBloom(1 << 20, 7)
    g.add(*O.fixed_arena(own))
    assert len(set(bench.gather_over_ranks(world, digest(g)))) == world


def test_c2_replicas_are_one_filter_gloo():
    _run(_replica_digests)
