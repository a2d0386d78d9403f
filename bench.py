#!/usr/bin/env python3
"""bench.py -- Bloom contains throughput on MI355X (BASELINE.json metric, config C2).

Step = one RBloomFilter.contains(Collection) pass (M/RedissonBloomFilter.java:153-186)
over a batch of 100M synthetic 32-byte keys (50% previously added) against ONE
2^32-bit filter with k = 7, keys resident in HBM when the timed region starts.

  python bench.py [--gpus N --steps K --warmup W] [--workload c2|c3|c4]

N > 1 is launched by torch.distributed.run, one rank per GPU; C2 does not shard
("replicas only"), so every rank runs its own replica with its own keys
(weak scaling) and `value` = keys of all ranks / max-over-ranks time.

Printed JSON (rank 0, one line) carries `roofline` for the contains call -- the partitioned
pipeline k_bk_stage1 -> k_bk_emit2 -> k_bk_probe -> k_bk_misses -> k_bk_final (contains_partitioned.hip),
timed with HIP events on the launch stream -- with its PMC traffic and memory-request count
(profiles/traffic.json, tools/profile_round.sh), an A/B against the direct early-exit kernel,
and `cpu_baseline`: the oracle's single-thread C restatement timed on a bounded sample.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md chip table (spec); 6.29 TB/s measured copy


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--workload", default="c2", choices=["c2", "c3", "c4", "c5"])
    p.add_argument("--keys", type=int, default=100_000_000, help="keys (C2/C3) or elements (C4) per step per GPU")
    p.add_argument("--tenants", type=int, default=100_000, help="C3 tenant count (whole node)")
    p.add_argument("--elements", type=int, default=1_000_000_000, help="C4 PFADD elements per step per GPU")
    p.add_argument("--stage1", type=int, default=None, help="contains early-exit schedule (rbx_tune)")
    p.add_argument("--tune", default="", help="extra rbx_tune settings for experiments: key=value,key=value")
    p.add_argument("--zipf-s", type=float, default=1.0, help="C5 tenant skew")
    p.add_argument("--add-fraction", type=float, default=0.1, help="C5 share of add commands")
    p.add_argument("--cpu-seconds", type=float, default=10.0, help="target CPU-baseline sample time")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "traffic.json"),
                   help="PMC-derived HBM bytes per launch (written by tools/pmc_traffic.py)")
    return p.parse_args()


def dist_setup(args):
    import torch

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # RBX_BENCH_SHARED_GPU=1 rehearses the multi-rank flow on a one-GPU box: every rank on
    # cuda:0, gloo for the barrier / max-over-ranks (RCCL cannot put two ranks on one GPU).
    shared = os.environ.get("RBX_BENCH_SHARED_GPU") == "1"
    if shared:
        local = 0
    torch.cuda.set_device(local)
    if world > 1:
        import torch.distributed as dist

        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if shared:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    return world, rank, local


def barrier(world):
    if world > 1:
        import torch.distributed as dist

        dist.barrier()


def _coll_device():
    import torch.distributed as dist

    return "cpu" if dist.get_backend() == "gloo" else "cuda"


def max_over_ranks(world, v: float) -> float:
    """The job's step time is the slowest rank's."""
    if world == 1:
        return v
    import torch
    import torch.distributed as dist

    t = torch.tensor([v], dtype=torch.float64, device=_coll_device())
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def sum_over_ranks(world, v: int) -> int:
    if world == 1:
        return v
    import torch
    import torch.distributed as dist

    t = torch.tensor([v], dtype=torch.int64, device=_coll_device())
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return int(t.item())


def load_traffic(path, kernel, field="hbm_bytes_per_launch"):
    try:
        with open(path) as fh:
            d = json.load(fh)
        return d.get(kernel, {}).get(field)
    except (OSError, ValueError):
        return None


def gather_peak(client, nbytes, nkeys, k, stream, gen):
    """Random 4-byte gathers/s over an nbytes table (k per key, nkeys keys): the request-rate
    roofline the Bloom kernels are measured against (k_gather_probe, same MLP structure)."""
    import torch

    from redisson_amd import _lib as L

    sptr = stream.cuda_stream
    sink = torch.zeros(1, dtype=torch.int32, device="cuda")
    table = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
    table.random_(0, 255, generator=gen)
    L.lib().rbx_bench_gather(client.ctx, table.data_ptr(), nbytes, nkeys, k, sink.data_ptr(), sptr)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(3):
        L.lib().rbx_bench_gather(client.ctx, table.data_ptr(), nbytes, nkeys, k, sink.data_ptr(), sptr)
    e1.record(stream)
    torch.cuda.synchronize()
    del table
    return nkeys * k / (e0.elapsed_time(e1) / 3 / 1e3)


def request_fields(traffic_json, kernel, ms, peak):
    """PMC memory requests per launch (TCC_EA0_RDREQ + WRREQ, profiles/traffic.json) vs the peak."""
    reqs = load_traffic(traffic_json, kernel, "requests_per_launch")
    return {"requests_per_launch": reqs, "request_rate_per_s": reqs / (ms / 1e3) if reqs else None,
            "request_peak_per_s": peak, "request_frac": reqs / (ms / 1e3) / peak if reqs and peak else None}


# ------------------------------------------------------------------------------------------
# CPU baseline: oracle restatement (single thread) on a bounded sample of the same workload
# ------------------------------------------------------------------------------------------
def cpu_baseline_c2(target_s: float):
    import numpy as np

    from oracle import oracle as O

    rng = np.random.default_rng(0x5EED0002)
    f = O.OracleBloom(1 << 32, 7)
    # calibrate on 200k keys
    cal = rng.integers(0, 256, size=(200_000, 32), dtype=np.uint8)
    f.add(*O.fixed_arena(cal))
    t0 = time.perf_counter()
    f.contains(*O.fixed_arena(cal))
    per_key = (time.perf_counter() - t0) / cal.shape[0]
    n = int(min(max(target_s / max(per_key, 1e-9), 200_000), 60_000_000))
    added = rng.integers(0, 256, size=(n // 2, 32), dtype=np.uint8)
    f.add(*O.fixed_arena(added))
    probe = np.concatenate([added, rng.integers(0, 256, size=(n - n // 2, 32), dtype=np.uint8)])
    b, o = O.fixed_arena(probe)
    t0 = time.perf_counter()
    c = f.contains(b, o)
    dt = time.perf_counter() - t0
    assert c >= n // 2
    return {"value": n / dt, "unit": "keys/s", "cores": 1, "kind": "port",
            "sample": f"CPU restatement, not reference (Redisson+redis-server absent): oracle/rbx_oracle.c "
                      f"contains of {n} 32-byte keys (50% present) on a 2^32-bit k=7 bitmap, 1 thread, "
                      f"{dt:.1f} s"}


# ------------------------------------------------------------------------------------------
# C2: single 2^32-bit filter, batch contains of 100M 32-byte keys
# ------------------------------------------------------------------------------------------
def run_c2(args, world, rank, local):
    import numpy as np
    import torch

    from redisson_amd import BloomHandle, RedissonClient, device_keys
    from redisson_amd import _lib as L

    K = 7
    SIZE = 1 << 32
    n = args.keys
    # a dedicated (non-null) stream: every engine launch and every timing event goes on it
    stream = torch.cuda.Stream()
    torch.cuda.set_stream(stream)
    sptr = stream.cuda_stream
    assert sptr, "need a non-default stream handle"
    client = RedissonClient(local)
    f = client.getBloomFilter("bench-c2")
    f.tryInitRaw(SIZE, K)
    h = BloomHandle(client, "bench-c2")

    g = torch.Generator(device="cuda")
    g.manual_seed(0x5EED0002 + 1000 * rank)
    half = n // 2
    added = torch.randint(0, 256, (half, 32), dtype=torch.uint8, device="cuda", generator=g)
    fresh = torch.randint(0, 256, (n - half, 32), dtype=torch.uint8, device="cuda", generator=g)
    probe = torch.cat([added, fresh])
    del fresh
    cnt = torch.zeros(4, dtype=torch.int64, device="cuda")  # [0] add, [1] warmup, [2] timed, [3] A/B

    # setup: add the first half (timed separately: the "add" half of the metric)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    h.add_dev(device_keys(added.data_ptr(), half, 32), cnt.data_ptr(), stream=sptr)
    e1.record(stream)
    torch.cuda.synchronize()
    add_ms = e0.elapsed_time(e1)
    n_new = int(cnt[0].item())

    dk = device_keys(probe.data_ptr(), n, 32)
    for _ in range(args.warmup):
        h.contains_dev(dk, cnt.data_ptr() + 8, stream=sptr)
    torch.cuda.synchronize()
    present_one = int(cnt[1].item()) // max(args.warmup, 1) if args.warmup else None

    # random-gather roofline probe at the same working-set size (the 512 MiB bitmap)
    sink = torch.zeros(1, dtype=torch.int32, device="cuda")
    bm_table = torch.empty(SIZE // 8, dtype=torch.uint8, device="cuda")
    bm_table.random_(0, 255, generator=g)
    L.lib().rbx_bench_gather(client.ctx, bm_table.data_ptr(), SIZE // 8, n, K, sink.data_ptr(), sptr)
    ge0, ge1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ge0.record(stream)
    for _ in range(3):
        L.lib().rbx_bench_gather(client.ctx, bm_table.data_ptr(), SIZE // 8, n, K, sink.data_ptr(), sptr)
    ge1.record(stream)
    torch.cuda.synchronize()
    gather_ms = ge0.elapsed_time(ge1) / 3
    gathers_per_s = n * K / (gather_ms / 1e3)
    del bm_table

    # timed region
    cnt[2].zero_()
    barrier(world)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ev0.record(stream)
    for _ in range(args.steps):
        h.contains_dev(dk, cnt.data_ptr() + 16, stream=sptr)
    ev1.record(stream)
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    barrier(world)
    kern_ms = ev0.elapsed_time(ev1) / args.steps
    total_present = int(cnt[2].item())
    if present_one is not None:
        assert total_present == present_one * args.steps, "contains count changed between steps"
    assert total_present >= half * args.steps  # no false negatives

    # A/B reference: the same step through the direct early-exit kernel (k_bloom_contains)
    L.lib().rbx_tune(b"contains_partition", 0)
    h.contains_dev(dk, cnt.data_ptr() + 24, stream=sptr)
    d0, d1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    d0.record(stream)
    for _ in range(3):
        h.contains_dev(dk, cnt.data_ptr() + 24, stream=sptr)
    d1.record(stream)
    torch.cuda.synchronize()
    L.lib().rbx_tune(b"contains_partition", 2)
    direct_ms = d0.elapsed_time(d1) / 3
    assert int(cnt[3].item()) == 4 * (total_present // args.steps), "direct and partitioned counts differ"

    step_s = max_over_ranks(world, max(kern_ms / 1e3, 0.0))
    keys_all = sum_over_ranks(world, n * args.steps)
    value = keys_all / (step_s * args.steps)
    algo_bytes = n * (32 + K * 8)  # 32 B key + k x 8 B gathered per key
    achieved = algo_bytes / (kern_ms / 1e3) / 1e9
    traffic = load_traffic(args.traffic_json, "contains_pipeline")
    reqs = load_traffic(args.traffic_json, "contains_pipeline", "requests_per_launch")
    res = {
        "metric": "Bloom contains keys/sec (whole node), C2: one 2^32-bit filter, k=7, 32-byte keys",
        "value": value, "unit": "keys/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": step_s * 1e3, "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
        "dtype": "u8", "data": "synthetic",
        "config": {"workload": "C2 RBloomFilter.contains(Collection) of 100M random 32-byte keys "
                               "(50% present) vs one 2^32-bit k=7 filter per GPU",
                   "keys_per_gpu": n, "key_bytes": 32, "size_bits": SIZE, "k": K,
                   "parallelism": f"replicas x{world} (no data-path collective)"},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                     "algorithmic_bytes_per_launch": algo_bytes,
                     # one contains call = the partitioned pipeline's kernels in sequence on one stream
                     "kernel": "contains pipeline: k_bk_stage1<32,8,512> + k_bk_emit2<1024> + k_bk_probe + k_bk_misses + k_bk_final",
                     "kernel_avg_ms": kern_ms,
                     # the binding limit: memory requests at the L2->EA interface (PMC TCC_EA0_RD/WRREQ),
                     # against the measured random-gather request rate at this working set
                     "requests_per_launch": reqs,
                     "request_rate_per_s": (reqs / (kern_ms / 1e3)) if reqs else None,
                     "request_peak_per_s": gathers_per_s,
                     "request_frac": (reqs / (kern_ms / 1e3) / gathers_per_s) if reqs else None,
                     # north-star definition: keys/s x k / measured random-gather peak at this
                     # working set (> 1: early exit and LDS probes avoid most random gathers)
                     "gather_peak_per_s": gathers_per_s, "gather_frac": (n * K / (kern_ms / 1e3)) / gathers_per_s},
        "extra": {"add_keys_per_s_per_gpu": half / (add_ms / 1e3), "add_new_keys": n_new,
                  "present_per_step": total_present // args.steps, "wall_s_timed": wall,
                  "contains_direct_kernel_ms": direct_ms,
                  "contains_direct_keys_per_s_per_gpu": n / (direct_ms / 1e3),
                  # the setup add = the partitioned add pipeline (add_partitioned.hip), PMC per call
                  "add_ms": add_ms,
                  "add_traffic": load_traffic(args.traffic_json, "add_pipeline"),
                  "add_requests_per_call": load_traffic(args.traffic_json, "add_pipeline", "requests_per_launch")},
    }
    h.close()
    client.shutdown()
    return res


# ------------------------------------------------------------------------------------------
# C3: 100k tenant filters tryInit(1e6, 1e-3), sharded by CRC16 slot across the node's GPUs
# ------------------------------------------------------------------------------------------
def run_c3(args, world, rank, local):
    import ctypes as C

    import numpy as np
    import torch

    from redisson_amd import BloomHandle, RedissonClient, calc_slot, device_keys, slot_to_gpu
    from redisson_amd import _lib as L

    NT = args.tenants
    stream = torch.cuda.Stream()
    torch.cuda.set_stream(stream)
    sptr = stream.cuda_stream
    client = RedissonClient(local)
    names = [f"tenant:{t:06d}" for t in range(NT)]
    mine = [nm for nm in names if slot_to_gpu(calc_slot(nm), world) == rank]
    nt = len(mine)
    g = torch.Generator(device="cuda")
    g.manual_seed(0x5EED0003 + rank)
    # a pool of random bytes: each bit set with p = 1/2 = the fill of a filter at its design
    # load (1 - exp(-k n / m) = 0.50 for n = 1e6, m = 14,377,587, k = 10)
    pool = torch.randint(0, 256, (64 << 20,), dtype=torch.uint8, device="cuda", generator=g)
    t0 = time.perf_counter()
    handles = []
    rng = np.random.default_rng(rank)
    for nm in mine:
        f = client.getBloomFilter(nm)
        f.tryInit(1_000_000, 1e-3)
        nbytes = (f._size + 7) // 8
        off = int(rng.integers(0, (pool.numel() - nbytes) // 256)) * 256
        assert L.lib().rbx_bloom_import_dev(client.ctx, nm.encode(), pool.data_ptr() + off, nbytes, sptr) == 0
        handles.append(BloomHandle(client, nm))
    setup_s = time.perf_counter() - t0
    size, k = handles[0].size, handles[0].k
    per = max(1, args.keys // nt)
    n = per * nt
    keys = torch.randint(0, 256, (n, 16), dtype=torch.uint8, device="cuda", generator=g)
    seg = torch.arange(nt + 1, dtype=torch.int64, device="cuda") * per
    counts = torch.zeros(nt, dtype=torch.int64, device="cuda")
    arr = (C.c_void_p * nt)(*[h.h.value for h in handles])
    dk = device_keys(keys.data_ptr(), n, 16)

    def step():
        assert L.lib().rbx_bloom_contains_multi_dev(client.ctx, arr, nt, seg.data_ptr(), C.byref(dk), None,
                                                     counts.data_ptr(), sptr) == 0

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    barrier(world)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(args.steps):
        step()
    e1.record(stream)
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / args.steps
    step_s = max_over_ranks(world, ms / 1e3)
    value = sum_over_ranks(world, n) / step_s
    present = int(counts.sum().item()) / max(args.warmup + args.steps, 1)
    peak = gather_peak(client, 4 << 30, n, 4, stream, g)  # random gathers over a table far past the caches
    algo = n * (16 + k * 8)
    achieved = algo / (ms / 1e3) / 1e9
    # 180 GB of bitmaps: the slot kernel unless a staged schedule was forced
    slots = args.stage1 is None or args.stage1 == 5
    kname = "k_bloom_contains_q" if slots else "k_bloom_contains_multi"
    kdesc = "k_bloom_contains_q<16,true,2,2>" if slots else f"k_bloom_contains_multi<16,16,{args.stage1}>"
    res = {
        "metric": "Bloom contains keys/sec (whole node), C3: 100k tenant filters tryInit(1e6,1e-3), CRC16-slot sharded",
        "value": value, "unit": "keys/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": step_s * 1e3, "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
        "dtype": "u8", "data": "synthetic",
        "config": {"workload": f"C3 one contains(Collection) per tenant, {per} random 16-byte keys each, "
                               f"{nt} of {NT} tenants on this GPU (slot*N/16384), filters at design fill 0.5",
                   "tenants_total": NT, "tenants_this_gpu": nt, "size_bits": size, "k": k, "keys_per_gpu": n,
                   "parallelism": f"CRC16-slot sharded x{world} (no data-path collective)"},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": load_traffic(args.traffic_json, kname),
                     "kernel": kdesc, "kernel_avg_ms": ms, **request_fields(args.traffic_json, kname, ms, peak)},
        "extra": {"setup_s": setup_s, "present_fraction": present / n},
    }
    for h in handles:
        h.close()
    client.shutdown()
    return res


# ------------------------------------------------------------------------------------------
# C5: ordered 90/10 contains/add stream, Zipf(1.0) tenants over the C3 set, 64-byte keys
# ------------------------------------------------------------------------------------------
def run_c5(args, world, rank, local):
    import ctypes as C

    import numpy as np
    import torch

    from redisson_amd import BloomHandle, RedissonClient, calc_slot, device_keys, slot_to_gpu
    from redisson_amd import _lib as L

    NT = args.tenants
    stream = torch.cuda.Stream()
    torch.cuda.set_stream(stream)
    sptr = stream.cuda_stream
    client = RedissonClient(local)
    names = [f"tenant:{t:06d}" for t in range(NT)]
    ranks = np.arange(1, NT + 1, dtype=np.float64)  # Zipf popularity rank of tenant t is t+1
    mine = [t for t in range(NT) if slot_to_gpu(calc_slot(names[t]), world) == rank]
    nt = len(mine)
    g = torch.Generator(device="cuda")
    g.manual_seed(0x5EED0005 + rank)
    pool = torch.randint(0, 256, (64 << 20,), dtype=torch.uint8, device="cuda", generator=g)
    rng = np.random.default_rng(rank)
    handles = []
    for t in mine:
        f = client.getBloomFilter(names[t])
        f.tryInit(1_000_000, 1e-3)
        nbytes = (f._size + 7) // 8
        off = int(rng.integers(0, (pool.numel() - nbytes) // 256)) * 256
        assert L.lib().rbx_bloom_import_dev(client.ctx, names[t].encode(), pool.data_ptr() + off, nbytes, sptr) == 0
        handles.append(BloomHandle(client, names[t]))
    n = args.keys
    w = torch.tensor(1.0 / ranks[mine] ** args.zipf_s, dtype=torch.float64, device="cuda")
    cdf = torch.cumsum(w, 0)
    cdf /= cdf[-1].clone()
    u = torch.rand(n, dtype=torch.float64, device="cuda", generator=g)
    kf = torch.searchsorted(cdf, u).clamp_(max=nt - 1).to(torch.int32)
    op = (torch.rand(n, device="cuda", generator=g) < args.add_fraction).to(torch.uint8)
    keys = torch.randint(0, 256, (n, 64), dtype=torch.uint8, device="cuda", generator=g)
    counts = torch.zeros(2, dtype=torch.int64, device="cuda")
    arr = (C.c_void_p * nt)(*[h.h.value for h in handles])
    dk = device_keys(keys.data_ptr(), n, 64)

    def step():
        assert L.lib().rbx_bloom_stream_dev(client.ctx, arr, nt, kf.data_ptr(), op.data_ptr(), C.byref(dk), None,
                                             counts.data_ptr(), sptr) == 0

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    barrier(world)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(args.steps):
        step()
    e1.record(stream)
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / args.steps
    step_s = max_over_ranks(world, ms / 1e3)
    value = sum_over_ranks(world, n) / step_s
    top = int(torch.bincount(kf.long(), minlength=nt).max().item())
    peak = gather_peak(client, 4 << 30, n, 4, stream, g)
    res = {
        "metric": "Bloom mixed contains+add ops/sec (whole node), C5: 90/10 stream, Zipf tenants, 64-byte keys",
        "value": value, "unit": "ops/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": step_s * 1e3, "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
        "dtype": "u8", "data": "synthetic",
        "config": {"workload": f"C5 ordered stream of {n} single-key commands ({args.add_fraction:.0%} add) over "
                               f"{nt} tenant filters tryInit(1e6,1e-3) at design fill, Zipf(s={args.zipf_s}) tenants, "
                               "64-byte keys, in-order semantics",
                   "tenants_this_gpu": nt, "ops_per_gpu": n, "hottest_tenant_ops": top,
                   "parallelism": f"CRC16-slot sharded x{world} (no data-path collective)"},
        "roofline": {"bound": "hbm", "achieved": n * (64 + 10 * 8) / (ms / 1e3) / 1e9, "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": n * (64 + 10 * 8) / (ms / 1e3) / 1e9 / HBM_PEAK_GBS,
                     "traffic": load_traffic(args.traffic_json, "stream_pipeline"),
                     "kernel": "k_stream_probe + k_stream_contains + k_stream_commit", "kernel_avg_ms": ms,
                     **request_fields(args.traffic_json, "stream_pipeline", ms, peak)},
    }
    for h in handles:
        h.close()
    client.shutdown()
    return res


# ------------------------------------------------------------------------------------------
# C4: 10k HLLs, PFADD of 16-byte elements, PFCOUNT of all, RCCL max merge
# ------------------------------------------------------------------------------------------
def run_c4(args, world, rank, local):
    import ctypes as C

    import numpy as np
    import torch

    from redisson_amd import RedissonClient, device_keys
    from redisson_amd import _lib as L

    NH = 10_000
    per = max(1, args.elements // NH)  # elements per HLL per GPU per step
    n = NH * per
    stream = torch.cuda.Stream()
    torch.cuda.set_stream(stream)
    sptr = stream.cuda_stream
    client = RedissonClient(local)
    hs = []
    for i in range(NH):
        hp = C.c_void_p()
        assert L.lib().rbx_hll_open(client.ctx, f"c4-{i}".encode(), 1, C.byref(hp)) == 0
        hs.append(hp.value)
    arr = (C.c_void_p * NH)(*hs)
    seg = np.arange(NH + 1, dtype=np.uint64) * np.uint64(per)
    g = torch.Generator(device="cuda")
    g.manual_seed(0x5EED0004 + rank)
    el = torch.randint(0, 256, (n, 16), dtype=torch.uint8, device="cuda", generator=g)
    changed = torch.zeros(NH, dtype=torch.int32, device="cuda")
    dk = device_keys(el.data_ptr(), n, 16)
    for _ in range(args.warmup):
        assert L.lib().rbx_hll_add_multi_dev(client.ctx, arr, NH, None, seg.ctypes.data_as(L.u64p), C.byref(dk),
                                             changed.data_ptr(), sptr) == 0
    torch.cuda.synchronize()
    barrier(world)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(args.steps):
        assert L.lib().rbx_hll_add_multi_dev(client.ctx, arr, NH, None, seg.ctypes.data_as(L.u64p), C.byref(dk),
                                             changed.data_ptr(), sptr) == 0
    e1.record(stream)
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / args.steps
    merge_ms = None
    if world > 1 and os.environ.get("RBX_BENCH_SHARED_GPU") != "1":
        # element-partitioned registers -> RCCL uint8 max all-reduce over xGMI
        import torch.distributed as dist

        uid = (C.c_uint8 * 128)()
        if rank == 0:
            assert L.lib().rbx_rccl_unique_id(uid) == 0
        obj = [bytes(uid)]
        dist.broadcast_object_list(obj, src=0)
        uid = (C.c_uint8 * 128).from_buffer_copy(obj[0])
        assert L.lib().rbx_rccl_init(client.ctx, uid, world, rank) == 0
        assert L.lib().rbx_hll_allreduce_max(client.ctx, arr, NH) == 0  # warm
        L.lib().rbx_synchronize(client.ctx)
        barrier(world)
        t0 = time.perf_counter()
        assert L.lib().rbx_hll_allreduce_max(client.ctx, arr, NH) == 0
        L.lib().rbx_synchronize(client.ctx)
        merge_ms = (time.perf_counter() - t0) * 1e3
    out = np.zeros(NH, np.uint64)
    t0 = time.perf_counter()
    assert L.lib().rbx_hll_count_each_handles(client.ctx, arr, NH, out.ctypes.data_as(L.u64p)) == 0
    count_ms = (time.perf_counter() - t0) * 1e3
    step_s = max_over_ranks(world, ms / 1e3)
    value = sum_over_ranks(world, n) / step_s
    achieved = n * 16 / (ms / 1e3) / 1e9
    res = {
        "metric": "HLL PFADD elems/sec (whole node), C4: 10k HLLs, 16-byte elements",
        "value": value, "unit": "elems/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": step_s * 1e3, "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
        "dtype": "u8", "data": "synthetic",
        "config": {"workload": f"C4 PFADD {per} x 16-byte elements into each of 10k HLLs per GPU",
                   "elements_per_gpu": n, "parallelism": f"element-partitioned x{world}"},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": load_traffic(args.traffic_json, "k_hll_pfadd"),
                     "kernel": "k_hll_pfadd<16>", "kernel_avg_ms": ms},
        "extra": {"pfcount_10k_ms": count_ms, "mean_count": float(out.mean()), "rccl_max_allreduce_ms": merge_ms,
                  "allreduce_bytes": NH * 16384},
    }
    for hp in hs:
        L.lib().rbx_hll_close(hp)
    client.shutdown()
    return res


def main():
    args = parse()
    world, rank, local = dist_setup(args)
    if args.stage1 is not None:
        from redisson_amd import _lib as L

        assert L.lib().rbx_tune(b"contains_stage1", args.stage1) == 0
        # a forced staged schedule applies to multi-tenant calls too (no automatic slot kernel)
        assert L.lib().rbx_tune(b"contains_multi_slots", 1 if args.stage1 == 5 else 0) == 0
    for kv in filter(None, args.tune.split(",")):
        from redisson_amd import _lib as L

        key, val = kv.split("=")
        assert L.lib().rbx_tune(key.encode(), int(val)) == 0, kv
    log(f"[bench] rank {rank}/{world} workload {args.workload}")
    if args.workload == "c2":
        res = run_c2(args, world, rank, local)
        if rank == 0 and world == 1 and not args.no_cpu_baseline:
            res["cpu_baseline"] = cpu_baseline_c2(args.cpu_seconds)
    elif args.workload == "c4":
        res = run_c4(args, world, rank, local)
    elif args.workload == "c5":
        res = run_c5(args, world, rank, local)
    else:
        res = run_c3(args, world, rank, local)
    if rank == 0:
        res.setdefault("cpu_baseline", None)
        print(json.dumps(res), flush=True)
    if world > 1:
        import torch.distributed as dist

        dist.destroy_process_group()


if __name__ == "__main__":
    main()
