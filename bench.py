#!/usr/bin/env python3
"""bench.py -- Bloom contains throughput on MI355X (BASELINE.json metric, config C2), with the
C1 / C3 / C4 / C5 legs of the same metric family carried in the same JSON line.

Step = one RBloomFilter.contains(Collection) pass (M/RedissonBloomFilter.java:153-186) over a
batch of 100M synthetic 32-byte keys (50% previously added) against ONE 2^32-bit filter with
k = 7, keys resident in HBM when the timed region starts.

  python bench.py [--gpus N --steps K --warmup W] [--workload c2|c3|c4|c5] [--legs c1,c3,c4,c5|none]

Multi-GPU: one rank per GPU.  The driver launches N > 1 through torch.distributed.run; when
WORLD_SIZE is unset and --gpus N > 1, bench.py launches those N ranks itself (a child
torch.distributed.run, started before anything touches the GPU) and exits with its status.
Every rank asserts WORLD_SIZE == --gpus.
  - C2 does not shard ("replicas only"): every rank holds a replica of ONE filter (the
    same adds, bitmap digests compared across ranks) and serves its own share of the contains
    stream (weak scaling); `value` = keys of all ranks / max-over-ranks time.
  - leg C3 shards 100k tenant filters by CRC16 slot (slot * N / 16384, ClusterConnectionManager
    .java:814-830) with no data-path collective;
  - leg C4 partitions PFADD elements over the ranks and merges the 10k x 16384 partial registers
    with one RCCL uint8 MAX all-reduce (163.84 MB) over xGMI.
RBX_BENCH_SHARED_GPU=1 rehearses N ranks on one GPU (gloo for the bench's own collectives and
for the C4 register exchange: RCCL needs a GPU per rank).

Printed JSON (rank 0, one line): `roofline` for the C2 contains call (the partitioned pipeline,
HIP events on the launch stream), its PMC traffic per access class (profiles/traffic.json from
tools/profile_round.sh), a streaming-floor roofline of the same call, and `cpu_baseline`: the
multithreaded C restatement (oracle/rbx_oracle_mt.c) on the host cores on C2 and C1 samples.
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
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
    p.add_argument("--legs", default="c1,c3,c4,c5",
                   help="legs carried in the C2 line: comma list of c1,c3,c4,c5 or 'none'")
    p.add_argument("--leg-steps", type=int, default=10)
    p.add_argument("--keys", type=int, default=100_000_000, help="keys (C2/C3) or elements (C4) per step per GPU")
    p.add_argument("--tenants", type=int, default=100_000, help="C3 tenant count (whole node)")
    p.add_argument("--elements", type=int, default=1_000_000_000, help="C4 PFADD elements per step per GPU")
    p.add_argument("--stage1", type=int, default=None, help="contains early-exit schedule (rbx_tune)")
    p.add_argument("--tune", default="", help="extra rbx_tune settings for experiments: key=value,key=value")
    p.add_argument("--zipf-s", type=float, default=1.0, help="C5 tenant skew")
    p.add_argument("--add-fraction", type=float, default=0.1, help="C5 share of add commands")
    p.add_argument("--c5-replies", type=int, default=1,
                   help="C5: write every command's reply in the timed step (1, the metric) or not (0, A/B only)")
    p.add_argument("--c5-fresh", type=int, default=1,
                   help="C5: step s gives command i key i+s of a pool of n+W+K keys, so every step's (tenant, key) "
                        "pairs are new (1), or replays the same stream each step (0)")
    p.add_argument("--cpu-seconds", type=float, default=10.0, help="target CPU-baseline C2 sample time")
    p.add_argument("--c3-add", type=int, default=1, help="C3 leg: also time the add half (one add_multi per step)")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--no-hostpath", action="store_true", help="skip the PCIe-inclusive host-buffer measurement")
    p.add_argument("--dry-run", action="store_true",
                   help="rank plumbing only (CPU, gloo): every rank reports in, rank 0 prints the rank census")
    p.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "traffic.json"),
                   help="PMC-derived HBM bytes per launch (written by tools/pmc_traffic.py)")
    return p.parse_args()


# ------------------------------------------------------------------------------------------
# ranks
# ------------------------------------------------------------------------------------------
def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def self_launch(args) -> int:
    """--gpus N > 1 without a launcher: start N ranks with torch.distributed.run as a CHILD
    process (nothing in this process has touched the GPU) and return its exit status."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", os.path.abspath(__file__), *sys.argv[1:]]
    log("[bench] launching", " ".join(cmd[2:]))
    return subprocess.call(cmd)


def dist_setup(args):
    import torch

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        log(f"[bench] WORLD_SIZE={world} but --gpus {args.gpus}: refusing to report a mislabelled run")
        sys.exit(2)
    # RBX_BENCH_SHARED_GPU=1 rehearses the multi-rank flow on a one-GPU box: every rank on
    # cuda:0, gloo for the barrier / max-over-ranks (RCCL cannot put two ranks on one GPU).
    shared = os.environ.get("RBX_BENCH_SHARED_GPU") == "1"
    if shared:
        local = 0
    if not args.dry_run:
        torch.cuda.set_device(local)
    if world > 1:
        import torch.distributed as dist

        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if shared or args.dry_run:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    return world, rank, local


def shared_gpu() -> bool:
    return os.environ.get("RBX_BENCH_SHARED_GPU") == "1"


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


def gather_over_ranks(world, v: int) -> list[int]:
    if world == 1:
        return [v]
    import torch
    import torch.distributed as dist

    t = torch.zeros(world, dtype=torch.int64, device=_coll_device())
    t[dist.get_rank()] = v
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return [int(x) for x in t.tolist()]


# ------------------------------------------------------------------------------------------
# measurement helpers
# ------------------------------------------------------------------------------------------
C2_PROFILED_KEYS = 100_000_000  # keys per contains call in the PMC profiles of profiles/traffic.json


def load_traffic(path, kernel, field="hbm_bytes_per_launch"):
    if path is None:
        return None
    try:
        with open(path) as fh:
            d = json.load(fh)
        return d.get(kernel, {}).get(field)
    except (OSError, ValueError):
        return None


class Timer:
    """HIP events on the launch stream (torch.cuda.Event records on the stream passed)."""

    def __init__(self, stream):
        import torch

        self.stream = stream
        self.e0, self.e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)

    def __enter__(self):
        self.e0.record(self.stream)
        return self

    def __exit__(self, *exc):
        import torch

        self.e1.record(self.stream)
        torch.cuda.synchronize()
        self.ms = self.e0.elapsed_time(self.e1)


def gather_peak(client, nbytes, nkeys, k, stream, gen):
    """Uniformly random 4-byte gathers/s over an nbytes table (k per key): the request roofline
    of a single large filter (k_gather_probe, same MLP structure as the contains kernels)."""
    import torch

    from redisson_amd import _lib as L

    sptr = stream.cuda_stream
    sink = torch.zeros(1, dtype=torch.int32, device="cuda")
    table = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
    table.random_(0, 255, generator=gen)
    L.lib().rbx_bench_gather(client.ctx, table.data_ptr(), nbytes, nkeys, k, sink.data_ptr(), sptr)
    with Timer(stream) as t:
        for _ in range(3):
            L.lib().rbx_bench_gather(client.ctx, table.data_ptr(), nbytes, nkeys, k, sink.data_ptr(), sptr)
    del table
    return nkeys * k / (t.ms / 3 / 1e3)


def segment_gather_peak(client, table_ptr, table_bytes, seg_bytes, keys_per_seg, nkeys, stream):
    """Random 4-byte gathers/s with the locality of a multi-tenant batch: consecutive keys share
    one seg_bytes slice (k_gather_segments, 4 loads per key) -- C3's request roofline."""
    import torch

    from redisson_amd import _lib as L

    sptr = stream.cuda_stream
    sink = torch.zeros(1, dtype=torch.int32, device="cuda")
    args = (client.ctx, table_ptr, table_bytes, seg_bytes, keys_per_seg, nkeys, sink.data_ptr(), sptr)
    L.lib().rbx_bench_gather_segments(*args)
    with Timer(stream) as t:
        for _ in range(3):
            L.lib().rbx_bench_gather_segments(*args)
    return nkeys * 4 / (t.ms / 3 / 1e3)


def stream_read_peak(client, nbytes, stream):
    """HBM stream-read GB/s (16-byte loads over an nbytes buffer): the PFADD roofline."""
    import torch

    from redisson_amd import _lib as L

    sptr = stream.cuda_stream
    sink = torch.zeros(1, dtype=torch.int32, device="cuda")
    buf = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
    L.lib().rbx_bench_stream_read(client.ctx, buf.data_ptr(), nbytes, sink.data_ptr(), sptr)
    with Timer(stream) as t:
        for _ in range(5):
            L.lib().rbx_bench_stream_read(client.ctx, buf.data_ptr(), nbytes, sink.data_ptr(), sptr)
    del buf
    return nbytes / (t.ms / 5 / 1e3) / 1e9


def stream_write_peak(client, nbytes, stream):
    """HBM stream-write rate (16-byte nontemporal stores over an nbytes buffer) in 64-byte write
    requests per second: the write side of the request roofline."""
    import torch

    from redisson_amd import _lib as L

    sptr = stream.cuda_stream
    buf = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
    L.lib().rbx_bench_stream_write(client.ctx, buf.data_ptr(), nbytes, sptr)
    with Timer(stream) as t:
        for _ in range(5):
            L.lib().rbx_bench_stream_write(client.ctx, buf.data_ptr(), nbytes, sptr)
    del buf
    return nbytes / 64 / (t.ms / 5 / 1e3)


def request_fields(traffic_json, kernel, ms, peak, write_peak=None):
    """PMC memory requests per launch (TCC_EA0_RDREQ + WRREQ, profiles/traffic.json) against the
    request rates measured in the same run: reads at `peak` (random gathers at the same working set
    and locality -- above the streaming-read request rate), writes at `write_peak` (whole 64-byte
    streaming writes).  request_frac = (reads / peak + writes / write_peak) / call time: the share
    of the call a request-bound design needs at those rates."""
    reqs = load_traffic(traffic_json, kernel, "requests_per_launch")
    rd = load_traffic(traffic_json, kernel, "read_requests_per_launch")
    wr = load_traffic(traffic_json, kernel, "write_requests_per_launch")
    at = load_traffic(traffic_json, kernel, "atomic_requests_per_launch")
    out = {"requests_per_launch": reqs, "request_rate_per_s": reqs / (ms / 1e3) if reqs else None,
           "request_peak_per_s": peak, "read_requests_per_launch": rd, "write_requests_per_launch": wr,
           "write_request_peak_per_s": write_peak,
           # atomic requests (PMC TCC_ATOMIC; all of them execute at the memory side and are
           # counted in the write requests too) and their throughput at this call time
           "atomic_requests_per_launch": at, "atomic_rate_per_s": at / (ms / 1e3) if at else None}
    if rd is not None and wr is not None and peak and write_peak:
        floor_s = rd / peak + wr / write_peak
        out["request_floor_ms"] = floor_s * 1e3
        out["request_frac"] = floor_s / (ms / 1e3)
    else:
        out["request_frac"] = reqs / (ms / 1e3) / peak if reqs and peak else None
    return out


# ------------------------------------------------------------------------------------------
# CPU baseline: the multithreaded C restatement on the host cores (BASELINE.md fallback)
# ------------------------------------------------------------------------------------------
def cpu_model() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_threads() -> int:
    """The host cores this job may use: OMP_NUM_THREADS (16 on the GPU box, its CPU share --
    os.cpu_count() there reports the whole machine) or else every core."""
    v = os.environ.get("RBX_CPU_THREADS") or os.environ.get("OMP_NUM_THREADS")
    return max(1, int(v)) if v else (os.cpu_count() or 1)


def cpu_baseline(target_s: float):
    import numpy as np

    from oracle import oracle as O

    T = cpu_threads()
    # C2 sample: contains of n 32-byte keys (50% present) on a 2^32-bit k = 7 bitmap, repeated
    # passes until ~target_s of wall time (n bounded to keep host memory small)
    rng = np.random.default_rng(0x5EED0002)
    f = O.OracleBloom(1 << 32, 7)
    n = 16_000_000
    added = rng.integers(0, 256, size=(n // 2, 32), dtype=np.uint8)
    f.add_mt(*O.fixed_arena(added), nthreads=T)
    probe = np.concatenate([added, rng.integers(0, 256, size=(n - n // 2, 32), dtype=np.uint8)])
    del added
    b, o = O.fixed_arena(probe)
    passes, t0 = 0, time.perf_counter()
    while True:
        c = f.contains_mt(b, o, nthreads=T)
        passes += 1
        dt = time.perf_counter() - t0
        if dt >= target_s or passes >= 50:
            break
    assert c >= n // 2
    c2_rate = n * passes / dt
    del probe, b, o, f
    # C1: tryInit(1e7, 0.01) -> 95,850,583 bits, k = 7; add 1M 16-byte keys, then contains the
    # same 1M + 1M fresh, repeated on fresh bitmaps for >= 3 s
    size, k = O.bloom_optimal(10_000_000, 0.01)
    rng = np.random.default_rng(0x5EED0001)
    keys = rng.integers(0, 256, size=(1_000_000, 16), dtype=np.uint8)
    probe = np.concatenate([keys, rng.integers(0, 256, size=(1_000_000, 16), dtype=np.uint8)])
    ka, pa = O.fixed_arena(keys), O.fixed_arena(probe)
    t_add = t_con = 0.0
    reps = 0
    while t_add + t_con < 3.0 or reps < 2:
        g = O.OracleBloom(size, k)
        t0 = time.perf_counter()
        added_new = g.add_mt(*ka, nthreads=T)
        t1 = time.perf_counter()
        present = g.contains_mt(*pa, nthreads=T)
        t2 = time.perf_counter()
        t_add, t_con, reps = t_add + t1 - t0, t_con + t2 - t1, reps + 1
    assert present >= 1_000_000 and added_new > 990_000
    return {"value": c2_rate, "unit": "keys/s", "cores": T, "kind": "port",
            "sample": f"CPU restatement, not reference (Redisson+redis-server absent): oracle/rbx_oracle_mt.c "
                      f"contains of {n} 32-byte keys (50% present) on a 2^32-bit k=7 bitmap, {passes} passes, "
                      f"{T} threads, {dt:.1f} s",
            "nproc": os.cpu_count(), "cpu_model": cpu_model(),
            "c1": {"workload": "tryInit(1e7,0.01) m=95,850,583 k=7: add 1M 16-byte keys, contains 1M present + "
                               "1M absent", "reps": reps, "threads": T,
                   "add_keys_per_s": 1_000_000 * reps / t_add, "contains_keys_per_s": 2_000_000 * reps / t_con,
                   "keys_per_s": 3_000_000 * reps / (t_add + t_con)}}


# ------------------------------------------------------------------------------------------
# C2: single 2^32-bit filter, batch contains of 100M 32-byte keys (the headline)
# ------------------------------------------------------------------------------------------
def host_path_rate(client, name, n=20_000_000):
    """The rate a Java caller handing over host buffers sees: rbx_bloom_contains on a pinned
    host arena (keys cross PCIe inside the call)."""
    import ctypes as C

    import numpy as np

    from redisson_amd import _lib as L

    p = C.c_void_p()
    assert L.lib().rbx_host_alloc(n * 32, C.byref(p)) == 0
    try:
        buf = np.ctypeslib.as_array((C.c_uint8 * (n * 32)).from_address(p.value))
        buf[:] = np.random.default_rng(7).integers(0, 256, size=n * 32, dtype=np.uint8)
        keys = L.RbxKeys(p.value, None, 32, n)
        cnt = C.c_uint64()
        assert L.lib().rbx_bloom_contains(client.ctx, name.encode(), 0, 0, C.byref(keys), None, C.byref(cnt)) == 0
        t0 = time.perf_counter()
        reps = 3
        for _ in range(reps):
            assert L.lib().rbx_bloom_contains(client.ctx, name.encode(), 0, 0, C.byref(keys), None,
                                              C.byref(cnt)) == 0
        dt = (time.perf_counter() - t0) / reps
    finally:
        L.lib().rbx_host_free(p)
    return {"keys_per_s_per_gpu": n / dt, "keys": n, "key_bytes": 32, "pinned": True,
            "note": "rbx_bloom_contains on a pinned host arena: PCIe-inclusive (what a Java caller handing "
                    "over off-heap buffers sees); `value` uses HBM-resident keys"}


def run_c2(args, world, rank, local):
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

    # Replicas of ONE filter (SURVEY 8e "replicas only"): every rank adds the same keys (the same
    # seed), so the bitmaps are identical -- checked below by a digest all-gather -- and each
    # replica serves its own share of the contains stream (its present half is the added keys, its
    # absent half is rank-specific).
    g = torch.Generator(device="cuda")
    g.manual_seed(0x5EED0002)
    half = n // 2
    added = torch.randint(0, 256, (half, 32), dtype=torch.uint8, device="cuda", generator=g)
    g.manual_seed(0x5EED0002 + 1000 * (rank + 1))
    fresh = torch.randint(0, 256, (n - half, 32), dtype=torch.uint8, device="cuda", generator=g)
    probe = torch.cat([added, fresh])
    del fresh
    cnt = torch.zeros(4, dtype=torch.int64, device="cuda")  # [0] add, [1] warmup, [2] timed, [3] A/B

    # setup: add the first half (timed separately: the "add" half of the metric), after one
    # untimed add of the same keys into a scratch filter (first-call scratch allocations)
    fw = client.getBloomFilter("bench-c2-warm")
    fw.tryInitRaw(SIZE, K)
    hw = BloomHandle(client, "bench-c2-warm")
    hw.add_dev(device_keys(added.data_ptr(), half, 32), cnt.data_ptr(), stream=sptr)
    torch.cuda.synchronize()
    hw.close()
    fw.delete()
    cnt.zero_()
    torch.cuda.synchronize()
    with Timer(stream) as t_add:
        h.add_dev(device_keys(added.data_ptr(), half, 32), cnt.data_ptr(), stream=sptr)
    n_new = int(cnt[0].item())
    # the replicas are one filter: equal digests of `GET bench-c2` on every rank
    digest = f.digest()
    digests = gather_over_ranks(world, digest - (1 << 64) if digest >= 1 << 63 else digest)
    assert len(set(digests)) == 1 and digests[0] != 0, f"replicas differ: {digests}"

    dk = device_keys(probe.data_ptr(), n, 32)
    for _ in range(args.warmup):
        h.contains_dev(dk, cnt.data_ptr() + 8, stream=sptr)
    torch.cuda.synchronize()
    present_one = int(cnt[1].item()) // max(args.warmup, 1) if args.warmup else None

    gathers_per_s = gather_peak(client, SIZE // 8, n, K, stream, g)  # same 512 MiB working set
    writes_per_s = stream_write_peak(client, 2 << 30, stream)

    # timed region
    cnt[2].zero_()
    barrier(world)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    with Timer(stream) as t_main:
        for _ in range(args.steps):
            h.contains_dev(dk, cnt.data_ptr() + 16, stream=sptr)
    wall = time.perf_counter() - t0
    barrier(world)
    kern_ms = t_main.ms / args.steps
    total_present = int(cnt[2].item())
    if present_one is not None:
        assert total_present == present_one * args.steps, "contains count changed between steps"
    assert total_present >= half * args.steps  # no false negatives

    # A/B reference: the same step through the direct early-exit kernel (k_bloom_contains)
    L.lib().rbx_tune(b"contains_partition", 0)
    h.contains_dev(dk, cnt.data_ptr() + 24, stream=sptr)
    with Timer(stream) as t_dir:
        for _ in range(3):
            h.contains_dev(dk, cnt.data_ptr() + 24, stream=sptr)
    L.lib().rbx_tune(b"contains_partition", 2)
    direct_ms = t_dir.ms / 3
    assert int(cnt[3].item()) == 4 * (total_present // args.steps), "direct and partitioned counts differ"
    # SURVEY 8(d) C2's second filter: tryInit(448_089_842, 0.01) -> m = 4,294,967,293 bits, k = 7
    # (not a power of two: the exact 63-bit modulo instead of a mask), the same keys
    fn = client.getBloomFilter("bench-c2-tryinit")
    assert fn.tryInit(448_089_842, 0.01)
    assert fn.getSize() == 4_294_967_293 and fn.getHashIterations() == K
    hn = BloomHandle(client, "bench-c2-tryinit")
    cnt.zero_()
    torch.cuda.synchronize()
    with Timer(stream) as t_addn:
        hn.add_dev(device_keys(added.data_ptr(), half, 32), cnt.data_ptr(), stream=sptr)
    hn.contains_dev(dk, cnt.data_ptr() + 8, stream=sptr)
    with Timer(stream) as t_conn:
        for _ in range(3):
            hn.contains_dev(dk, cnt.data_ptr() + 16, stream=sptr)
    assert int(cnt[2].item()) == 3 * int(cnt[1].item()) and int(cnt[1].item()) >= half
    nonpow2 = {"size_bits": 4_294_967_293, "k": K, "tryInit": [448_089_842, 0.01],
               "add_ms": t_addn.ms, "add_keys_per_s_per_gpu": half / (t_addn.ms / 1e3),
               "contains_ms": t_conn.ms / 3, "contains_keys_per_s_per_gpu": n / (t_conn.ms / 3 / 1e3),
               "present_per_step": int(cnt[1].item())}
    hn.close()
    fn.delete()
    hostpath = None if args.no_hostpath or rank != 0 else host_path_rate(client, "bench-c2")

    step_s = max_over_ranks(world, max(kern_ms / 1e3, 0.0))
    keys_all = sum_over_ranks(world, n * args.steps)
    value = keys_all / (step_s * args.steps)
    algo_bytes = n * (32 + K * 8)  # 32 B key + k x 8 B gathered per key
    achieved = algo_bytes / (kern_ms / 1e3) / 1e9
    floor_bytes = n * 32 + SIZE // 8  # what any streaming design must move: the keys and the bitmap once
    # profiles/traffic.json holds PMC counts of 100M-key calls (the default workload); a run with
    # another --keys gets no PMC-derived fields rather than counts of a different call
    pmc_ok = n == C2_PROFILED_KEYS
    traffic = (load_traffic(args.traffic_json, "contains_pipeline", "hbm_bytes_by_class") or
               load_traffic(args.traffic_json, "contains_pipeline")) if pmc_ok else None
    reqf = request_fields(args.traffic_json if pmc_ok else None, "contains_pipeline", kern_ms, gathers_per_s,
                          writes_per_s)
    res = {
        "metric": "Bloom contains keys/sec (whole node), C2: one 2^32-bit filter, k=7, 32-byte keys",
        "value": value, "unit": "keys/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": step_s * 1e3, "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
        "dtype": "u8", "data": "synthetic",
        "config": {"workload": f"C2 RBloomFilter.contains(Collection) of {n / 1e6:g}M random 32-byte keys "
                               "(50% present) vs one 2^32-bit k=7 filter per GPU",
                   "keys_per_gpu": n, "key_bytes": 32, "size_bits": SIZE, "k": K,
                   "parallelism": f"replicas x{world} of one filter (same adds on every rank, bitmap digests "
                                  f"equal), each replica serving its own {n / 1e6:g}M-key contains stream "
                                  "(weak scaling), no data-path collective"},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                     "algorithmic_bytes_per_launch": algo_bytes,
                     # one contains call = the partitioned pipeline's kernels in sequence on one stream
                     "kernel": "contains pipeline: k_bk_stage1<32,8,512,2> + k_bk_emit2<1024,6> + k_bk_probe + "
                               "k_bk_misses + k_bk_final",
                     "kernel_avg_ms": kern_ms,
                     # the pipeline's own floor: keys + bitmap streamed once (3.74 GB per call)
                     "streaming_floor": {"bytes_per_launch": floor_bytes,
                                         "achieved": floor_bytes / (kern_ms / 1e3) / 1e9,
                                         "frac": floor_bytes / (kern_ms / 1e3) / 1e9 / HBM_PEAK_GBS},
                     # the binding limit: memory requests at the L2->EA interface (PMC TCC_EA0_RD/WRREQ),
                     # reads against the measured random-gather request rate at this working set,
                     # writes against the measured streaming-write request rate
                     **reqf,
                     # north-star definition: keys/s x k / measured random-gather peak at this
                     # working set (> 1: early exit and LDS probes avoid most random gathers)
                     "gather_peak_per_s": gathers_per_s, "gather_frac": (n * K / (kern_ms / 1e3)) / gathers_per_s},
        "extra": {"add_keys_per_s_per_gpu": half / (t_add.ms / 1e3), "add_new_keys": n_new,
                  "pmc_fields": "profiles/traffic.json (100M-key calls)" if pmc_ok else
                  f"omitted: PMC profiled at {C2_PROFILED_KEYS} keys per call, this run {n}",
                  "replica_digest": f"{digest:016x}", "replicas_identical": len(set(digests)) == 1,
                  "present_per_step": total_present // args.steps, "wall_s_timed": wall,
                  "contains_direct_kernel_ms": direct_ms,
                  "contains_direct_keys_per_s_per_gpu": n / (direct_ms / 1e3),
                  # the setup add = the partitioned add pipeline (add_partitioned.hip), PMC per call
                  "add_ms": t_add.ms,
                  "add_traffic": (load_traffic(args.traffic_json, "add_pipeline", "hbm_bytes_by_class") or
                                  load_traffic(args.traffic_json, "add_pipeline")) if pmc_ok else None,
                  "add_requests_per_call": load_traffic(args.traffic_json, "add_pipeline", "requests_per_launch")
                  if pmc_ok else None,
                  # of which atomics (PMC TCC_ATOMIC: non-owner counters, stage-1 reservations)
                  "add_atomic_requests_per_call": load_traffic(args.traffic_json, "add_pipeline",
                                                               "atomic_requests_per_launch") if pmc_ok else None,
                  "host_path": hostpath,
                  "c2_tryinit_nonpow2": nonpow2},
    }
    h.close()
    f.delete()
    client.shutdown()
    del added, probe
    torch.cuda.empty_cache()
    return res


# ------------------------------------------------------------------------------------------
# C1 leg: tryInit(1e7, 0.01), add 1M 16-byte keys, contains 1M present + 1M absent
# ------------------------------------------------------------------------------------------
def run_c1(args, world, rank, local):
    import torch

    from redisson_amd import BloomHandle, RedissonClient, device_keys

    stream = torch.cuda.Stream()
    torch.cuda.set_stream(stream)
    sptr = stream.cuda_stream
    client = RedissonClient(local)
    g = torch.Generator(device="cuda")
    g.manual_seed(0x5EED0001)  # replicas: the same adds on every rank, rank-specific absent probes
    keys = torch.randint(0, 256, (1_000_000, 16), dtype=torch.uint8, device="cuda", generator=g)
    g.manual_seed(0x5EED0001 + 1000 * (rank + 1))
    probe = torch.cat([keys, torch.randint(0, 256, (1_000_000, 16), dtype=torch.uint8, device="cuda", generator=g)])
    cnt = torch.zeros(2, dtype=torch.int64, device="cuda")
    t_add = t_con = 0.0
    reps = max(2, args.leg_steps)
    for r in range(args.warmup + reps):  # a fresh filter per rep: add() sees the empty bitmap every time
        name = f"bench-c1-{r}"
        f = client.getBloomFilter(name)
        assert f.tryInit(10_000_000, 0.01)
        h = BloomHandle(client, name)
        cnt.zero_()
        torch.cuda.synchronize()
        with Timer(stream) as ta:
            h.add_dev(device_keys(keys.data_ptr(), 1_000_000, 16), cnt.data_ptr(), stream=sptr)
        with Timer(stream) as tc:
            h.contains_dev(device_keys(probe.data_ptr(), 2_000_000, 16), cnt.data_ptr() + 8, stream=sptr)
        if r >= args.warmup:
            t_add, t_con = t_add + ta.ms, t_con + tc.ms
        added, present = cnt.tolist()
        assert added > 990_000 and present >= 1_000_000
        h.close()
        f.delete()
    client.shutdown()
    add_s = max_over_ranks(world, t_add / reps / 1e3)
    con_s = max_over_ranks(world, t_con / reps / 1e3)
    return {"metric": "C1 Bloom add+contains keys/sec (whole node)", "unit": "keys/s",
            "value": 3_000_000 * world / (add_s + con_s), "reps": reps,
            "add_keys_per_s": 1_000_000 * world / add_s, "contains_keys_per_s": 2_000_000 * world / con_s,
            "add_ms": add_s * 1e3, "contains_ms": con_s * 1e3, "size_bits": 95_850_583, "k": 7,
            "config": "tryInit(1e7,0.01): add 1M 16-byte keys, contains 1M present + 1M absent, keys in HBM, "
                      "per GPU (replicas)"}


# ------------------------------------------------------------------------------------------
# C3: 100k tenant filters tryInit(1e6, 1e-3), sharded by CRC16 slot across the node's GPUs
# ------------------------------------------------------------------------------------------
def run_c3(args, world, rank, local, steps, warmup):
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

    for _ in range(warmup):
        step()
    torch.cuda.synchronize()
    barrier(world)
    with Timer(stream) as t:
        for _ in range(steps):
            step()
    ms = t.ms / steps
    step_s = max_over_ranks(world, ms / 1e3)
    value = sum_over_ranks(world, n) / step_s
    per_rank_tenants = gather_over_ranks(world, nt)
    present = int(counts.sum().item()) / max(warmup + steps, 1)
    add = c3_add_half(args, client, arr, nt, per, k, seg, stream, g, steps, warmup, world) if args.c3_add else None
    del pool
    # request roofline at C3's locality: `per` consecutive keys gather inside one 1.8 MB slice
    tbl = torch.empty(4 << 30, dtype=torch.uint8, device="cuda")
    peak = segment_gather_peak(client, tbl.data_ptr(), tbl.numel(), (size + 7) // 8, per, n, stream)
    del tbl
    wpeak = stream_write_peak(client, 1 << 30, stream)
    if add is not None:
        # the add half against the same request roofline (reads at the segment-gather rate, writes at
        # the stream-write rate): request_frac = its request floor / its call time
        pipe, atj, ams = add.pop("_pipe"), add.pop("_tj"), add.pop("_ms")
        if pipe:
            add["roofline"].update(request_fields(atj, pipe, ams, peak, wpeak))
    algo = n * (16 + k * 8)
    achieved = algo / (ms / 1e3) / 1e9
    # PMC counts of profiles/traffic.json are of the default workload's calls only
    tj = args.traffic_json if (args.keys, args.tenants, world) == (100_000_000, 100_000, 1) else None
    # 180 GB of bitmaps: the slot kernel unless a staged schedule was forced
    slots = args.stage1 is None or args.stage1 == 5
    kname = "k_bloom_contains_q" if slots else "k_bloom_contains_multi"
    kdesc = "k_bloom_contains_q<16,true,2,2>" if slots else f"k_bloom_contains_multi<16,16,{args.stage1}>"
    res = {
        "metric": "Bloom contains keys/sec (whole node), C3: 100k tenant filters tryInit(1e6,1e-3), CRC16-slot sharded",
        "value": value, "unit": "keys/s", "n_gpus": world, "steps": steps, "warmup": warmup,
        "ms_per_step": step_s * 1e3, "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
        "dtype": "u8", "data": "synthetic",
        "config": {"workload": f"C3 one contains(Collection) per tenant, {per} random 16-byte keys each, "
                               f"{nt} of {NT} tenants on this GPU (slot*N/16384), filters at design fill 0.5",
                   "tenants_total": NT, "tenants_this_gpu": nt, "tenants_per_rank": per_rank_tenants,
                   "size_bits": size, "k": k, "keys_per_gpu": n,
                   "parallelism": f"CRC16-slot sharded x{world} (no data-path collective)"},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS,
                     "traffic": load_traffic(tj, kname, "hbm_bytes_by_class") or load_traffic(tj, kname),
                     "kernel": kdesc, "kernel_avg_ms": ms,
                     "request_peak_kind": "k_gather_segments: 4 random loads per key inside its tenant's slice",
                     **request_fields(tj, kname, ms, peak, wpeak)},
        "extra": {"setup_s": setup_s, "present_fraction": present / n},
    }
    if add is not None:
        res["add"] = add
    for h in handles:
        h.close()
    client.shutdown()
    del keys
    torch.cuda.empty_cache()
    return res


def c3_add_half(args, client, arr, nt, per, k, seg, stream, g, steps, warmup, world):
    """C3's add half: one multi-tenant add(Collection) per step -- `per` fresh random
    16-byte keys into each of the rank's tenants (rbx_bloom_add_multi_dev: the 8-byte first-setter
    table by default).  The key window slides by one tenant's worth of keys per step (tenant t of step
    s takes the keys tenant t + s took in step 0), so every step's (tenant, key) pairs are new and the
    adds meet zero bits (~k/2 each at the design fill 0.5).  (A one-key slide keeps 999 of a tenant's
    1,000 keys in the same tenant: after the first step almost nothing is new.)"""
    import ctypes as C

    import torch

    from redisson_amd import device_keys
    from redisson_amd import _lib as L

    n = per * nt
    extra = warmup + steps + 1
    keys = torch.randint(0, 256, (n + extra * per, 16), dtype=torch.uint8, device="cuda", generator=g)
    counts = torch.zeros(nt, dtype=torch.int64, device="cuda")
    sptr = stream.cuda_stream
    windows = [device_keys(keys.data_ptr() + 16 * per * j, n, 16) for j in range(extra)]
    it = [0]

    def step():
        dk = windows[it[0] % len(windows)]
        it[0] += 1
        assert L.lib().rbx_bloom_add_multi_dev(client.ctx, arr, nt, seg.data_ptr(), C.byref(dk), None,
                                                counts.data_ptr(), sptr) == 0

    for _ in range(warmup):
        step()
    torch.cuda.synchronize()
    barrier(world)
    with Timer(stream) as t:
        for _ in range(steps):
            step()
    ms = t.ms / steps
    step_s = max_over_ranks(world, ms / 1e3)
    new = int(counts.sum().item()) / max(warmup + steps, 1)
    # a key + k x 8 B gathered + k x 8 B RMW
    algo = n * (16 + 2 * k * 8)
    tj = args.traffic_json if (args.keys, args.tenants, world) == (100_000_000, 100_000, 1) else None
    tune = dict(kv.split("=") for kv in args.tune.split(",") if "=" in kv)
    mode, seg_path = tune.get("add_multi_table8", "2"), tune.get("add_multi_segment", "1") != "0"
    if mode == "2" and seg_path:  # every tenant of the batch distinct: one workgroup per segment
        pipe = "k_madd_seg"
        path = ("one workgroup per segment (k_madd_seg: tiles of <= 256 keys, LDS first setters, plain word "
                "stores)")
    else:
        pipe = {"0": None}.get(mode, "maddx_pipeline")
        path = {"0": "16-byte epoch table (k_bloom_add_probe + commit)"}.get(
            mode, "optimistic SETBITs + conflict repair (k_maddx_gather + set + claim + reply)")
    del keys
    return {"metric": "Bloom add keys/sec (whole node), C3 tenants: one add(Collection) per tenant",
            "value": sum_over_ranks(world, n) / step_s, "unit": "keys/s", "ms_per_step": step_s * 1e3,
            "keys_per_gpu": n, "new_keys_per_step": new, "steps": steps, "warmup": warmup,
            "path": path, "_pipe": pipe, "_tj": tj, "_ms": ms,
            "roofline": {"bound": "hbm", "achieved": algo / (ms / 1e3) / 1e9, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": algo / (ms / 1e3) / 1e9 / HBM_PEAK_GBS, "algorithmic_bytes_per_launch": algo,
                         "traffic": load_traffic(tj, pipe, "hbm_bytes_by_class") if pipe else None,
                         "requests_per_launch": load_traffic(tj, pipe, "requests_per_launch") if pipe else None,
                         "atomic_requests_per_launch": load_traffic(tj, pipe, "atomic_requests_per_launch")
                         if pipe else None}}


# ------------------------------------------------------------------------------------------
# C5: ordered 90/10 contains/add stream, Zipf(1.0) tenants over the C3 set, 64-byte keys
# ------------------------------------------------------------------------------------------
# the kernels one default C5 call runs per chunk (rbx_bloom_stream_dev with the default tuning)
C5_KERNELS = "k_stream_compact + k_stream_probe8 + k_stream_contains_q + k_stream_final8 + k_stream_walk"


def run_c5(args, world, rank, local, steps, warmup):
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
    extra = warmup + steps + 1 if args.c5_fresh else 0  # the key window slides one key per step
    keys = torch.randint(0, 256, (n + extra, 64), dtype=torch.uint8, device="cuda", generator=g)
    counts = torch.zeros(2, dtype=torch.int64, device="cuda")
    # every command's reply (add(T): newly added, contains(T): present -- the booleans the reference
    # returns, M/RedissonBloomFilter.java:99-102,198-201) is written in the timed step
    replies = torch.empty(n, dtype=torch.uint8, device="cuda")
    arr = (C.c_void_p * nt)(*[h.h.value for h in handles])
    windows = [device_keys(keys.data_ptr() + 64 * j, n, 64) for j in range(max(extra, 1))]
    it = [0]

    def step():
        dk = windows[it[0] % len(windows)]
        it[0] += 1
        assert L.lib().rbx_bloom_stream_dev(client.ctx, arr, nt, kf.data_ptr(), op.data_ptr(), C.byref(dk),
                                             replies.data_ptr() if args.c5_replies else None, counts.data_ptr(),
                                             sptr) == 0

    for _ in range(warmup):
        step()
    torch.cuda.synchronize()
    barrier(world)
    with Timer(stream) as t:
        for _ in range(steps):
            step()
    ms = t.ms / steps
    step_s = max_over_ranks(world, ms / 1e3)
    value = sum_over_ranks(world, n) / step_s
    top = int(torch.bincount(kf.long(), minlength=nt).max().item())
    del pool
    tbl = torch.empty(4 << 30, dtype=torch.uint8, device="cuda")
    # read-request peak: the larger of the tenant-slice gather rate (uniform tenants, one key per
    # slice) and the uniform 512 MiB gather rate -- Zipf-hot tenants gather above the former
    peak = max(segment_gather_peak(client, tbl.data_ptr(), tbl.numel(), 1_797_199, 1, n, stream),
               gather_peak(client, 512 << 20, n, 7, stream, g))
    del tbl
    nadds = int(op.sum().item())
    # a contains = 64 B key + k x 8 B gathered = 144 B, an add +80 B RMW (k x 8 B); plus
    # the 1-byte reply every command writes
    algo = n * (64 + 10 * 8 + 1) + nadds * 10 * 8
    # PMC counts of profiles/traffic.json are of the default workload's calls only
    tj = args.traffic_json if (n, args.tenants, world, args.zipf_s, args.add_fraction, args.c5_fresh) == \
        (100_000_000, 100_000, 1, 1.0, 0.1, 1) else None
    res = {
        "metric": "Bloom mixed contains+add ops/sec (whole node), C5: 90/10 stream, Zipf tenants, 64-byte keys",
        "value": value, "unit": "ops/s", "n_gpus": world, "steps": steps, "warmup": warmup,
        "ms_per_step": step_s * 1e3, "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
        "dtype": "u8", "data": "synthetic",
        "config": {"workload": f"C5 ordered stream of {n} single-key commands ({args.add_fraction:.0%} add) over "
                               f"{nt} tenant filters tryInit(1e6,1e-3) at design fill, Zipf(s={args.zipf_s}) tenants, "
                               "64-byte keys, in-order semantics",
                   "tenants_this_gpu": nt, "ops_per_gpu": n, "hottest_tenant_ops": top,
                   "replies": "one u8 reply per command written to HBM in every timed step" if args.c5_replies
                   else "NOT written (A/B run; not the metric)",
                   "stream": "fresh per step: command i of step s takes key i+s (new (tenant, key) pairs)"
                   if args.c5_fresh else "the same stream every step (adds after the first step re-set their bits)",
                   "parallelism": f"CRC16-slot sharded x{world} (no data-path collective)"},
        "roofline": {"bound": "hbm", "achieved": algo / (ms / 1e3) / 1e9, "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": algo / (ms / 1e3) / 1e9 / HBM_PEAK_GBS,
                     "traffic": load_traffic(tj, "stream_pipeline", "hbm_bytes_by_class") or
                     load_traffic(tj, "stream_pipeline"),
                     "kernel": C5_KERNELS, "kernel_avg_ms": ms,
                     "algorithmic_bytes_per_launch": algo, "adds_per_launch": nadds,
                     "request_peak_kind": "max(k_gather_segments one key per tenant slice, k_gather_probe "
                                          "over 512 MiB) for reads; k_stream_write for writes",
                     **request_fields(tj, "stream_pipeline", ms, peak,
                                      stream_write_peak(client, 1 << 30, stream))},
    }
    for h in handles:
        h.close()
    client.shutdown()
    del keys, kf, op, replies
    torch.cuda.empty_cache()
    return res


# ------------------------------------------------------------------------------------------
# C4: 10k HLLs, PFADD of 16-byte elements, PFCOUNT of all, RCCL max merge
# ------------------------------------------------------------------------------------------
def run_c4(args, world, rank, local, steps, warmup):
    import ctypes as C

    import numpy as np
    import torch

    from redisson_amd import RedissonClient, device_keys
    from redisson_amd import _lib as L

    NH = 10_000
    per = max(1, args.elements // NH)  # elements per HLL per GPU per step (this rank's partition)
    n = NH * per
    stream = torch.cuda.Stream()
    torch.cuda.set_stream(stream)
    sptr = stream.cuda_stream
    client = RedissonClient(local)
    # every step PFADDs fresh elements into 10k newly created HLLs (RedissonHyperLogLog
    # .java:76-81 on keys that do not exist yet): each starts as Redis's sparse string and is promoted
    # to dense inside the timed region, and every register update is a real change.  One set of 10k
    # HLLs per (warmup + timed) step, all created before the timed region.
    nsets = warmup + steps
    sets = []
    for j in range(nsets):
        hs = []
        for i in range(NH):
            hp = C.c_void_p()
            assert L.lib().rbx_hll_open(client.ctx, f"c4-{j}-{i}".encode(), 1, C.byref(hp)) == 0
            hs.append(hp.value)
        sets.append(hs)
    arrs = [(C.c_void_p * NH)(*hs) for hs in sets]
    seg = np.arange(NH + 1, dtype=np.uint64) * np.uint64(per)
    g = torch.Generator(device="cuda")
    g.manual_seed(0x5EED0004 + rank)
    # the element window slides by one HLL's share per step: HLL i of step j takes the elements HLL i + j
    # took in step 0, so no (HLL, element) pair repeats
    el = torch.randint(0, 256, (n + nsets * per, 16), dtype=torch.uint8, device="cuda", generator=g)
    changed = torch.zeros(NH, dtype=torch.int32, device="cuda")
    windows = [device_keys(el.data_ptr() + 16 * per * j, n, 16) for j in range(nsets)]
    it = [0]

    def step():
        j = it[0]
        it[0] += 1
        assert L.lib().rbx_hll_add_multi_dev(client.ctx, arrs[j], NH, None, seg.ctypes.data_as(L.u64p),
                                             C.byref(windows[j]), changed.data_ptr(), sptr) == 0

    for _ in range(warmup):
        step()
    torch.cuda.synchronize()
    barrier(world)
    with Timer(stream) as t:
        for _ in range(steps):
            step()
    ms = t.ms / steps
    changed_last = int((changed != 0).sum().item())
    arr = arrs[-1]
    del el
    nbytes = NH * 16384
    merge = {"allreduce_bytes": nbytes, "nranks_rccl": None, "rccl_max_allreduce_ms": None}
    if world > 1 and not shared_gpu():
        # element-partitioned registers -> ONE RCCL uint8 max all-reduce over xGMI
        import torch.distributed as dist

        uid = (C.c_uint8 * 128)()
        if rank == 0:
            assert L.lib().rbx_rccl_unique_id(uid) == 0
        obj = [bytes(uid)]
        dist.broadcast_object_list(obj, src=0)
        uid = (C.c_uint8 * 128).from_buffer_copy(obj[0])
        assert L.lib().rbx_rccl_init(client.ctx, uid, world, rank) == 0, L.last_error()
        nr, rk = C.c_int(), C.c_int()
        assert L.lib().rbx_rccl_info(client.ctx, C.byref(nr), C.byref(rk)) == 0
        assert L.lib().rbx_hll_allreduce_max(client.ctx, arr, NH) == 0  # warm
        L.lib().rbx_synchronize(client.ctx)
        times = []
        for _ in range(3):
            barrier(world)
            t0 = time.perf_counter()
            assert L.lib().rbx_hll_allreduce_max(client.ctx, arr, NH) == 0
            L.lib().rbx_synchronize(client.ctx)
            times.append(time.perf_counter() - t0)
        mt = max_over_ranks(world, min(times))
        algbw = nbytes / mt / 1e9
        merge.update({"exchange": "RCCL ncclAllReduce(ncclUint8, ncclMax), pack -> all-reduce -> unpack_max",
                      "nranks_rccl": nr.value, "rccl_max_allreduce_ms": mt * 1e3,
                      "algbw_GBps": algbw, "busbw_GBps": algbw * 2 * (world - 1) / world})
    elif world > 1:
        # shared-GPU rehearsal: the same pack / unpack_max exchange, the all-reduce over gloo
        import torch.distributed as dist

        buf = torch.zeros(nbytes, dtype=torch.uint8, device="cuda")
        barrier(world)
        t0 = time.perf_counter()
        assert L.lib().rbx_hll_pack_registers(client.ctx, arr, NH, buf.data_ptr(), sptr) == 0
        torch.cuda.synchronize()
        host = buf.cpu()
        dist.all_reduce(host, op=dist.ReduceOp.MAX)
        buf.copy_(host.cuda())
        assert L.lib().rbx_hll_unpack_max_registers(client.ctx, arr, NH, buf.data_ptr(), sptr) == 0
        torch.cuda.synchronize()
        mt = max_over_ranks(world, time.perf_counter() - t0)
        merge.update({"exchange": "gloo (shared-GPU rehearsal: RCCL needs one GPU per rank)",
                      "exchange_ms": mt * 1e3})
    out = np.zeros(NH, np.uint64)
    t0 = time.perf_counter()
    assert L.lib().rbx_hll_count_each_handles(client.ctx, arr, NH, out.ctypes.data_as(L.u64p)) == 0
    count_ms = (time.perf_counter() - t0) * 1e3
    peak_gbs = stream_read_peak(client, 8 << 30, stream)
    step_s = max_over_ranks(world, ms / 1e3)
    value = sum_over_ranks(world, n) / step_s
    achieved = n * 16 / (ms / 1e3) / 1e9
    res = {
        "metric": "HLL PFADD elems/sec (whole node), C4: 10k HLLs, 16-byte elements",
        "value": value, "unit": "elems/s", "n_gpus": world, "steps": steps, "warmup": warmup,
        "ms_per_step": step_s * 1e3, "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
        "dtype": "u8", "data": "synthetic",
        "config": {"workload": f"C4 PFADD {per} fresh 16-byte elements into each of 10k newly created HLLs per "
                               f"GPU per step (sparse -> dense promotion inside the timed region)",
                   "elements_per_gpu": n, "parallelism": f"element-partitioned x{world}"},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS,
                     "traffic": (load_traffic(args.traffic_json, "k_hll_pfadd", "hbm_bytes_by_class") or
                                 load_traffic(args.traffic_json, "k_hll_pfadd"))
                     if (args.elements, world) == (1_000_000_000, 1) else None,
                     # the step: PFADD registers (k_hll_pfadd) + the sparse strings of the fresh keys
                     # replayed to their promotion (k_hll_sparse_replay); achieved over the whole step
                     "kernel": "k_hll_pfadd<16> + k_hll_sparse_replay<16>", "kernel_avg_ms": ms,
                     # elems/s x 16 B / the measured HBM stream-read peak
                     "stream_read_peak_GBps": peak_gbs, "stream_frac": achieved / peak_gbs},
        "extra": {"pfcount_10k_ms": count_ms, "mean_count": float(out.mean()), "merge": merge,
                  "changed_replies_last_step": changed_last},
    }
    for hs in sets:
        for hp in hs:
            L.lib().rbx_hll_close(hp)
    client.shutdown()
    torch.cuda.empty_cache()
    return res


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(self_launch(args))
    world, rank, local = dist_setup(args)
    if args.stage1 is not None:
        from redisson_amd import _lib as L

        assert L.lib().rbx_tune(b"contains_stage1", args.stage1) == 0
        # a forced staged schedule applies to multi-tenant calls too (no automatic slot kernel)
        assert L.lib().rbx_tune(b"contains_multi_slots", 1 if args.stage1 == 5 else 0) == 0
    for kv in filter(None, args.tune.split(",")):
        from redisson_amd import _lib as L

        key, val = kv.split("=")
        if key == "c5_replies":  # bench-side A/B switch (not an engine knob): C5 timed without replies
            args.c5_replies = int(val)
            continue
        if key == "c5_fresh":  # bench-side switch: a fresh stream per step (see --c5-fresh)
            args.c5_fresh = int(val)
            continue
        assert L.lib().rbx_tune(key.encode(), int(val)) == 0, kv
    log(f"[bench] rank {rank}/{world} workload {args.workload}")
    if args.dry_run:
        census = gather_over_ranks(world, os.getpid())
        if rank == 0:
            print(json.dumps({"dry_run": True, "n_gpus": world, "ranks": len(census), "pids": census}), flush=True)
        if world > 1:
            import torch.distributed as dist

            dist.destroy_process_group()
        return
    if args.workload == "c2":
        res = run_c2(args, world, rank, local)
        legs = [] if args.legs == "none" else [x for x in args.legs.split(",") if x]
        ls, lw = min(args.steps, args.leg_steps), min(args.warmup, 2)
        res["legs"] = {}
        for leg in legs:
            if leg not in ("c1", "c3", "c4", "c5"):
                raise SystemExit(f"unknown leg {leg}")
        for leg in legs:
            log(f"[bench] rank {rank} leg {leg}")
            # a leg that raises (on every rank alike, e.g. a failed RCCL init) is reported in the
            # line instead of taking the C2 headline down with it
            try:
                if leg == "c1":
                    res["legs"]["c1"] = run_c1(args, world, rank, local)
                elif leg == "c3":
                    res["legs"]["c3"] = run_c3(args, world, rank, local, ls, lw)
                elif leg == "c5":
                    res["legs"]["c5"] = run_c5(args, world, rank, local, ls, lw)
                else:
                    res["legs"]["c4"] = run_c4(args, world, rank, local, ls, lw)
            except Exception as e:  # noqa: BLE001
                import traceback

                traceback.print_exc()
                res["legs"][leg] = {"error": f"{type(e).__name__}: {e}"}
        if rank == 0 and world == 1 and not args.no_cpu_baseline:
            res["cpu_baseline"] = cpu_baseline(args.cpu_seconds)
    elif args.workload == "c4":
        res = run_c4(args, world, rank, local, args.steps, args.warmup)
    elif args.workload == "c5":
        res = run_c5(args, world, rank, local, args.steps, args.warmup)
    else:
        res = run_c3(args, world, rank, local, args.steps, args.warmup)
    if rank == 0:
        res.setdefault("cpu_baseline", None)
        print(json.dumps(res), flush=True)
    if world > 1:
        import torch.distributed as dist

        dist.destroy_process_group()


if __name__ == "__main__":
    main()
