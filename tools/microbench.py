#!/usr/bin/env python3
"""Microbenchmarks on one MI355X (run through gpurun).

  gather  : random 4-byte gather rate vs working-set size (the Bloom roofline)
  stage1  : contains early-exit width A/B, interleaved rounds in one process
  sizes   : contains throughput vs filter size (C1 12 MB, C3 1.8 MB, C2 512 MiB)
  add     : add throughput
Prints one JSON object per measurement.
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from redisson_amd import BloomHandle, RedissonClient, device_keys  # noqa: E402
from redisson_amd import _lib as L  # noqa: E402


def timed(stream, fn, reps):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(reps):
        fn()
    e1.record(stream)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def murmur64a_16(mat):
    """MurmurHash64A (seed 0xadc83b19, redis hyperloglog.c) of 16-byte rows, vectorized (numpy u64)."""
    import numpy as np

    m, r = np.uint64(0xC6A4A7935BD1E995), np.uint64(47)
    with np.errstate(over="ignore"):
        h = np.uint64(0xADC83B19) ^ (np.uint64(16) * m)
        h = np.full(mat.shape[0], h, dtype=np.uint64)
        for b in range(2):
            k = mat[:, 8 * b:8 * b + 8].copy().view(np.uint64).reshape(-1)
            k = k * m
            k ^= k >> r
            k = k * m
            h ^= k
            h = h * m
        h ^= h >> r
        h = h * m
        h ^= h >> r
    return h


def murmur_count1_elements(indexes, rng):
    """One 16-byte element per register index with hllPatLen count 1 (bit 14 of the hash set)."""
    import numpy as np

    want, found = set(int(i) for i in indexes), {}
    while len(found) < len(want):
        cand = rng.integers(0, 256, size=(1 << 20, 16), dtype=np.uint8)
        h = murmur64a_16(cand)
        ok = ((h >> np.uint64(14)) & np.uint64(1)) == np.uint64(1)
        for j in np.nonzero(ok)[0]:
            i = int(h[j] & np.uint64(16383))
            if i in want and i not in found:
                found[i] = cand[j]
    return np.stack([found[i] for i in sorted(want)])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("what", nargs="*", default=["gather", "stage1", "sizes", "add"])
    ap.add_argument("--keys", type=int, default=100_000_000)
    ap.add_argument("--tiny-keys", type=int, default=16384)  # smallbatch: host_tiny_keys
    ap.add_argument("--seg-keys", type=int, default=256)  # smallbatch: add_single_seg_keys
    a = ap.parse_args()
    for kv in filter(None, os.environ.get("RBX_TUNE", "").split(",")):  # process-wide rbx_tune settings
        key, val = kv.split("=")
        assert L.lib().rbx_tune(key.encode(), int(val)) == 0, kv
    stream = torch.cuda.Stream()
    torch.cuda.set_stream(stream)
    sp = stream.cuda_stream
    client = RedissonClient(0)
    g = torch.Generator(device="cuda")
    g.manual_seed(1)
    n = a.keys
    keys = torch.randint(0, 256, (n, 32), dtype=torch.uint8, device="cuda", generator=g)
    sink = torch.zeros(1, dtype=torch.int32, device="cuda")

    if "gather" in a.what:
        for mb in [2, 8, 32, 64, 128, 192, 256, 384, 512, 1024, 4096, 16384]:
            tb = torch.empty(mb << 20, dtype=torch.uint8, device="cuda")
            tb.random_(0, 255, generator=g)
            f = lambda: L.lib().rbx_bench_gather(client.ctx, tb.data_ptr(), tb.numel(), n, 7, sink.data_ptr(), sp)
            f()
            ms = timed(stream, f, 3)
            print(json.dumps({"bench": "gather", "table_MiB": mb, "ms": ms, "gathers_per_s": n * 7 / (ms / 1e3)}),
                  flush=True)
            del tb

    if "regions" in a.what:
        tb = torch.empty(512 << 20, dtype=torch.uint8, device="cuda")
        tb.random_(0, 255, generator=g)
        lanes = 54_000_000  # survivors of stage 1 at C2, 6 remaining loads each
        for rmb in [1, 2, 4, 8]:
            for grid in [2048, 4096, 8192]:
                f = lambda: L.lib().rbx_bench_gather_regions(client.ctx, tb.data_ptr(), tb.numel(), rmb << 20, lanes,
                                                             grid, sink.data_ptr(), sp)
                f()
                ms = timed(stream, f, 3)
                print(json.dumps({"bench": "gather_regions", "region_MiB": rmb, "grid": grid, "ms": ms,
                                  "gathers_per_s": lanes * 6 / (ms / 1e3)}), flush=True)
        del tb

    if "slices" in a.what:
        # the L2-sliced probe: 324M 8-byte entries (C2's survivor pairs) bucketed by bitmap slice,
        # each testing one word of its slice; vs the random gather over the whole 512 MiB
        bm = torch.empty(512 << 20, dtype=torch.uint8, device="cuda")
        bm.random_(0, 255, generator=g)
        total = 324_000_000
        ent = torch.randint(0, 2**31 - 1, (total * 2,), dtype=torch.int32, device="cuda", generator=g)
        for slice_mb in [1, 2, 4, 8]:
            nb = (512 << 20) // (slice_mb << 20)
            per = total // nb
            for grid in [2048, 4096, 8192]:
                f = lambda: L.lib().rbx_bench_slice_probe(client.ctx, ent.data_ptr(), per, nb, bm.data_ptr(),
                                                          slice_mb << 20, grid, sink.data_ptr(), sp)
                f()
                ms = timed(stream, f, 5)
                print(json.dumps({"bench": "slice_probe", "slice_MiB": slice_mb, "grid": grid, "entries": per * nb,
                                  "ms": ms, "entries_per_s": per * nb / (ms / 1e3),
                                  "stream_GBps": per * nb * 8 / (ms / 1e3) / 1e9}), flush=True)
        f = lambda: L.lib().rbx_bench_gather(client.ctx, bm.data_ptr(), bm.numel(), total // 7, 7, sink.data_ptr(), sp)
        f()
        ms = timed(stream, f, 3)
        print(json.dumps({"bench": "gather_512MiB", "gathers": total, "ms": ms, "gathers_per_s": total / (ms / 1e3)}),
              flush=True)
        del ent, bm

    if "hostpath" in a.what:
        import ctypes as C
        import time as T

        import numpy as np

        from redisson_amd import Arena
        nh = 20_000_000
        fb = client.getBloomFilter("hp")
        fb.tryInitRaw(1 << 32, 7)
        host = np.random.default_rng(3).integers(0, 256, size=(nh, 32), dtype=np.uint8)
        p = C.c_void_p()
        assert L.lib().rbx_host_alloc(nh * 32, C.byref(p)) == 0
        pinned = np.ctypeslib.as_array((C.c_uint8 * (nh * 32)).from_address(p.value)).reshape(nh, 32)
        pinned[:] = host
        for label, arr in [("pageable", host), ("pinned", pinned)]:
            a_ = Arena.fixed(arr)
            fb.add(a_) if label == "pageable" else None
            for _ in range(2):
                t0 = T.perf_counter()
                c = fb.contains(a_)
                dt = T.perf_counter() - t0
            print(json.dumps({"bench": "host_contains", "memory": label, "keys": nh, "s": dt,
                              "keys_per_s": nh / dt, "present": c}), flush=True)
        L.lib().rbx_host_free(p)
        fb.delete()

    if "partition" in a.what:
        cnt = torch.zeros(8, dtype=torch.int64, device="cuda")
        for name, size, k, n_add in [("C2_2^32", 1 << 32, 7, n // 2), ("C2_twin", 4294967293, 7, n // 2),
                                     ("C1", 95850583, 7, 10_000_000)]:
            fb = client.getBloomFilter("pc-" + name)
            fb.tryInitRaw(size, k)
            h = BloomHandle(client, "pc-" + name)
            h.add_dev(device_keys(keys.data_ptr(), n_add, 32), cnt.data_ptr(), stream=sp)
            torch.cuda.synchronize()
            dk = device_keys(keys.data_ptr(), n, 32)
            res = {0: [], 1: []}
            counts = {}
            for rnd in range(5):
                for mode in res:
                    L.lib().rbx_tune(b"contains_partition", mode)
                    cnt[1].zero_()
                    res[mode].append(timed(stream, lambda: h.contains_dev(dk, cnt.data_ptr() + 8, stream=sp), 2))
                    counts[mode] = int(cnt[1].item())
            assert counts[0] == counts[1], counts
            for mode, v in res.items():
                med = statistics.median(v)
                print(json.dumps({"bench": "contains_partition", "filter": name, "mode": mode, "ms_median": med,
                                  "ms_min": min(v), "keys_per_s": n / (med / 1e3), "present_x2": counts[mode]}),
                      flush=True)
            L.lib().rbx_tune(b"contains_partition", 2)
            h.close()
            fb.delete()

    if "pc2" in a.what:
        # C2 contains through the default (partitioned) path only: a short run for PMC passes
        cnt = torch.zeros(8, dtype=torch.int64, device="cuda")
        fb = client.getBloomFilter("pc2")
        fb.tryInitRaw(1 << 32, 7)
        h = BloomHandle(client, "pc2")
        h.add_dev(device_keys(keys.data_ptr(), n // 2, 32), cnt.data_ptr(), stream=sp)
        dk = device_keys(keys.data_ptr(), n, 32)
        ms = timed(stream, lambda: h.contains_dev(dk, cnt.data_ptr() + 8, stream=sp), 3)
        print(json.dumps({"bench": "pc2", "ms": ms, "keys_per_s": n / (ms / 1e3)}), flush=True)
        h.close()
        fb.delete()

    if "psizes" in a.what:
        # direct vs partitioned contains and add over filter sizes, at C2's fill (86 bits per added key)
        cnt = torch.zeros(4, dtype=torch.int64, device="cuda")
        for lg in [26, 27, 28, 29, 30, 31, 32]:
            size = 1 << lg
            n_add = min(n // 2, size // 86)
            res = {}
            for mode in (0, 1):
                L.lib().rbx_tune(b"add_partition", mode)
                L.lib().rbx_tune(b"contains_partition", mode)
                fb = client.getBloomFilter(f"ps-{lg}-{mode}")
                fb.tryInitRaw(size, 7)
                h = BloomHandle(client, f"ps-{lg}-{mode}")
                cnt.zero_()
                add_ms = timed(stream, lambda: h.add_dev(device_keys(keys.data_ptr(), n_add, 32), cnt.data_ptr(),
                                                         stream=sp), 1)
                dk = device_keys(keys.data_ptr(), n, 32)
                h.contains_dev(dk, cnt.data_ptr() + 8, stream=sp)
                c_ms = statistics.median([timed(stream, lambda: h.contains_dev(dk, cnt.data_ptr() + 16, stream=sp), 2)
                                          for _ in range(3)])
                res[mode] = (add_ms, c_ms, int(cnt[0].item()), int(cnt[1].item()))
                h.close()
                fb.delete()
            assert res[0][2:] == res[1][2:], res
            print(json.dumps({"bench": "psizes", "size_log2": lg, "added": n_add,
                              "add_ms_direct": res[0][0], "add_ms_part": res[1][0],
                              "contains_ms_direct": res[0][1], "contains_ms_part": res[1][1]}), flush=True)
        L.lib().rbx_tune(b"add_partition", 2)
        L.lib().rbx_tune(b"contains_partition", 2)

    if "pa2" in a.what:
        # one default-path add of n/2 keys into an empty 2^32-bit filter (short run for PMC passes)
        cnt = torch.zeros(2, dtype=torch.int64, device="cuda")
        fb = client.getBloomFilter("pa2")
        fb.tryInitRaw(1 << 32, 7)
        h = BloomHandle(client, "pa2")
        ms = timed(stream, lambda: h.add_dev(device_keys(keys.data_ptr(), n // 2, 32), cnt.data_ptr(), stream=sp), 1)
        print(json.dumps({"bench": "pa2", "ms": ms, "keys_per_s": n // 2 / (ms / 1e3), "new": int(cnt[0].item())}))
        h.close()
        fb.delete()

    if "padiag" in a.what:
        # partitioned add with its diagnostic switches (wrong results, timing only)
        cnt = torch.zeros(2, dtype=torch.int64, device="cuda")
        m = n // 2
        res = {0: [], 4: []}
        for rnd in range(3):
            for dg in res:
                L.lib().rbx_tune(b"add_partition_diag", dg)
                fb = client.getBloomFilter(f"pd-{rnd}-{dg}")
                fb.tryInitRaw(1 << 32, 7)
                h = BloomHandle(client, f"pd-{rnd}-{dg}")
                res[dg].append(timed(stream, lambda: h.add_dev(device_keys(keys.data_ptr(), m, 32), cnt.data_ptr(),
                                                               stream=sp), 1))
                h.close()
                fb.delete()
        L.lib().rbx_tune(b"add_partition_diag", 0)
        for dg, v in res.items():
            print(json.dumps({"bench": "add_partition_diag", "diag": dg, "ms_median": statistics.median(v)}), flush=True)

    if "smallbatch" in a.what:
        # per-call latency of the batch sizes Redisson callers send (contains(T) / add(T) are one key) on the
        # C1 filter (tryInit(1e7, 0.01), 1M keys added): the synchronous by-name host-arena calls
        # (rbx_bloom_contains / rbx_bloom_add: name lookup, staging upload, kernel, result readback) and
        # the handle calls on keys already in HBM plus a stream sync; median wall time of 300 calls
        import time

        import numpy as np

        from redisson_amd import Arena

        fb = client.getBloomFilter("sb")
        fb.tryInit(10_000_000, 0.01)
        h = BloomHandle(client, "sb")
        base = torch.randint(0, 256, (1_000_000, 16), dtype=torch.uint8, device="cuda", generator=g)
        cnt = torch.zeros(2, dtype=torch.int64, device="cuda")
        h.add_dev(device_keys(base.data_ptr(), 1_000_000, 16), cnt.data_ptr(), stream=sp)
        torch.cuda.synchronize()
        rng = np.random.default_rng(5)
        hostkeys = base[:65536].cpu().numpy()
        fresh = torch.randint(0, 256, (2 * 320 * 4096, 16), dtype=torch.uint8, device="cuda", generator=g)
        tiny_keys, seg_keys = a.tiny_keys, a.seg_keys
        assert L.lib().rbx_tune(b"host_tiny_keys", tiny_keys) == 0
        assert L.lib().rbx_tune(b"add_single_seg_keys", seg_keys) == 0
        for nb in [1, 16, 64, 256, 1024, 4096, 65536]:
            res = {}
            present = Arena.fixed(hostkeys[:nb])
            adds = [Arena.fixed(rng.integers(0, 256, size=(nb, 16), dtype=np.uint8)) for _ in range(20)]
            # adds of new keys: every call (warmup and timed, and every variant below) its own keys
            hpool = rng.integers(0, 256, size=(5 * 320 * nb, 16), dtype=np.uint8) if nb <= 4096 else None

            def add_host_new(v):
                ars = [Arena.fixed(hpool[(v * 320 + j) * nb:(v * 320 + j + 1) * nb]) for j in range(320)]
                return lambda i: fb.add(ars[i])

            def add_dev_new(v):
                return lambda i: (h.add_dev(device_keys(fresh.data_ptr() + 16 * (v * 320 + i) * min(nb, 4096), nb, 16),
                                            cnt.data_ptr(), stream=sp), stream.synchronize())

            calls = {
                "contains_host": lambda i: fb.contains(present),
                "add_host": lambda i: fb.add(adds[i % 20]),  # re-adds: 20 batches in turn
                "contains_dev": lambda i: (h.contains_dev(device_keys(base.data_ptr(), nb, 16), cnt.data_ptr() + 8,
                                                          stream=sp), stream.synchronize()),
            }
            if nb <= 4096:
                calls["add_host_new"] = add_host_new(0)
                calls["add_dev_new"] = add_dev_new(0)
            if nb == 1:  # the Python object forms (one encoded key, no arena)
                one_new = [bytes(r) for r in rng.integers(0, 256, size=(320, 16), dtype=np.uint8)]
                calls["contains_one_object"] = lambda i: fb.contains(bytes(hostkeys[0]))
                calls["add_one_object_new"] = lambda i: fb.add(one_new[i])
            if nb >= 4 and nb <= 4096:  # one multi-tenant host call over 4 filters (an RBatch of 4 collections)
                from redisson_amd import bloom_add_multi, bloom_contains_multi

                mh = []
                for t in range(4):
                    mf = client.getBloomFilter(f"sb-m{t}")
                    mf.tryInit(1_000_000, 0.01)
                    mh.append(BloomHandle(client, f"sb-m{t}"))
                seg = np.array([0, nb // 4, nb // 2, 3 * nb // 4, nb], np.uint64)
                calls["contains_multi4_host"] = lambda i: bloom_contains_multi(client, mh, seg, present)
                calls["add_multi4_host"] = lambda i: bloom_add_multi(client, mh, seg, adds[i % 20])
            if nb <= 256:  # PFADD of nb host elements: a dense HLL, and a sparse one (a new HLL every 20 calls)
                hd = client.getHyperLogLog(f"sb-hd-{nb}")
                hd.addAll(Arena.fixed(rng.integers(0, 256, size=(200_000, 16), dtype=np.uint8)))
                calls["pfadd_dense_host"] = lambda i: hd.addAll(adds[i % 20])
                calls["pfadd_sparse_host"] = lambda i: client.getHyperLogLog(f"sb-hs-{nb}-{i // 20}").addAll(
                    adds[i % 20])
                calls["pfcount_dense_host"] = lambda i: hd.count()
                if nb == 1:
                    calls["pfadd_one_object"] = lambda i: hd.add(one_new[i])
            # the tiny path (bloom_host_tiny, <= host_tiny_keys keys) and the one-segment add
            # (add_single_seg_keys) against the r05 paths
            def off(fn, *knobs):
                def g(i):
                    for kb in knobs:
                        L.lib().rbx_tune(kb, 0)
                    try:
                        return fn(i)
                    finally:
                        L.lib().rbx_tune(b"host_tiny_keys", tiny_keys)
                        L.lib().rbx_tune(b"add_single_seg_keys", seg_keys)
                        L.lib().rbx_tune(b"add_one_key", 1)
                        L.lib().rbx_tune(b"host_tiny_spin", 1)
                return g

            if nb <= 16384:
                calls["contains_host_tiny_off"] = off(calls["contains_host"], b"host_tiny_keys")
                calls["add_host_tiny_off"] = off(calls["add_host"], b"host_tiny_keys")
                calls["add_host_seg_off"] = off(calls["add_host"], b"add_single_seg_keys")
                calls["add_host_r05"] = off(calls["add_host"], b"host_tiny_keys", b"add_single_seg_keys")
            if nb <= 4096:
                calls["add_host_new_seg_off"] = off(add_host_new(1), b"add_single_seg_keys")
                calls["add_host_new_r05"] = off(add_host_new(2), b"host_tiny_keys", b"add_single_seg_keys")
                calls["add_dev_new_seg_off"] = off(add_dev_new(1), b"add_single_seg_keys")
            if nb == 1:  # the one-segment kernel instead of k_bloom_add_one
                calls["add_host_new_one_off"] = off(add_host_new(3), b"add_one_key")
                calls["add_host_new_spin_off"] = off(add_host_new(4), b"host_tiny_spin")
                calls["contains_host_spin_off"] = off(calls["contains_host"], b"host_tiny_spin")
                calls["add_dev_new_one_off"] = off(add_dev_new(3), b"add_one_key")
            for kind, fn in calls.items():
                for i in range(20):
                    fn(i)
                ts = []
                for i in range(20, 320):
                    t0 = time.perf_counter()
                    fn(i)
                    ts.append(time.perf_counter() - t0)
                res[kind] = round(statistics.median(ts) * 1e6, 1)
            print(json.dumps({"bench": "smallbatch", "keys": nb, "median_us": res}), flush=True)
        h.close()
        fb.delete()

    if "regstamp" in a.what:
        # region-pass phase times (add_partition_diag 64, exact results; the profiling build:
        # RBX_LIB_PATH=redisson_amd/librbx_diag.so), C2 add of n/2 keys into an empty 2^32-bit filter;
        # summed over blocks, in ms of one CU's wave 0 (s_memtime ticks at 100 MHz) per block slot
        import ctypes as C

        cnt = torch.zeros(2, dtype=torch.int64, device="cuda")
        m = n // 2
        names = ["top_wait", "setup", "prefetch", "pass1", "pass2", "table", "owners", "writeback"]
        for rk in (2, 2):
            assert L.lib().rbx_tune(b"add_partition_diag", 64) == 0
            fb = client.getBloomFilter(f"rs-{rk}")
            fb.tryInitRaw(1 << 32, 7)
            h = BloomHandle(client, f"rs-{rk}")
            buf = (C.c_ulonglong * 16)()
            L.lib().rbx_bench_add_stamps(client.ctx, buf, 16)  # clear
            cnt.zero_()
            ms = timed(stream, lambda: h.add_dev(device_keys(keys.data_ptr(), m, 32), cnt.data_ptr(), stream=sp), 1)
            assert L.lib().rbx_bench_add_stamps(client.ctx, buf, 16) == 0
            tot = sum(buf[:8])
            rtot = sum(buf[8:12])
            rb = ["load_count", "scan_reserve", "place", "store"]
            print(json.dumps({"bench": "regstamp", "region_kernel": rk, "add_ms": ms, "new": int(cnt[0].item()),
                              "share": {nm: buf[i] / tot for i, nm in enumerate(names)},
                              "ticks_per_block_slot": tot / 512,
                              "rebucket_share": {nm: buf[8 + i] / max(rtot, 1) for i, nm in enumerate(rb)},
                              "rebucket_ticks_per_cu": rtot / 256}), flush=True)
            h.close()
            fb.delete()
        L.lib().rbx_tune(b"add_partition_diag", 0)

    if "pcstamp" in a.what:
        # partitioned contains phase times (contains_partition_flags 64, exact results), C2 contains
        # of n keys against a 2^32-bit filter holding n/2: emit2 (count, scan/reserve, place, store)
        # and probe (top wait, probe loop, miss records) shares of block time
        import ctypes as C

        cnt = torch.zeros(8, dtype=torch.int64, device="cuda")
        fb = client.getBloomFilter("pcs")
        fb.tryInitRaw(1 << 32, 7)
        h = BloomHandle(client, "pcs")
        h.add_dev(device_keys(keys.data_ptr(), n // 2, 32), cnt.data_ptr(), stream=sp)
        dk = device_keys(keys.data_ptr(), n, 32)
        buf = (C.c_ulonglong * 16)()
        for fl in (0, 64, 0, 64):
            assert L.lib().rbx_tune(b"contains_partition_flags", fl) == 0
            L.lib().rbx_bench_add_stamps(client.ctx, buf, 16)  # clear
            cnt[2:].zero_()
            ms = timed(stream, lambda: h.contains_dev(dk, cnt.data_ptr() + 16, stream=sp), 1)
            assert L.lib().rbx_bench_add_stamps(client.ctx, buf, 16) == 0
            etot = sum(buf[:4])
            ptot = sum(buf[8:11])
            print(json.dumps({"bench": "pcstamp", "flags": fl, "ms": ms, "present": int(cnt[2].item()),
                              "emit2_share": {nm: buf[i] / max(etot, 1) for i, nm in
                                              enumerate(["count", "scan_reserve", "place", "store"])},
                              "emit2_ticks_per_cu": etot / 256,
                              "probe_share": {nm: buf[8 + i] / max(ptot, 1) for i, nm in
                                              enumerate(["top_wait", "probe", "miss_records"])},
                              "probe_ticks_per_cu": ptot / 256}), flush=True)
        L.lib().rbx_tune(b"contains_partition_flags", 0)
        h.close()
        fb.delete()

    if "hllfirst" in a.what:
        # C4-shaped PFADD batch into fresh HLLs (created sparse: the string replay runs until each
        # promotes) vs the same batch again (dense keys), 10k HLLs x `per` 16-byte elements
        import ctypes as C

        import numpy as np

        NH = 10_000
        # warm-up on other keys (module loading, pool chunks), deleted again: the measured keys
        # then reuse those pool slots (zeroed together on the first allocation)
        wel = torch.randint(0, 256, (NH * 10, 16), dtype=torch.uint8, device="cuda")
        wh = []
        for i in range(NH):
            hp = C.c_void_p()
            assert L.lib().rbx_hll_open(client.ctx, f"hw-{i}".encode(), 1, C.byref(hp)) == 0
            wh.append(hp.value)
        warr = (C.c_void_p * NH)(*wh)
        wseg = np.arange(NH + 1, dtype=np.uint64) * np.uint64(10)
        wch = torch.zeros(NH, dtype=torch.int32, device="cuda")
        wdk = device_keys(wel.data_ptr(), NH * 10, 16)
        assert L.lib().rbx_hll_add_multi_dev(client.ctx, warr, NH, None, wseg.ctypes.data_as(L.u64p), C.byref(wdk),
                                             wch.data_ptr(), sp) == 0
        torch.cuda.synchronize()
        for hp in wh:
            L.lib().rbx_hll_close(C.c_void_p(hp))
        for i in range(NH):
            client.getHyperLogLog(f"hw-{i}").delete()
        for per in (1_000, 10_000):
            hs = []
            for i in range(NH):
                hp = C.c_void_p()
                assert L.lib().rbx_hll_open(client.ctx, f"hf-{per}-{i}".encode(), 1, C.byref(hp)) == 0
                hs.append(hp.value)
            arr = (C.c_void_p * NH)(*hs)
            seg = np.arange(NH + 1, dtype=np.uint64) * np.uint64(per)
            el = torch.randint(0, 256, (NH * per, 16), dtype=torch.uint8, device="cuda")
            changed = torch.zeros(NH, dtype=torch.int32, device="cuda")
            dk = device_keys(el.data_ptr(), NH * per, 16)
            res = []
            for _ in range(3):
                res.append(timed(stream, lambda: L.lib().rbx_hll_add_multi_dev(
                    client.ctx, arr, NH, None, seg.ctypes.data_as(L.u64p), C.byref(dk), changed.data_ptr(), sp), 1))
            buf = np.zeros(16 + 12288, np.uint8)
            ln = C.c_uint64()
            assert L.lib().rbx_hll_export_enc(client.ctx, f"hf-{per}-0".encode(), 2, buf.ctypes.data_as(L.u8p),
                                              buf.size, C.byref(ln)) == 0
            print(json.dumps({"bench": "hllfirst", "hlls": NH, "per": per, "first_ms": res[0], "again_ms": res[1:],
                              "hll0_encoding": "sparse" if buf[4] else "dense", "hll0_bytes": int(ln.value)}),
                  flush=True)
            for hp in hs:
                L.lib().rbx_hll_close(C.c_void_p(hp))
            del el

    if "hllruns" in a.what:
        # the sparse replay's residual case.  10k fresh HLLs, three multi-key PFADD
        # batches (tests/test_hll_gpu.py::test_sparse_first_batches_many_keys at 10k keys): 1,000 and
        # 150 random 16-byte elements per key (the normalized-string shortcut), then 20 per key plus,
        # on every third key, five elements raising registers 5000..5004 to 1 in descending order
        # (a run of five equal registers: element-by-element replay).  Time of each batch.
        import ctypes as C

        import numpy as np

        NH = 10_000
        rng = np.random.default_rng(67)
        run5 = murmur_count1_elements(range(5000, 5005), rng)[::-1]
        hs = []
        for i in range(NH):
            hp = C.c_void_p()
            assert L.lib().rbx_hll_open(client.ctx, f"hr-{i}".encode(), 1, C.byref(hp)) == 0
            hs.append(hp.value)
        arr = (C.c_void_p * NH)(*hs)
        out = {"bench": "hllruns", "hlls": NH}
        for tag, per, extra in (("first", 1000, False), ("second", 150, False), ("third", 20, True)):
            els = [rng.integers(0, 256, size=(per, 16), dtype=np.uint8) for _ in range(NH)]
            if extra:
                for i in range(0, NH, 3):
                    els[i] = np.concatenate([els[i], run5])
            seg = np.zeros(NH + 1, np.uint64)
            seg[1:] = np.cumsum([len(e) for e in els])
            el = torch.from_numpy(np.concatenate(els)).cuda()
            changed = torch.zeros(NH, dtype=torch.int32, device="cuda")
            dk = device_keys(el.data_ptr(), int(seg[-1]), 16)
            torch.cuda.synchronize()
            out[tag + "_ms"] = timed(stream, lambda: L.lib().rbx_hll_add_multi_dev(
                client.ctx, arr, NH, None, seg.ctypes.data_as(L.u64p), C.byref(dk), changed.data_ptr(), sp), 1)
            buf = np.zeros(16 + 12288, np.uint8)
            ln = C.c_uint64()
            assert L.lib().rbx_hll_export_enc(client.ctx, b"hr-0", 2, buf.ctypes.data_as(L.u8p), buf.size,
                                              C.byref(ln)) == 0
            out[tag + "_hll0"] = ("sparse" if buf[4] else "dense", int(ln.value))
        out["third_over_first"] = out["third_ms"] / out["first_ms"]
        print(json.dumps(out), flush=True)
        for hp in hs:
            L.lib().rbx_hll_close(C.c_void_p(hp))
        # first batches that leave the shortcut: runs of five in a 1,000-element batch, and batches
        # near the size limit (the B bound fails, the fewest-bytes encoding still fits)
        for per, runs in ((1000, False), (1000, True), (1300, False), (1500, False), (1700, False)):
            hs = []
            for i in range(NH):
                hp = C.c_void_p()
                assert L.lib().rbx_hll_open(client.ctx, f"hq-{per}-{int(runs)}-{i}".encode(), 1, C.byref(hp)) == 0
                hs.append(hp.value)
            arr = (C.c_void_p * NH)(*hs)
            els = [rng.integers(0, 256, size=(per, 16), dtype=np.uint8) for _ in range(NH)]
            if runs:
                for i in range(0, NH, 3):
                    els[i] = np.concatenate([els[i], run5])
            seg = np.zeros(NH + 1, np.uint64)
            seg[1:] = np.cumsum([len(e) for e in els])
            el = torch.from_numpy(np.concatenate(els)).cuda()
            changed = torch.zeros(NH, dtype=torch.int32, device="cuda")
            dk = device_keys(el.data_ptr(), int(seg[-1]), 16)
            torch.cuda.synchronize()
            ms = timed(stream, lambda: L.lib().rbx_hll_add_multi_dev(
                client.ctx, arr, NH, None, seg.ctypes.data_as(L.u64p), C.byref(dk), changed.data_ptr(), sp), 1)
            enc = []
            for i in (0, 1):
                buf = np.zeros(16 + 12288, np.uint8)
                ln = C.c_uint64()
                assert L.lib().rbx_hll_export_enc(client.ctx, f"hq-{per}-{int(runs)}-{i}".encode(), 2,
                                                  buf.ctypes.data_as(L.u8p), buf.size, C.byref(ln)) == 0
                enc.append(("sparse" if buf[4] else "dense", int(ln.value)))
            print(json.dumps({"bench": "hllruns_first", "hlls": NH, "per": per, "runs_of_five": runs, "ms": ms,
                              "hll0_hll1": enc}), flush=True)
            for hp in hs:
                L.lib().rbx_hll_close(C.c_void_p(hp))
            for i in range(NH):
                client.getHyperLogLog(f"hq-{per}-{int(runs)}-{i}").delete()

    if "addab" in a.what:
        # C2 add (n/2 keys into an empty 2^32-bit filter), rbx_tune variants interleaved round by
        # round, fresh filter per run: RBX_ADDAB="key=v,key=v;key=v" ("-" = defaults)
        cnt = torch.zeros(2, dtype=torch.int64, device="cuda")
        m = n // 2
        variants = os.environ.get("RBX_ADDAB", "-;add_records=0").split(";")
        res = {v: [] for v in variants}
        news = {}
        for rnd in range(5):
            for v in variants:
                for kv in filter(None, ("" if v == "-" else v).split(",")):
                    key, val = kv.split("=")
                    assert L.lib().rbx_tune(key.encode(), int(val)) == 0, kv
                fb = client.getBloomFilter(f"ab-{rnd}")
                fb.tryInitRaw(1 << 32, 7)
                h = BloomHandle(client, f"ab-{rnd}")
                cnt.zero_()
                res[v].append(timed(stream, lambda: h.add_dev(device_keys(keys.data_ptr(), m, 32), cnt.data_ptr(),
                                                              stream=sp), 1))
                news[v] = int(cnt[0].item())
                h.close()
                fb.delete()
                for kv in filter(None, ("" if v == "-" else v).split(",")):
                    key = kv.split("=")[0]
                    L.lib().rbx_tune(key.encode(), {"add_records": 2, "add_partition": 2, "add_region_grid": 2048,
                                                       "add_rec_lds_limit": 7168}.get(key, 0))
        assert len(set(news.values())) == 1, news
        for v, t in res.items():
            med = statistics.median(t)
            print(json.dumps({"bench": "addab", "tune": v, "keys": m, "ms_median": med, "ms_min": min(t),
                              "ms_max": max(t), "keys_per_s": m / (med / 1e3), "new": news[v]}), flush=True)

    if "addfill" in a.what:
        # C2-size add (n/2 keys) into a 2^32-bit filter whose bitmap was imported with fill f
        # (random bits: AND/OR of uniform bytes), each add_records mode, fresh import per run
        import ctypes as C

        cnt = torch.zeros(2, dtype=torch.int64, device="cuda")
        m = n // 2
        nbytes = 1 << 29

        def bits(f):
            r = lambda: torch.randint(0, 256, (nbytes,), dtype=torch.uint8, device="cuda", generator=g)
            return {0.0: lambda: torch.zeros(nbytes, dtype=torch.uint8, device="cuda"), 0.125: lambda: r() & r() & r(),
                    0.25: lambda: r() & r(), 0.5: r, 0.75: lambda: r() | r()}[f]()

        for fill in (0.0, 0.125, 0.25, 0.5, 0.75):
            img = bits(fill)
            for rec in [int(x) for x in os.environ.get("RBX_ADDFILL_MODES", "0,1,2").split(",")]:
                L.lib().rbx_tune(b"add_records", rec)
                ts, news = [], None
                for rnd in range(2):
                    nm = f"af-{fill}-{rec}-{rnd}"
                    fb = client.getBloomFilter(nm)
                    fb.tryInitRaw(1 << 32, 7)
                    assert L.lib().rbx_bloom_import_dev(client.ctx, nm.encode(), img.data_ptr(), nbytes, sp) == 0
                    h = BloomHandle(client, nm)
                    cnt.zero_()
                    ts.append(timed(stream, lambda: h.add_dev(device_keys(keys.data_ptr(), m, 32), cnt.data_ptr(),
                                                              stream=sp), 1))
                    news = int(cnt[0].item())
                    h.close()
                    fb.delete()
                print(json.dumps({"bench": "addfill", "fill": fill, "add_records": rec, "ms": min(ts), "new": news}),
                      flush=True)
            del img
        L.lib().rbx_tune(b"add_records", 2)

    if "addsweep" in a.what:
        # table vs partitioned add by batch size and filter size (fresh filter per run, 16-B keys)
        cnt = torch.zeros(2, dtype=torch.int64, device="cuda")
        k16 = torch.randint(0, 256, (4_000_000, 16), dtype=torch.uint8, device="cuda", generator=g)
        for size in (1 << 24, 95_850_583, 1 << 28, 1 << 32):
            for nk in (20_000, 100_000, 250_000, 500_000, 1_000_000, 4_000_000):
                res = {}
                for mode in (0, 1):
                    L.lib().rbx_tune(b"add_partition", mode)
                    ts = []
                    for rnd in range(3):
                        nm = f"as-{size}-{nk}-{mode}-{rnd}"
                        fb = client.getBloomFilter(nm)
                        fb.tryInitRaw(size, 7)
                        h = BloomHandle(client, nm)
                        h.add_dev(device_keys(k16.data_ptr(), nk, 16), cnt.data_ptr(), stream=sp)  # first call: allocations
                        h.close()
                        fb.delete()
                        fb = client.getBloomFilter(nm)
                        fb.tryInitRaw(size, 7)
                        h = BloomHandle(client, nm)
                        ts.append(timed(stream, lambda: h.add_dev(device_keys(k16.data_ptr(), nk, 16), cnt.data_ptr(),
                                                                  stream=sp), 1))
                        h.close()
                        fb.delete()
                    res[mode] = statistics.median(ts)
                print(json.dumps({"bench": "addsweep", "size": size, "keys": nk, "table_ms": res[0],
                                  "partitioned_ms": res[1]}), flush=True)
        L.lib().rbx_tune(b"add_partition", 2)

    if "c1con" in a.what:
        # the C1 leg's contains: 1M added + 1M fresh 16-byte keys against tryInit(1e7, 0.01)
        cnt = torch.zeros(2, dtype=torch.int64, device="cuda")
        k16 = torch.randint(0, 256, (2_000_000, 16), dtype=torch.uint8, device="cuda", generator=g)
        fb = client.getBloomFilter("c1c")
        fb.tryInitRaw(95_850_583, 7)
        h = BloomHandle(client, "c1c")
        h.add_dev(device_keys(k16.data_ptr(), 1_000_000, 16), cnt.data_ptr(), stream=sp)
        torch.cuda.synchronize()
        res = {}
        for s1 in [int(x) for x in os.environ.get("RBX_C1_STAGE1", "4").split(",")]:
            L.lib().rbx_tune(b"contains_stage1", s1)
            ts = [timed(stream, lambda: h.contains_dev(device_keys(k16.data_ptr(), 2_000_000, 16), cnt.data_ptr() + 8,
                                                       stream=sp), 5) for _ in range(5)]
            res[s1] = statistics.median(ts)
        L.lib().rbx_tune(b"contains_stage1", 4)
        print(json.dumps({"bench": "c1con", "ms_by_stage1": res}), flush=True)
        h.close()
        fb.delete()

    if "c1add" in a.what:
        # the C1 leg's add: 1M 16-byte keys into a fresh tryInit(1e7, 0.01) filter, 5 times
        cnt = torch.zeros(2, dtype=torch.int64, device="cuda")
        k16 = torch.randint(0, 256, (1_000_000, 16), dtype=torch.uint8, device="cuda", generator=g)
        ts = []
        for rnd in range(6):
            nm = f"c1a-{rnd}"
            fb = client.getBloomFilter(nm)
            fb.tryInitRaw(95_850_583, 7)
            h = BloomHandle(client, nm)
            torch.cuda.synchronize()
            ts.append(timed(stream, lambda: h.add_dev(device_keys(k16.data_ptr(), 1_000_000, 16), cnt.data_ptr(),
                                                      stream=sp), 1))
            h.close()
            fb.delete()
        print(json.dumps({"bench": "c1add", "ms": ts[1:], "median": statistics.median(ts[1:])}), flush=True)

    if "padd" in a.what:
        # add of n/2 keys into an empty filter: first-setter table (0) vs partitioned (1), fresh filters
        cnt = torch.zeros(2, dtype=torch.int64, device="cuda")
        m = n // 2
        for name, size, k in [("C2_2^32", 1 << 32, 7), ("C2_twin", 4294967293, 7)]:
            res = {0: [], 1: []}
            news = {}
            for rnd in range(3):
                for mode in res:
                    L.lib().rbx_tune(b"add_partition", mode)
                    fb = client.getBloomFilter(f"pa-{name}-{rnd}-{mode}")
                    fb.tryInitRaw(size, k)
                    h = BloomHandle(client, f"pa-{name}-{rnd}-{mode}")
                    cnt.zero_()
                    res[mode].append(timed(stream, lambda: h.add_dev(device_keys(keys.data_ptr(), m, 32),
                                                                     cnt.data_ptr(), stream=sp), 1))
                    news[mode] = int(cnt[0].item())
                    h.close()
                    fb.delete()
            assert news[0] == news[1], news
            for mode, v in res.items():
                med = statistics.median(v)
                print(json.dumps({"bench": "add_partition", "filter": name, "mode": mode, "keys": m, "ms_median": med,
                                  "keys_per_s": m / (med / 1e3), "new": news[mode]}), flush=True)
        L.lib().rbx_tune(b"add_partition", 2)

    if "c3ab" in a.what:
        # C3 set up once (bench.py run_c3 shape), then contains kernels interleaved round by round
        # in one process: RBX_C3AB="stage1:grid,..." (grid only used by stage 5)
        import ctypes as C

        import numpy as np

        nt = int(os.environ.get("RBX_C3_TENANTS", "100000"))
        pool = torch.randint(0, 256, (64 << 20,), dtype=torch.uint8, device="cuda", generator=g)
        rng = np.random.default_rng(0)
        hs = []
        for t in range(nt):
            nm = f"ab:{t:06d}"
            f = client.getBloomFilter(nm)
            f.tryInit(1_000_000, 1e-3)
            nbytes = (f._size + 7) // 8
            off = int(rng.integers(0, (pool.numel() - nbytes) // 256)) * 256
            assert L.lib().rbx_bloom_import_dev(client.ctx, nm.encode(), pool.data_ptr() + off, nbytes, sp) == 0
            hs.append(BloomHandle(client, nm))
        per = max(1, n // nt)
        m = per * nt
        k16 = torch.randint(0, 256, (m, 16), dtype=torch.uint8, device="cuda", generator=g)
        seg = torch.arange(nt + 1, dtype=torch.int64, device="cuda") * per
        counts = torch.zeros(nt, dtype=torch.int64, device="cuda")
        arr = (C.c_void_p * nt)(*[h.h.value for h in hs])
        dk = device_keys(k16.data_ptr(), m, 16)
        variants = [tuple(int(x) for x in v.split(":")) for v in
                    os.environ.get("RBX_C3AB", "4:0,5:2048,5:1024").split(",")]

        def run():
            assert L.lib().rbx_bloom_contains_multi_dev(client.ctx, arr, nt, seg.data_ptr(), C.byref(dk), None,
                                                         counts.data_ptr(), sp) == 0

        res = {v: [] for v in variants}
        ref = None
        for rnd in range(6):
            for v in variants:
                L.lib().rbx_tune(b"contains_stage1", v[0])
                L.lib().rbx_tune(b"contains_multi_slots", 1 if v[0] == 5 else 0)
                if v[0] == 5:
                    L.lib().rbx_tune(b"contains_qgrid", v[1])
                counts.zero_()
                run()
                c = counts.clone()
                ref = c if ref is None else ref
                assert torch.equal(c, ref), v
                res[v].append(timed(stream, run, 3))
        L.lib().rbx_tune(b"contains_stage1", 4)
        L.lib().rbx_tune(b"contains_multi_slots", 2)
        for v, t in res.items():
            med = statistics.median(t)
            print(json.dumps({"bench": "c3ab", "stage1": v[0], "grid": v[1], "ms_median": med,
                              "ms_min": min(t), "ms_max": max(t), "keys_per_s": m / (med / 1e3)}), flush=True)
        for h in hs:
            h.close()

    if "c3add" in a.what:
        # C3's add half (bench.py c3_add_half shape: 1,000 fresh 16-byte keys per tenant per call, filters at
        # design fill) with the per-segment kernel shapes interleaved call by call in one process:
        # RBX_C3ADD="grid,..." (rbx_tune add_multi_seg_grid), every call on a new key window
        import ctypes as C

        import numpy as np

        nt = int(os.environ.get("RBX_C3_TENANTS", "100000"))
        pool = torch.randint(0, 256, (64 << 20,), dtype=torch.uint8, device="cuda", generator=g)
        rng = np.random.default_rng(0)
        hs = []
        for t in range(nt):
            nm = f"aa:{t:06d}"
            f = client.getBloomFilter(nm)
            f.tryInit(1_000_000, 1e-3)
            nbytes = (f._size + 7) // 8
            off = int(rng.integers(0, (pool.numel() - nbytes) // 256)) * 256
            assert L.lib().rbx_bloom_import_dev(client.ctx, nm.encode(), pool.data_ptr() + off, nbytes, sp) == 0
            hs.append(BloomHandle(client, nm))
        del pool
        per = max(1, n // nt)
        m = per * nt
        variants = [tuple(int(y) for y in x.split(":")) for x in os.environ.get("RBX_C3ADD", "8192,4096").split(",")]
        rounds = int(os.environ.get("RBX_C3ADD_ROUNDS", "5"))
        ncalls = rounds * len(variants) + 1
        k16 = torch.randint(0, 256, (m + ncalls * per, 16), dtype=torch.uint8, device="cuda", generator=g)
        seg = torch.arange(nt + 1, dtype=torch.int64, device="cuda") * per
        counts = torch.zeros(nt, dtype=torch.int64, device="cuda")
        arr = (C.c_void_p * nt)(*[h.h.value for h in hs])
        call = [0]

        def run():
            dk = device_keys(k16.data_ptr() + 16 * per * call[0], m, 16)
            call[0] += 1
            assert L.lib().rbx_bloom_add_multi_dev(client.ctx, arr, nt, seg.data_ptr(), C.byref(dk), None,
                                                    counts.data_ptr(), sp) == 0

        run()  # warm
        res = {v: [] for v in variants}
        for rnd in range(rounds):
            for v in variants:
                assert L.lib().rbx_tune(b"add_multi_seg_grid", v[0]) == 0
                if len(v) > 1:  # "grid:tune_value" with RBX_C3ADD_KEY naming the knob
                    assert L.lib().rbx_tune(os.environ["RBX_C3ADD_KEY"].encode(), v[1]) == 0
                counts.zero_()
                res[v].append(timed(stream, run, 1))
                assert int(counts.sum().item()) > m * 0.99
        L.lib().rbx_tune(b"add_multi_seg_grid", 8192)
        for v, t in res.items():
            med = statistics.median(t)
            print(json.dumps({"bench": "c3add", "seg_grid": v, "ms_median": med, "ms_min": min(t), "ms_max": max(t),
                              "keys_per_s": m / (med / 1e3)}), flush=True)
        for h in hs:
            h.close()

    if "pflags" in a.what:
        # direct vs partitioned contains, and the partitioned path with its diagnostic switches
        cnt = torch.zeros(8, dtype=torch.int64, device="cuda")
        fb = client.getBloomFilter("pf-C2")
        fb.tryInitRaw(1 << 32, 7)
        h = BloomHandle(client, "pf-C2")
        h.add_dev(device_keys(keys.data_ptr(), n // 2, 32), cnt.data_ptr(), stream=sp)
        torch.cuda.synchronize()
        dk = device_keys(keys.data_ptr(), n, 32)
        variants = [(0, 0), (1, 0), (1, 4), (1, 8)]  # flags 4, 8: diagnostics (wrong results, timing only)
        if os.environ.get("RBX_PFLAGS"):  # e.g. "1:0,1:16": A/B of experimental switches
            variants = [tuple(int(x) for x in v.split(":")) for v in os.environ["RBX_PFLAGS"].split(",")]
        res = {v: [] for v in variants}
        counts = {}
        for rnd in range(5):
            for mode, fl in variants:
                L.lib().rbx_tune(b"contains_partition", mode)
                L.lib().rbx_tune(b"contains_partition_flags", fl)
                cnt[1].zero_()
                res[(mode, fl)].append(timed(stream, lambda: h.contains_dev(dk, cnt.data_ptr() + 8, stream=sp), 2))
                if not fl & 44:
                    counts[(mode, fl)] = int(cnt[1].item())
        assert len(set(counts.values())) == 1, counts
        for (mode, fl), v in res.items():
            med = statistics.median(v)
            print(json.dumps({"bench": "contains_pflags", "mode": mode, "flags": fl, "ms_median": med,
                              "keys_per_s": n / (med / 1e3)}), flush=True)
        L.lib().rbx_tune(b"contains_partition", 2)
        L.lib().rbx_tune(b"contains_partition_flags", 0)
        h.close()
        fb.delete()

    if "stage1" in a.what or "sizes" in a.what:
        cnt = torch.zeros(8, dtype=torch.int64, device="cuda")
        plan = []
        if "stage1" in a.what:
            plan.append(("C2_2^32", 1 << 32, 7, [0, 1, 2, 4, 5]))
        if "sizes" in a.what:
            plan += [("C1", 95850583, 7, [1, 4, 5]), ("C3", 14377587, 10, [1, 4, 5]), ("C2_twin", 4294967293, 7, [1, 4, 5])]
        for name, size, k, s1s in plan:
            fb = client.getBloomFilter("mb-" + name)
            fb.tryInitRaw(size, k)
            h = BloomHandle(client, "mb-" + name)
            # fill to the design load: n_add keys so that fill matches (C2: 50M; C1: 10M; C3: 1M)
            n_add = {"C2_2^32": n // 2, "C2_twin": n // 2, "C1": 10_000_000, "C3": 1_000_000}[name]
            h.add_dev(device_keys(keys.data_ptr(), n_add, 32), cnt.data_ptr(), stream=sp)
            torch.cuda.synchronize()
            dk = device_keys(keys.data_ptr(), n, 32)
            res = {}
            for s1 in s1s:
                res[s1] = []
            for rnd in range(5):
                for s1 in res:
                    L.lib().rbx_tune(b"contains_stage1", s1)
                    res[s1].append(timed(stream, lambda: h.contains_dev(dk, cnt.data_ptr() + 8, stream=sp), 2))
            for s1, v in res.items():
                med = statistics.median(v)
                print(json.dumps({"bench": "contains", "filter": name, "size": size, "k": k, "n_added": n_add,
                                  "stage1": s1, "ms_median": med, "ms_min": min(v),
                                  "keys_per_s": n / (med / 1e3)}), flush=True)
            L.lib().rbx_tune(b"contains_stage1", 4)
            h.close()
            fb.delete()

    if "add" in a.what:
        cnt = torch.zeros(2, dtype=torch.int64, device="cuda")
        for name, size, k in [("C2_2^32", 1 << 32, 7), ("C1", 95850583, 7)]:
            fb = client.getBloomFilter("ad-" + name)
            fb.tryInitRaw(size, k)
            h = BloomHandle(client, "ad-" + name)
            m = n // 2
            ms = timed(stream, lambda: h.add_dev(device_keys(keys.data_ptr(), m, 32), cnt.data_ptr(), stream=sp), 1)
            print(json.dumps({"bench": "add", "filter": name, "keys": m, "ms": ms, "keys_per_s": m / (ms / 1e3)}),
                  flush=True)
            h.close()
            fb.delete()
    client.shutdown()


if __name__ == "__main__":
    main()
