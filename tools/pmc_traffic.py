#!/usr/bin/env python3
"""Per-kernel HBM traffic per launch from rocprofv3 --pmc CSVs -> profiles/traffic.json.

Usage: python tools/pmc_traffic.py <pass_dir>... -o profiles/traffic.json
           [--calls pipeline=N ...] [--stream-bytes kernel=B ...]

Follows MI355X_MICROARCH.md §HBM: FETCH_SIZE / WRITE_SIZE are in KiB, collected in separate
passes; FETCH_SIZE = TCC_EA0_RDREQ x 64 B, and on gfx950 it reports exactly half the bytes of a
wide coalesced streaming read (128-B requests tallied at 64 B).  The x2 correction therefore
applies ONLY to streaming reads.  `hbm_bytes_by_class` prices each access class separately:
  stream  kernels (every read a wide streaming read):  RDREQ x 128 B
  gather  kernels (random 4-byte loads):               RDREQ x 64 B -- one 64-B request each
  mixed   kernels (a key stream + random gathers):     S x 128 B + (RDREQ - S) x 64 B, with
          S = the kernel's streamed bytes per launch / 128 (--stream-bytes, from the workload)
plus WRITE_SIZE (exact for 16-B streaming stores).  Infinity-Cache hits are counted by these
TCC counters, not excluded (the guide's note): for gather kernels over tables below 256 MiB
the figure is an upper bound on DRAM bytes.  The old uniform "x2" figure stays beside it as
`hbm_bytes_per_launch` (an over-count for gather kernels).
"""
from __future__ import annotations

import argparse
import collections
import csv
import glob
import json
import os
import re

SHORT = [("k_bk_stage1", r"k_bk_stage1<"), ("k_bk_emit2", r"k_bk_emit2<"), ("k_bk_probe", r"k_bk_probe"),
         ("k_bk_misses", r"k_bk_misses"), ("k_bk_final", r"k_bk_final"), ("k_stream_compact", r"k_stream_compact"),
         ("k_ba_stage1", r"k_ba_stage1<"), ("k_ba_rebucket", r"k_ba_rebucket"), ("k_ba_region", r"k_ba_region"),
         ("k_ba_keys_rec", r"k_ba_keys_rec"), ("k_ba_keys", r"k_ba_keys\("), ("k_ba_mode", r"k_ba_mode"), ("k_ba_final", r"k_ba_final"),
         ("k_stream_probe", r"k_stream_probe<"), ("k_stream_probe8", r"k_stream_probe8<"),
         ("k_stream_walk", r"k_stream_walk"), ("k_stream_final8", r"k_stream_final8<"),
         ("k_stream_final", r"k_stream_final\("), ("k_madd_probe8", r"k_madd_probe8<"),
         ("k_madd_final8", r"k_madd_final8<"), ("k_maddx_gather", r"k_maddx_gather<"),
         ("k_maddx_set", r"k_maddx_set<"), ("k_maddx_claim", r"k_maddx_claim<"), ("k_maddx_reply", r"k_maddx_reply<"),
         ("k_maddx_reset", r"k_maddx_reset"), ("k_madd_seg", r"k_madd_seg<"), ("k_madd_tiles", r"k_madd_tiles<"),
         ("k_stream_contains_q", r"k_stream_contains_q<"),
         ("k_stream_contains", r"k_stream_contains<"),
         ("k_stream_commit", r"k_stream_commit<"),
         ("k_bloom_contains_multi", r"k_bloom_contains_multi<"), ("k_bloom_contains_q", r"k_bloom_contains_q<"),
         ("k_bloom_contains", r"k_bloom_contains<"),
         ("k_bloom_add_probe", r"k_bloom_add_probe"), ("k_bloom_add_commit", r"k_bloom_add_commit"),
         ("k_gather_probe", r"k_gather_probe"), ("k_hll_pfadd", r"k_hll_pfadd"), ("k_hll_count", r"k_hll_count"),
         ("k_bitcount", r"k_bitcount")]


CLASS = {"k_bk_stage1": "mixed", "k_bloom_contains": "mixed", "k_bloom_contains_multi": "mixed",
         "k_bloom_contains_q": "mixed", "k_stream_probe": "mixed", "k_stream_contains": "mixed",
         "k_stream_contains_q": "mixed",
         "k_stream_commit": "mixed", "k_stream_probe8": "mixed", "k_madd_probe8": "mixed", "k_maddx_gather": "mixed", "k_madd_seg": "mixed", "k_madd_tiles": "mixed", "k_gather_probe": "gather",
         "k_bloom_add_probe": "gather",
         "k_bloom_add_commit": "gather"}  # every other kernel: stream


def short(name: str) -> str | None:
    for s, pat in SHORT:
        if re.search(pat, name):
            return s
    return None


def load(d: str):
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    # a pass directory, or the per-pass rows kept by tools/profile_round.sh (pmc_*_rbx_rows.csv)
    paths = [d] if os.path.isfile(d) else glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    for p in paths:
        for r in csv.DictReader(open(p)):
            s = short(r["Kernel_Name"])
            if s:
                agg[s][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return agg


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dirs", nargs="+")
    ap.add_argument("-o", default="profiles/traffic.json")
    ap.add_argument("--calls", nargs="*", default=[],
                    help="pipeline=N: API calls of that pipeline in the profiled run (per-call totals)")
    ap.add_argument("--stream-bytes", nargs="*", default=[],
                    help="kernel=B: streamed (key) bytes per launch of a mixed-class kernel")
    a = ap.parse_args()
    calls = {kv.split("=")[0]: int(kv.split("=")[1]) for kv in a.calls}
    streamed = {kv.split("=")[0]: float(kv.split("=")[1]) for kv in a.stream_bytes}
    merged = collections.defaultdict(dict)
    launches = {}
    for d in a.dirs:
        for k, cs in load(d).items():
            for c, v in cs.items():
                merged[k][c] = sum(v) / len(v)
                launches[k] = len(v)
    out = {}
    for k, cs in merged.items():
        fetch = cs.get("FETCH_SIZE")
        write = cs.get("WRITE_SIZE")
        e = {"counters_avg_per_launch": cs}
        if fetch is not None:
            e["fetch_bytes_uncorrected"] = fetch * 1024
            e["fetch_bytes_x2"] = 2 * fetch * 1024
        if write is not None:
            e["write_bytes"] = write * 1024
        if fetch is not None:
            e["hbm_bytes_per_launch"] = 2 * fetch * 1024 + (write or 0) * 1024
            e["correction"] = "FETCH_SIZE KiB x1024 x2 (gfx950 half-count) + WRITE_SIZE KiB x1024"
        if "TCC_HIT_sum" in cs and "TCC_MISS_sum" in cs:
            t = cs["TCC_HIT_sum"] + cs["TCC_MISS_sum"]
            e["tcc_hit_rate"] = cs["TCC_HIT_sum"] / t if t else None
        if "TCC_EA0_RDREQ_sum" in cs and "TCC_EA0_WRREQ_sum" in cs:
            # memory requests at the L2 -> EA interface (the binding rate for these kernels)
            e["requests_per_launch"] = cs["TCC_EA0_RDREQ_sum"] + cs["TCC_EA0_WRREQ_sum"]
            e["read_requests_per_launch"] = cs["TCC_EA0_RDREQ_sum"]
            e["write_requests_per_launch"] = cs["TCC_EA0_WRREQ_sum"]
        if "TCC_ATOMIC_sum" in cs:
            # atomic requests at the L2 (all types), and those sent on to memory (EA): the atomic
            # throughput north_star asks for; EA atomics also count in TCC_EA0_WRREQ
            e["atomic_requests_per_launch"] = cs["TCC_ATOMIC_sum"]
        if "TCC_EA0_ATOMIC_sum" in cs:
            e["ea_atomic_requests_per_launch"] = cs["TCC_EA0_ATOMIC_sum"]
        rd = cs.get("TCC_EA0_RDREQ_sum")
        if rd is None and fetch is not None:
            rd = fetch * 1024 / 64  # FETCH_SIZE = RDREQ x 64 B
        if rd is not None and write is not None:
            cls = CLASS.get(k, "stream")
            if cls == "stream":
                sb, gr = rd * 128, 0.0
            elif cls == "gather":
                sb, gr = 0.0, rd
            else:
                sb = streamed.get(k, 0.0)
                gr = max(0.0, rd - sb / 128)
            e["access_class"] = cls
            e["read_bytes_stream"] = sb
            e["read_requests_gather"] = gr
            e["hbm_bytes_by_class"] = sb + 64 * gr + write * 1024
        out[k] = e
    for k in out:
        out[k]["launches_profiled"] = launches.get(k)
    # one API call = these kernels in sequence, possibly once per chunk: per-call totals =
    # all profiled launches' counters / the calls in the profiled run (--calls)
    for name, parts in (("contains_pipeline", ("k_bk_stage1", "k_bk_emit2", "k_bk_probe", "k_bk_misses", "k_bk_final")),
                        ("add_pipeline", ("k_ba_mode", "k_ba_stage1", "k_ba_rebucket", "k_ba_region", "k_ba_keys",
                                          "k_ba_keys_rec", "k_ba_final")),
                        ("stream_pipeline", ("k_stream_compact", "k_stream_probe", "k_stream_probe8", "k_stream_contains",
                                             "k_stream_contains_q", "k_stream_commit", "k_stream_final8",
                                             "k_stream_walk", "k_stream_final")),
                        ("madd_pipeline", ("k_madd_probe8", "k_madd_final8", "k_stream_walk")),
                        ("maddx_pipeline", ("k_maddx_gather", "k_maddx_set", "k_maddx_claim", "k_maddx_reply",
                                            "k_maddx_reset"))):
        # the stream pipeline runs one of its two contains kernels (staged or slot)
        parts = tuple(k for k in parts if k in out)
        if len(parts) < 3 or name not in calls:
            continue
        agg = {"kernels": list(parts), "calls_profiled": calls[name],
               "note": "per API call: sum over the profiled launches / calls (the keys "
                       "written '_per_launch' here mean per call)"}
        for f in ("hbm_bytes_per_launch", "hbm_bytes_by_class", "requests_per_launch", "read_requests_per_launch",
                  "write_requests_per_launch", "fetch_bytes_x2", "write_bytes", "atomic_requests_per_launch",
                  "ea_atomic_requests_per_launch"):
            if all(f in out[k] for k in parts):
                agg[f] = sum(out[k][f] * launches[k] for k in parts) / calls[name]
        out[name] = agg
    os.makedirs(os.path.dirname(a.o) or ".", exist_ok=True)
    with open(a.o, "w") as fh:
        json.dump(out, fh, indent=1, sort_keys=True)
    print(json.dumps(out, indent=1, sort_keys=True))


if __name__ == "__main__":
    main()
