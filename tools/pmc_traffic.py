#!/usr/bin/env python3
"""Per-kernel HBM traffic per launch from rocprofv3 --pmc CSVs -> profiles/traffic.json.

Usage: python tools/pmc_traffic.py <fetch_pass_dir> <write_pass_dir> [<hit_pass_dir>] -o profiles/traffic.json

Follows MI355X_MICROARCH.md §HBM: FETCH_SIZE / WRITE_SIZE are in KiB, collected in
separate passes; on gfx950 FETCH_SIZE reports exactly half the bytes of a wide coalesced
streaming read, so it is doubled ("x2 correction").  For these kernels most fetches are
random 4-byte gathers (one 64-byte request each, uncalibrated width) -- the uncorrected
figure is kept beside the corrected one and both are per launch, averaged over launches.
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
         ("k_ba_keys", r"k_ba_keys"), ("k_ba_final", r"k_ba_final"),
         ("k_stream_probe", r"k_stream_probe<"), ("k_stream_contains", r"k_stream_contains<"),
         ("k_stream_commit", r"k_stream_commit<"),
         ("k_bloom_contains_multi", r"k_bloom_contains_multi<"), ("k_bloom_contains_q", r"k_bloom_contains_q<"),
         ("k_bloom_contains", r"k_bloom_contains<"),
         ("k_bloom_add_probe", r"k_bloom_add_probe"), ("k_bloom_add_commit", r"k_bloom_add_commit"),
         ("k_gather_probe", r"k_gather_probe"), ("k_hll_pfadd", r"k_hll_pfadd"), ("k_hll_count", r"k_hll_count"),
         ("k_bitcount", r"k_bitcount")]


def short(name: str) -> str | None:
    for s, pat in SHORT:
        if re.search(pat, name):
            return s
    return None


def load(d: str):
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for p in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
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
    a = ap.parse_args()
    calls = {kv.split("=")[0]: int(kv.split("=")[1]) for kv in a.calls}
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
        out[k] = e
    for k in out:
        out[k]["launches_profiled"] = launches.get(k)
    # one API call = these kernels in sequence, possibly once per chunk: per-call totals =
    # all profiled launches' counters / the calls in the profiled run (--calls)
    for name, parts in (("contains_pipeline", ("k_bk_stage1", "k_bk_emit2", "k_bk_probe", "k_bk_misses", "k_bk_final")),
                        ("add_pipeline", ("k_ba_stage1", "k_ba_rebucket", "k_ba_region", "k_ba_keys", "k_ba_final")),
                        ("stream_pipeline", ("k_stream_compact", "k_stream_probe", "k_stream_contains", "k_stream_commit"))):
        if not all(k in out for k in parts) or name not in calls:
            continue
        agg = {"kernels": list(parts), "calls_profiled": calls[name],
               "note": "per API call: sum over the profiled launches / calls (the keys "
                       "written '_per_launch' here mean per call)"}
        for f in ("hbm_bytes_per_launch", "requests_per_launch", "fetch_bytes_x2", "write_bytes"):
            if all(f in out[k] for k in parts):
                agg[f] = sum(out[k][f] * launches[k] for k in parts) / calls[name]
        out[name] = agg
    os.makedirs(os.path.dirname(a.o) or ".", exist_ok=True)
    with open(a.o, "w") as fh:
        json.dump(out, fh, indent=1, sort_keys=True)
    print(json.dumps(out, indent=1, sort_keys=True))


if __name__ == "__main__":
    main()
