#!/usr/bin/env python3
"""Copy one profiling pass (tools/profile_gpu.sh TAG) from gpurun_out/prof into
profiles/<round>/ and derive profiles/spmv_pmc_bytes.json, the per-launch HBM
traffic bench.py reports for the Lanczos SpMV.

FETCH_SIZE / WRITE_SIZE are in kB per dispatch. On gfx950, FETCH_SIZE counts
half the bytes of wide coalesced reads (MI355X_MICROARCH.md, HBM section), so
reads are doubled. The counters see L2 memory-side requests, including
Infinity-Cache hits.

usage: python tools/summarize_profiles.py TAG ROUND   (e.g. r01b r01)
"""
import collections
import csv
import json
import os
import shutil
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SPMV = "k_spmv_adaptive"


def per_kernel(path):
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        agg[r["Kernel_Name"].split("(")[0]].append(float(r["Counter_Value"]))
    return {k: {"dispatches": len(v), "avg_kB": round(sum(v) / len(v), 1)} for k, v in agg.items()
            if "ek::dev::" in k}


def main(tag, rnd):
    src = os.path.join(REPO, "gpurun_out", "prof")
    dst = os.path.join(REPO, "profiles", rnd)
    os.makedirs(dst, exist_ok=True)
    stats = os.path.join(src, "trace", f"{tag}_kernel_stats.csv")
    shutil.copy(stats, os.path.join(dst, "bench_kernel_stats.csv"))
    lab = os.path.join(src, f"{tag}_spmv_lab.txt")
    if os.path.exists(lab):
        shutil.copy(lab, os.path.join(dst, "spmv_lab.txt"))
    fetch = per_kernel(os.path.join(src, "pmc_fetch", f"{tag}_counter_collection.csv"))
    write = per_kernel(os.path.join(src, "pmc_write", f"{tag}_counter_collection.csv"))
    name = next(k for k in fetch if SPMV in k)
    avg_ns = next(float(r["AverageNs"]) for r in csv.DictReader(open(stats)) if SPMV in r["Name"])
    f_b, w_b = fetch[name]["avg_kB"] * 1024, write[name]["avg_kB"] * 1024
    out = {
        "workload": "syn1x-seed1",
        "command": "rocprofv3 --pmc FETCH_SIZE | --pmc WRITE_SIZE (separate passes) -- python3 bench.py "
                   "--steps 3 --warmup 1 --no-cpu-baseline --no-sweep",
        "kernel": name,
        "rocprof_avg_launch_us": round(avg_ns / 1e3, 3),
        "fetch_bytes_raw": round(f_b), "write_bytes": round(w_b),
        "correction": "reads doubled (gfx950 FETCH_SIZE counts half of wide coalesced reads); L2 memory-side "
                      "requests, Infinity-Cache hits included",
        "hbm_bytes_per_launch": round(2 * f_b + w_b),
        "per_kernel": {"FETCH_SIZE": fetch, "WRITE_SIZE": write},
    }
    json.dump(out, open(os.path.join(REPO, "profiles", "spmv_pmc_bytes.json"), "w"), indent=1)
    json.dump(out, open(os.path.join(dst, "spmv_pmc_bytes.json"), "w"), indent=1)
    print(json.dumps({k: out[k] for k in ("kernel", "rocprof_avg_launch_us", "hbm_bytes_per_launch")}))


if __name__ == "__main__":
    main(*sys.argv[1:3])
