"""Summarise a tools/profile_round.sh output directory into profiles/.

Writes <out>_kernel_stats.csv (rocprofv3 --kernel-trace --stats, verbatim)
and <out>_summary.json: per kernel the average duration and, from the
separate FETCH_SIZE / WRITE_SIZE passes, the HBM-side bytes per launch
(FETCH_SIZE and WRITE_SIZE are KiB; FETCH_SIZE doubled per
MI355X_MICROARCH.md §HBM, which calibrates it at 1/2 of the bytes of a wide
coalesced read -- the correction is uncalibrated for other access widths).

usage: python tools/summarize_prof.py gpurun_out/prof_r01 profiles/r01
"""
import csv
import json
import os
import shutil
import sys


def short(name):
    name = name.replace("(anonymous namespace)::", "").replace("void ", "")
    return name.split("(")[0].replace("fs::gpu::", "")


def main(src, out):
    stats = {}
    with open(f"{src}/trace/run_kernel_stats.csv") as f:
        for r in csv.DictReader(f):
            stats[short(r["Name"])] = {"calls": int(r["Calls"]), "avg_ms": float(r["AverageNs"]) / 1e6,
                                       "pct": float(r["Percentage"])}
    shutil.copy(f"{src}/trace/run_kernel_stats.csv", f"{out}_kernel_stats.csv")
    for kind in ("fetch", "write"):
        agg = {}
        with open(f"{src}/{kind}/run_counter_collection.csv") as f:
            for r in csv.DictReader(f):
                agg.setdefault(short(r["Kernel_Name"]), []).append(float(r["Counter_Value"]))
        for k, v in agg.items():
            if k in stats:
                stats[k][f"{kind}_KiB_per_launch"] = sum(v) / len(v)
    for k, s in stats.items():
        if "fetch_KiB_per_launch" in s and "write_KiB_per_launch" in s:
            s["hbm_bytes_per_launch"] = (2.0 * s["fetch_KiB_per_launch"] + s["write_KiB_per_launch"]) * 1024
            s["hbm_GBps"] = s["hbm_bytes_per_launch"] / (s["avg_ms"] * 1e-3) / 1e9
    # pass 2 of the sparse path runs one launch per feature width
    # (k_score_sparse2<8>, <4> for a tail): bench.py prices them together as
    # "k_score_sparse" (its HIP events span the pass)
    parts = [s for k, s in stats.items() if k.startswith("k_score_sparse2<")]
    if parts and all("hbm_bytes_per_launch" in s for s in parts):
        stats["k_score_sparse"] = {
            "calls": parts[0]["calls"], "avg_ms": sum(s["avg_ms"] for s in parts),
            "hbm_bytes_per_launch": sum(s["hbm_bytes_per_launch"] for s in parts),
            "parts": [k for k in stats if k.startswith("k_score_sparse2<")]}
        stats["k_score_sparse"]["hbm_GBps"] = (stats["k_score_sparse"]["hbm_bytes_per_launch"]
                                               / (stats["k_score_sparse"]["avg_ms"] * 1e-3) / 1e9)
    bench = json.load(open(f"{src}/bench_trace.json"))
    with open(f"{out}_summary.json", "w") as f:
        json.dump({"bench": bench, "kernels": stats}, f, indent=1)
    # the per-launch HBM bytes bench.py reports as roofline.traffic
    cfg = bench["config"]
    traffic = {"n": cfg["n_samples"], "p": cfg["n_features"], "world": bench["n_gpus"],
               "source": f"{out}_summary.json (rocprofv3 FETCH_SIZE x2 + WRITE_SIZE, KiB x 1024)",
               "kernels": {k: {"hbm_bytes_per_launch": s["hbm_bytes_per_launch"], "avg_ms": s["avg_ms"]}
                           for k, s in stats.items() if "hbm_bytes_per_launch" in s and k.startswith("k_")}}
    with open(os.path.join(os.path.dirname(out), "pmc_traffic.json"), "w") as f:
        json.dump(traffic, f, indent=1)
    for k, s in sorted(stats.items(), key=lambda kv: -kv[1]["avg_ms"])[:12]:
        print(f"{k:28s} {s['avg_ms']:10.3f} ms  {s.get('hbm_GBps', float('nan')):8.1f} GB/s")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
