"""Summarise tools/raster_traffic.sh (dev tool): per GEMM shape and tile-order raster, the kernel's average time, its
L2-miss read bytes (FETCH_SIZE x 2, the gfx950 correction of MI355X_MICROARCH.md §HBM) against the operand bytes,
and the L2 hit rate.  Usage: python3 tools/raster_traffic_summary.py [TAG]"""
import csv
import glob
import os
import sys

tag = sys.argv[1] if len(sys.argv) > 1 else "rtraffic"
root = f"gpurun_out/{tag}"
M = 25800
print(f"persistent GEMM (algo 11), M = {M}, plain bf16 output; FETCH x 2 = L2-miss read bytes per launch")
for d in sorted(glob.glob(f"{root}/n*_k*_r*")):
    n, k, r = (int(x[1:]) for x in os.path.basename(d).split("_"))
    t = [float(x["AverageNs"]) / 1e3 for x in csv.DictReader(open(f"{d}/kt/run_kernel_stats.csv")) if "gemm8s" in x["Name"]]
    vals = {}
    for sub in ("fetch", "hit"):
        rows = [x for x in csv.DictReader(open(f"{d}/{sub}/run_counter_collection.csv")) if "gemm8s" in x["Kernel_Name"]]
        for x in rows:
            vals.setdefault(x["Counter_Name"], []).append(float(x["Counter_Value"]))
    avg = {c: sum(v) / len(v) for c, v in vals.items()}
    fetch = 2 * avg["FETCH_SIZE"] * 1024   # FETCH_SIZE is in KB
    operands = (M * k + n * k) * 2
    hit = avg["TCC_HIT_sum"] / (avg["TCC_HIT_sum"] + avg["TCC_MISS_sum"])
    print(f"N={n:5d} K={k:5d} raster {r:2d}: {t[0]:7.1f} us  L2-miss reads {fetch / 1e6:7.1f} MB = {fetch / operands:4.2f}x "
          f"operands ({operands / 1e6:.1f} MB)  L2 hit {hit:.3f}")
