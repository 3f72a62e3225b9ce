"""Print averaged PMC counters of the pdm kernels in gpurun_out/pmc_TAG (dev tool)."""
import collections
import csv
import glob
import sys

for tag in sys.argv[1:]:
    print("==", tag)
    for r in csv.DictReader(open(f"gpurun_out/pmc_{tag}/kt/run_kernel_stats.csv")):
        if "pdm" in r["Name"]:
            print(f"  {r['Name'][:70]} calls {r['Calls']} avg us {float(r['AverageNs']) / 1e3:.1f}")
    acc = collections.defaultdict(list)
    for f in sorted(glob.glob(f"gpurun_out/pmc_{tag}/p*/run_counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            if "pdm" not in r["Kernel_Name"]:
                continue
            acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, v in acc.items():
        print(f"  {k:28s} {sum(v) / len(v):.4g}")
