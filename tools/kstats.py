"""Print the top kernels of a rocprofv3 --stats kernel_stats.csv (share, calls, average, name)."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
div = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0   # e.g. the number of steps in the trace
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print(f"total {tot / 1e6 / div:.2f} ms per unit")
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:int(sys.argv[3]) if len(sys.argv) > 3 else 25]:
    n = r["Name"].replace("(anonymous namespace)::", "").replace("pdm::", "")[:80]
    print(f"{float(r['TotalDurationNs']) / tot * 100:5.1f}% {float(r['TotalDurationNs']) / 1e6 / div:7.2f}ms "
          f"{int(r['Calls']):5d} {float(r['AverageNs']) / 1e3:9.1f}us {n}")
