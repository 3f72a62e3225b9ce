"""Per-kernel breakdown of a profiled decode (dev tool): rocprofv3 --kernel-trace of tools/decode_bench.py, summed
durations per (kernel, workgroup count) divided by the number of decodes the script ran (2 warmup + 5 timed).
Usage: python3 tools/decode_prof_summary.py TRACE_CSV [ndecodes]"""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
nd = int(sys.argv[2]) if len(sys.argv) > 2 else 7
agg = collections.defaultdict(lambda: [0, 0])
for r in rows:
    n = r["Kernel_Name"].replace("void pdm::(anonymous namespace)::", "").replace("pdm::(anonymous namespace)::", "")
    n = n.split("(")[0]
    wgs = int(r["Grid_Size_X"]) // int(r["Workgroup_Size_X"]) * int(r["Grid_Size_Y"])
    d = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    agg[(n[:48], wgs)][0] += d
    agg[(n[:48], wgs)][1] += 1
tot = sum(v[0] for v in agg.values())
print(f"sum of kernel durations {tot / 1e6 / nd:.2f} ms per decode (two lanes overlap)")
for (n, w), (d, c) in sorted(agg.items(), key=lambda x: -x[1][0])[:24]:
    print(f"{d / 1e6 / nd:8.2f} ms {c / nd:5.1f}x avg {d / c / 1e3:8.1f} us wgs {w:7d}  {n}")
