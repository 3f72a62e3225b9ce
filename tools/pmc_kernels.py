"""Per-kernel SQ-counter summary of tools/pmc_forward.sh output (dev tool).

    python tools/pmc_kernels.py gpurun_out/r04pmc [tag ...]  -> prints a markdown table per tag

Counters are averaged per dispatch over every dispatch of a kernel name (templates kept apart).  Derived:
  VALU/MFMA    SQ_INSTS_VALU / SQ_INSTS_MFMA (instructions issued per matrix instruction)
  MFMA busy    SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 x 1024 SIMDs): the fraction of every SIMD's cycles
               over the dispatch that the matrix pipe was busy (GRBM_GUI_ACTIVE sums the 8 XCDs' clocks)
  VALU active  SQ_ACTIVE_INST_VALU / SQ_WAVE_CYCLES (both quad-cycles: share of a wave's life issuing VALU)
  wait         SQ_WAIT_INST_ANY / SQ_WAVE_CYCLES (waiting on an instruction dependency: memory / LDS counters)
  LDS conflict SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE
"""
import collections
import csv
import glob
import os
import sys


def load(d):
    dur = {}
    for r in csv.DictReader(open(os.path.join(d, "kt", "run_kernel_stats.csv"))):
        dur[r["Name"]] = (int(r["Calls"]), float(r["AverageNs"]) / 1e3, float(r["Percentage"]))
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in sorted(glob.glob(os.path.join(d, "p*", "run_counter_collection.csv"))):
        for r in csv.DictReader(open(f)):
            acc[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return dur, acc


def short(n):
    n = n.replace("void ", "").replace("pdm::(anonymous namespace)::", "")
    return n.split("(")[0][:48]


def main():
    root = sys.argv[1]
    tags = sys.argv[2:] or sorted(os.path.basename(p) for p in glob.glob(os.path.join(root, "*")) if os.path.isdir(p))
    for tag in tags:
        d = os.path.join(root, tag)
        if not os.path.isdir(os.path.join(d, "kt")):
            continue
        dur, acc = load(d)
        print(f"\n### {tag}\n")
        print("| kernel | calls | avg µs | % time | VALU/MFMA | MFMA busy | VALU active | wait | LDS conflict |")
        print("|---|---|---|---|---|---|---|---|---|")
        rows = []
        for name, c in acc.items():
            if "pdm" not in name or not c.get("SQ_WAVE_CYCLES"):
                continue
            m = {k: sum(v) / len(v) for k, v in c.items()}
            ds = next((v for k, v in dur.items() if short(k) == short(name) and k.split("(")[0] == name.split("(")[0]), None)
            if ds is None or ds[2] < 0.5:
                continue
            mf = m.get("SQ_INSTS_MFMA", 0.0)
            grbm = m.get("GRBM_GUI_ACTIVE", 0.0)
            busy = m.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0) / (grbm / 8 * 1024) if grbm else float("nan")
            wc = m["SQ_WAVE_CYCLES"]
            rows.append((ds[2], f"| {short(name)} | {ds[0]} | {ds[1]:.1f} | {ds[2]:.1f} | "
                                f"{m.get('SQ_INSTS_VALU', 0) / mf if mf else float('nan'):.2f} | {busy:.3f} | "
                                f"{m.get('SQ_ACTIVE_INST_VALU', 0) / wc:.3f} | {m.get('SQ_WAIT_INST_ANY', 0) / wc:.3f} | "
                                f"{m.get('SQ_LDS_BANK_CONFLICT', 0) / max(1.0, m.get('SQ_LDS_IDX_ACTIVE', 0)):.4f} |"))
        for _, r in sorted(rows, reverse=True):
            print(r)


if __name__ == "__main__":
    main()
