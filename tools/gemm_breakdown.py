#!/usr/bin/env python3
"""Per-Linear timing of the U-ViT forward from a rocprofv3 kernel trace (run_kernel_trace.csv of
tools/profile_bench.sh): every block GEMM launch is classified by its predecessor in stream order
(qkv -> attention -> proj -> fc1 -> fc2, out-blocks open with skip_linear), then reported with its algorithmic
TFLOP/s and its epilogue + operand HBM bytes at that rate.

  python tools/gemm_breakdown.py TRACE.csv CONFIG ROWS
"""
import collections
import csv
import sys

sys.path.insert(0, ".")
from panopticdiffusionmodels_amd import configs  # noqa: E402


def main():
    path, name, rows = sys.argv[1], sys.argv[2], int(sys.argv[3])
    cfg = configs.nnet_kwargs(name)
    D = cfg["embed_dim"]
    Hd = int(D * cfg.get("mlp_ratio", 4))
    L = (cfg["img_size"] // cfg["patch_size"]) ** 2 + (2 if cfg.get("num_classes", -1) > 0 else 1)
    M = rows * L
    # (FLOPs, algorithmic HBM bytes): A operand(s) + weights + what the epilogue reads / writes
    shapes = {"qkv": (2 * M * 3 * D * D, M * D * 2 + 3 * D * D * 2 + M * 3 * D * 2),
              "proj": (2 * M * D * D, M * D * 2 + D * D * 2 + M * D * (4 + 4 + 2)),
              "fc1": (2 * M * Hd * D, M * D * 2 + Hd * D * 2 + M * Hd * 2),
              "fc2": (2 * M * D * Hd, M * Hd * 2 + Hd * D * 2 + M * D * (4 + 4 + 2)),
              "skip": (2 * M * D * 2 * D, 2 * M * D * 2 + 2 * D * D * 2 + M * D * (4 + 2))}
    trace = list(csv.DictReader(open(path)))
    t = collections.defaultdict(list)
    prev = None
    for r in trace:
        n = r["Kernel_Name"]
        kind = None
        if "attention" in n:
            kind = "attn"
        elif "gemm" in n and "GemmArgs" in n:
            g = int(r["Grid_Size_X"]) // int(r["Workgroup_Size_X"])
            if prev == "attn":
                kind = "proj"
            elif prev == "fc1":
                kind = "fc2"
            elif prev in ("skip", "fc2", "proj_pre") or prev is None or prev == "other":
                kind = "skip" if g == (M + 255) // 256 * ((D + 255) // 256) else None
            if kind is None:
                kind = {3 * D: "qkv", Hd: "fc1"}.get(g // ((M + 255) // 256) * 256, "other")
        else:
            kind = "other"
        dur = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        if kind in shapes or kind == "attn":
            t[kind].append(dur)
        prev = kind
    print(f"{name} rows={rows} M={M}")
    for k in ("qkv", "proj", "fc1", "fc2", "skip", "attn"):
        v = t.get(k)
        if not v:
            continue
        us = sum(v) / len(v)
        if k in shapes:
            fl, by = shapes[k]
            print(f"  {k:5s} {len(v):6d} launches  {us:8.1f} us  {fl / us / 1e6:7.1f} TF/s  "
                  f"algorithmic {by / 1e6:7.1f} MB -> {by / us / 1e3:6.2f} TB/s")
        else:
            print(f"  {k:5s} {len(v):6d} launches  {us:8.1f} us")


if __name__ == "__main__":
    main()
