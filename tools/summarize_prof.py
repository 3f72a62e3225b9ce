"""Turn a tools/profile_bench.sh run (gpurun_out/prof_TAG_CONFIG) into the committed evidence under profiles/:

  profiles/TAG_CONFIG_bench_kernel_stats.csv  rocprofv3 --kernel-trace --stats summary of the bench command
  profiles/TAG_CONFIG_traffic.json            per-kernel HBM traffic per launch from the FETCH_SIZE / WRITE_SIZE
                                              passes (FETCH_SIZE doubled: MI355X_MICROARCH.md §HBM, 16-B streaming
                                              reads are tallied at half their bytes; values are KiB in rocprofv3),
                                              keyed by config / rows / precision for bench.py measured_traffic()

Usage: python tools/summarize_prof.py TAG [CONFIG [BATCH [PRECISION]]]
"""
import csv
import json
import os
import shutil
import sys
from collections import defaultdict

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def short(name):
    n = name.replace("(anonymous namespace)::", "").replace("void ", "")
    return n.split("(")[0].replace("pdm::", "")


def per_kernel(path, counter):
    acc = defaultdict(lambda: [0.0, 0])
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter:
            continue
        k = short(r["Kernel_Name"]) + f" grid={r['Grid_Size']}"
        acc[k][0] += float(r["Counter_Value"])
        acc[k][1] += 1
    return {k: (v[0] / v[1], v[1]) for k, v in acc.items()}


def roofline_check(src, bench_log):
    """The bench line's roofline kernel time, recomputed from the kernel trace: the bench times the GEMM launches of
    the LAST forward of its eager roofline pass (after the timed region; nothing else runs on the GPU after it), so
    the last `launches_per_forward` GEMM launches of the trace by start time are those launches."""
    trace = os.path.join(src, "kt", "run_kernel_trace.csv")
    if not (os.path.exists(trace) and os.path.exists(bench_log)):
        return None
    line = [l for l in open(bench_log) if l.startswith("{")]
    if not line:
        return None
    roof = json.loads(line[-1]).get("roofline") or {}
    n = roof.get("launches_per_forward")
    if not n:
        return None
    rows = []
    for r in csv.DictReader(open(trace)):
        name = short(r["Kernel_Name"])
        if name.startswith("gemm"):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]) - int(r["Start_Timestamp"]), name))
    rows.sort()
    last = rows[-n:]
    avg_ms = sum(d for _, d, _ in last) / len(last) / 1e6
    by = defaultdict(list)
    for _, d, k in last:
        by[k].append(d)
    return {"launches": len(last), "avg_launch_ms_rocprof": round(avg_ms, 4),
            "avg_launch_ms_bench": roof.get("avg_launch_ms"),
            "per_kernel_avg_ms": {k: round(sum(v) / len(v) / 1e6, 4) for k, v in sorted(by.items())},
            "note": "the bench's HIP-event average over the same launches (last forward of the eager roofline pass)"}


def main():
    tag = sys.argv[1]
    config = sys.argv[2] if len(sys.argv) > 2 else "imagenet256_uvit_large"
    batch = int(sys.argv[3]) if len(sys.argv) > 3 else 95
    precision = sys.argv[4] if len(sys.argv) > 4 else "bf16"
    src = os.path.join(REPO, "gpurun_out", f"prof_{tag}_{config}")
    dst = os.environ.get("PDM_PROF_DST") or os.path.join(REPO, "profiles")   # on the GPU box: a gpurun_out dir
    os.makedirs(dst, exist_ok=True)
    kt = os.path.join(src, "kt", "run_kernel_stats.csv")
    if os.path.exists(kt):
        shutil.copy(kt, os.path.join(dst, f"{tag}_{config}_bench_kernel_stats.csv"))
    roof = roofline_check(src, os.path.join(src, "bench_kt.log"))
    fetch = per_kernel(os.path.join(src, "fetch", "run_counter_collection.csv"), "FETCH_SIZE")
    write = per_kernel(os.path.join(src, "write", "run_counter_collection.csv"), "WRITE_SIZE")
    out = {"config": config, "rows": 2 * batch, "precision": precision,
           "source": f"rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE (separate passes) over tools/time_forward.py "
                     f"{config} {2 * batch} 2 {precision} (CFG forwards at the bench batch, {batch} images x 2 rows)",
           "correction": "fetch_bytes = FETCH_SIZE[KiB] x 1024 x 2 (gfx950 tallies 16-B streaming reads at half); "
                         "write_bytes = WRITE_SIZE[KiB] x 1024",
           "kernels": {}}
    gemm_f = gemm_w = gemm_n = 0.0
    for k in sorted(set(fetch) | set(write)):
        f, n = fetch.get(k, (0.0, 0))
        w, _ = write.get(k, (0.0, 0))
        fb, wb = f * 1024 * 2, w * 1024
        out["kernels"][k] = {"launches": n, "fetch_bytes_per_launch": round(fb), "write_bytes_per_launch": round(wb)}
        if k.startswith("gemm"):
            gemm_f += fb * n
            gemm_w += wb * n
            gemm_n += n
    if gemm_n:
        out["gemm_family"] = {"launches": int(gemm_n), "hbm_bytes_per_launch": round((gemm_f + gemm_w) / gemm_n)}
    if roof:
        out["roofline_check"] = roof
    json.dump(out, open(os.path.join(dst, f"{tag}_{config}_traffic.json"), "w"), indent=1)
    print(json.dumps(out.get("gemm_family"), indent=1))


if __name__ == "__main__":
    main()
