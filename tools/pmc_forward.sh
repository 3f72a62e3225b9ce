#!/bin/bash
# SQ-counter passes (one rocprofv3 --pmc run per pass, each time-limited) over whole workloads, so every kernel of
# the path is counted at its real shapes: the L/2 bf16 forward (gemm8s, attention_v2), the H/4 MXFP8 forward
# (gemm_mx, gemm8s MX output, attention_h72), the t2i forward (L = 334 / 590 attention) and a training step
# (wgrad_kernel, attn_bwd_kernel).  Summaries: python3 tools/pmc_kernels.py gpurun_out/<tag>.
OUT=${GRAFT_REPO_ROOT:-.}/gpurun_out/${1:-r04pmc}
mkdir -p $OUT
export TMPDIR=/tmp
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU"
P2="SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE GRBM_COUNT"
run() {   # tag, command...
  local tag=$1; shift
  timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $OUT/$tag/kt -o run --output-format csv -- "$@" > $OUT/$tag.kt.log 2>&1 || return $?
  timeout -s KILL 180 rocprofv3 --pmc $P1 -d $OUT/$tag/p1 -o run --output-format csv -- "$@" > $OUT/$tag.p1.log 2>&1 || return $?
  timeout -s KILL 180 rocprofv3 --pmc $P2 -d $OUT/$tag/p2 -o run --output-format csv -- "$@" > $OUT/$tag.p2.log 2>&1 || return $?
  echo "pmc done: $tag"
}
run l2_fwd python3 tools/time_forward.py imagenet256_uvit_large 100 2 bf16 || exit $?
run h4_fwd python3 tools/time_forward.py imagenet512_uvit_huge 100 2 fp8 || exit $?
run t2i_fwd python3 tools/time_forward.py mscoco_uvit_small 100 2 bf16 || exit $?
run l2_train python3 tools/train_bench.py --config imagenet256_uvit_large --batch 64 --steps 2 --warmup 1 || exit $?
# summarise on the box, then keep only the per-kernel stats (the per-dispatch CSVs exceed what gpurun returns)
python3 tools/pmc_kernels.py $OUT > $OUT/SUMMARY.md
for t in l2_fwd h4_fwd t2i_fwd l2_train; do
  find $OUT/$t -type f ! -name 'run_kernel_stats.csv' -delete
done
cat $OUT/SUMMARY.md
echo done
