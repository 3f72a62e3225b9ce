#!/bin/bash
# Round 6: epilogue change A/B (working-tree libpdm.so vs ab/libpdm_head.so) + the GEMM / forward tests it touches
set -o pipefail
O=gpurun_out/${1:-r06h}; mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_streamk.py -k "gemm or streamk" > $O/pytest.txt 2>&1 || exit 1
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_uvit.py tests/test_fullsize_golden.py -k "forward" > $O/pytest_fwd.txt 2>&1 || exit 1
for r in 1 2; do
  for lib in ab/libpdm_head.so panopticdiffusionmodels_amd/libpdm.so; do
    for rows in 100 50; do
      echo "== $lib rows $rows" >> $O/ab.txt
      PDM_LIB_PATH=$lib timeout -k 10 120 python tools/g8s_diag.py $rows 2>&1 | grep -v amdgpu.ids >> $O/ab.txt || exit 1
    done
  done
done
