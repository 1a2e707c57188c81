#!/bin/bash
# round 5, session r07x: split dPQ planes as a separate scatter instantiation — tests, bf16 scatter time vs the pre-split build, step A/B
set -o pipefail
export PYTHONDONTWRITEBYTECODE=1
mkdir -p gpurun_out
T="--timeout 120 --timeout-method thread"
timeout -k 10 400 python -u -m pytest tests/test_scatter_push_gpu.py tests/test_fused_finalize_gpu.py tests/test_edgeconv_gpu.py tests/test_host_ext_gpu.py -x -q $T > gpurun_out/r07x_tests.log 2>&1 || { tail -30 gpurun_out/r07x_tests.log; exit 1; }
tail -1 gpurun_out/r07x_tests.log
for v in new pre; do
  L=$(pwd)/labs_$v.so; [ $v = new ] && L=$(pwd)/dgcnn.pytorch_amd/dgx/libdgx.so
  DGX_LIB=$L KT_ONLY=1 timeout -k 10 300 bash tools/profile.sh r07x_$v --steps 10 --warmup 3 > gpurun_out/r07x_prof_$v.log 2>&1 || { tail -20 gpurun_out/r07x_prof_$v.log; exit 1; }
  echo "$v: $(grep 'edge_bwd_scatter_kernel' gpurun_out/prof_r07x_$v/kt_summary.txt)"
done
timeout -k 10 600 bash tools/ab_lib.sh labs_pre.so dgcnn.pytorch_amd/dgx/libdgx.so 2 > gpurun_out/r07x_ab.log 2>&1; cat gpurun_out/r07x_ab.log
