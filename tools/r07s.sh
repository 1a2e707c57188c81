#!/bin/bash
# round 5, session r07s: reverse graph with the index words kept in registers (one scan) — tests, kernel time
set -o pipefail
export PYTHONDONTWRITEBYTECODE=1
mkdir -p gpurun_out
T="--timeout 120 --timeout-method thread"
timeout -k 10 240 python -u -m pytest tests/test_graph_reverse_gpu.py -x -q $T > gpurun_out/r07s_tests0.log 2>&1 || { tail -30 gpurun_out/r07s_tests0.log; exit 1; }
tail -1 gpurun_out/r07s_tests0.log
timeout -k 10 400 python -u -m pytest tests/test_graph_feature_gpu.py tests/test_edgeconv_gpu.py tests/test_model_gpu.py tests/test_fused_finalize_gpu.py -x -q $T > gpurun_out/r07s_tests.log 2>&1 || { tail -30 gpurun_out/r07s_tests.log; exit 1; }
tail -1 gpurun_out/r07s_tests.log
for v in reg sort; do
  L=$(pwd)/labs_rg_$v.so; [ $v = reg ] && L=$(pwd)/dgcnn.pytorch_amd/dgx/libdgx.so
  DGX_LIB=$L KT_ONLY=1 timeout -k 10 300 bash tools/profile.sh r07s_$v --steps 10 --warmup 3 > gpurun_out/r07s_prof_$v.log 2>&1 || { tail -20 gpurun_out/r07s_prof_$v.log; exit 1; }
  echo "$v: $(grep rev_graph gpurun_out/prof_r07s_$v/kt_summary.txt)"
done
