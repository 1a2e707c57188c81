#!/bin/bash
# round 5, session r07q: reverse graph ranges per cloud (P) variants
set -o pipefail
export PYTHONDONTWRITEBYTECODE=1
mkdir -p gpurun_out
T="--timeout 300 --timeout-method thread"
timeout -k 10 400 python -u -m pytest tests/test_graph_reverse_gpu.py -q $T > gpurun_out/r07q_tests.log 2>&1 || { tail -30 gpurun_out/r07q_tests.log; exit 1; }
tail -2 gpurun_out/r07q_tests.log
for v in xcd p8 p2; do
  L=$(pwd)/labs_rg_$v.so; [ $v = xcd ] && L=$(pwd)/dgcnn.pytorch_amd/dgx/libdgx.so
  DGX_LIB=$L KT_ONLY=1 timeout -k 10 300 bash tools/profile.sh r07q_$v --steps 10 --warmup 3 > gpurun_out/r07q_prof_$v.log 2>&1 || { tail -20 gpurun_out/r07q_prof_$v.log; exit 1; }
  echo "$v: $(grep rev_graph gpurun_out/prof_r07q_$v/kt_summary.txt)"
done
