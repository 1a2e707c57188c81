#!/bin/bash
# round 5, session r07o: reverse-graph rank sort unrolled — kernel time per variant lib, step A/B, reverse-graph tests
set -o pipefail
export PYTHONDONTWRITEBYTECODE=1
mkdir -p gpurun_out
T="--timeout 300 --timeout-method thread"
timeout -k 10 400 python -u -m pytest tests/test_graph_reverse_gpu.py tests/test_graph_feature_gpu.py -q $T > gpurun_out/r07o_tests.log 2>&1 || { tail -30 gpurun_out/r07o_tests.log; exit 1; }
tail -2 gpurun_out/r07o_tests.log
for v in u8 base nosort u4; do
  L=$(pwd)/labs_rg_$v.so; [ $v = u8 ] && L=$(pwd)/dgcnn.pytorch_amd/dgx/libdgx.so
  DGX_LIB=$L KT_ONLY=1 timeout -k 10 300 bash tools/profile.sh r07o_$v --steps 10 --warmup 3 > gpurun_out/r07o_prof_$v.log 2>&1 || { tail -20 gpurun_out/r07o_prof_$v.log; exit 1; }
  echo "$v: $(grep rev_graph gpurun_out/prof_r07o_$v/kt_summary.txt)"
done
timeout -k 10 600 bash tools/ab_lib.sh labs_rg_base.so dgcnn.pytorch_amd/dgx/libdgx.so 3 > gpurun_out/r07o_ab.log 2>&1; cat gpurun_out/r07o_ab.log
