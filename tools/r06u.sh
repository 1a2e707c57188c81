#!/bin/bash
# round 5, session u: push scatter (chunked push) + fp32 conv5 split passes: tests, A/B bench, traces, cfg4 split32 probe
set -o pipefail
export PYTHONDONTWRITEBYTECODE=1
mkdir -p gpurun_out
T="--timeout 300 --timeout-method thread"
timeout -k 10 300 python -u -m pytest tests/test_scatter_push_gpu.py tests/test_pointconv_split_gpu.py -q -s $T > gpurun_out/r06u_tests.log 2>&1; rc=$?
grep -E "push |passed|failed|Error" gpurun_out/r06u_tests.log | head -30
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 1
for v in 1 0 1 0; do
  DGX_SCATTER_PUSH=$v timeout -k 10 300 python -u bench.py --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/r06u_bench_push$v.log 2>&1 || { tail -30 gpurun_out/r06u_bench_push$v.log; exit 1; }
  echo "push=$v $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r06u_bench_push$v.log | head -2 | tr '\n' ' ')"
done
KT_ONLY=1 timeout -k 10 400 bash tools/profile.sh r06u_cfg2 --steps 10 --warmup 3 > gpurun_out/r06u_prof_cfg2.log 2>&1 || { tail -20 gpurun_out/r06u_prof_cfg2.log; exit 1; }
head -12 gpurun_out/prof_r06u_cfg2/kt_summary.txt
KT_ONLY=1 timeout -k 10 400 bash tools/profile.sh r06u_fp32 --precision fp32 --steps 10 --warmup 3 > gpurun_out/r06u_prof_fp32.log 2>&1 || { tail -20 gpurun_out/r06u_prof_fp32.log; exit 1; }
head -24 gpurun_out/prof_r06u_fp32/kt_summary.txt
DGX_SPLIT32=0 timeout -k 10 300 python -u -m pytest tests/test_partseg.py -q -s -k "cfg4_routed and False" $T > gpurun_out/r06u_cfg4_nosplit.log 2>&1; rc=$?
grep -E "Net cfg4|passed|failed" gpurun_out/r06u_cfg4_nosplit.log | cut -c1-600
exit 0
