#!/bin/bash
# round 5, session r07u: fp32 mode EdgeConv dW / dX as 3-pass split bf16 on the scatter's split dPQ planes —
# whole GPU suite, fp32 bench A/B (DGX_SPLIT32_EDGE=1 / 0), fp32 kernel trace
set -o pipefail
export PYTHONDONTWRITEBYTECODE=1
mkdir -p gpurun_out
T="--timeout 300 --timeout-method thread"
timeout -k 10 900 python -u -m pytest tests -m gpu -q $T -rf > gpurun_out/r07u_pytest_gpu.log 2>&1; rc=$?
tail -12 gpurun_out/r07u_pytest_gpu.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 1
A="--precision fp32 --steps 30 --warmup 5 --no-cpu-baseline --no-eager-baseline --no-edgeconv-leg --no-posemb-leg --no-attention-leg"
for r in 1 2; do
  for v in 1 0; do
    DGX_SPLIT32_EDGE=$v timeout -k 10 300 python -u bench.py $A > gpurun_out/r07u_bench_fp32_$v.log 2>&1 || { tail -30 gpurun_out/r07u_bench_fp32_$v.log; exit 1; }
    echo "edge split $v: $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r07u_bench_fp32_$v.log | head -1)"
  done
done
KT_ONLY=1 timeout -k 10 400 bash tools/profile.sh r07u_fp32 --precision fp32 --steps 10 --warmup 3 > gpurun_out/r07u_prof_fp32.log 2>&1 || { tail -20 gpurun_out/r07u_prof_fp32.log; exit 1; }
head -24 gpurun_out/prof_r07u_fp32/kt_summary.txt
exit $rc
