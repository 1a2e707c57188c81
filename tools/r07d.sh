#!/bin/bash
# round 5, session r07d: one-launch SGD (dgx.optim.SGD): parity test, fused-torch vs dgx A/B at cfg2 and B=4
set -o pipefail
export PYTHONDONTWRITEBYTECODE=1
mkdir -p gpurun_out
T="--timeout 300 --timeout-method thread"
timeout -k 10 300 python -u -m pytest tests/test_optim_gpu.py -q $T > gpurun_out/r07d_tests.log 2>&1; rc=$?
tail -3 gpurun_out/r07d_tests.log
[ $rc -eq 0 ] || exit 1
A="--steps 30 --warmup 5 --no-cpu-baseline --no-eager-baseline --no-edgeconv-leg --no-posemb-leg --no-attention-leg --no-fp32-leg"
for s in fused dgx fused dgx; do
  timeout -k 10 300 python -u bench.py $A --sgd $s > gpurun_out/r07d_sgd_$s.log 2>&1 || { tail -20 gpurun_out/r07d_sgd_$s.log; exit 1; }
  timeout -k 10 300 python -u bench.py --batch 4 $A --sgd $s > gpurun_out/r07d_sgd_b4_$s.log 2>&1 || { tail -20 gpurun_out/r07d_sgd_b4_$s.log; exit 1; }
  echo "$s cfg2 $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r07d_sgd_$s.log | head -1) b4 $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r07d_sgd_b4_$s.log | head -1)"
done
