#!/bin/bash
# round 5, session r07y: final tree — whole GPU suite, default bench line, b4/cfg3/cfg5 lines, kernel traces
set -o pipefail
export PYTHONDONTWRITEBYTECODE=1
mkdir -p gpurun_out
T="--timeout 300 --timeout-method thread"
timeout -k 10 900 python -u -m pytest tests -m gpu -q $T -rf > gpurun_out/r07y_pytest_gpu.log 2>&1; rc=$?
tail -4 gpurun_out/r07y_pytest_gpu.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 1
timeout -k 10 400 python -u bench.py > gpurun_out/r07y_bench.log 2>&1 || { tail -30 gpurun_out/r07y_bench.log; exit 1; }
grep -o '"ms_per_step": [0-9.]*' gpurun_out/r07y_bench.log | head -3
A="--no-cpu-baseline --no-eager-baseline --no-edgeconv-leg --no-posemb-leg --no-attention-leg"
timeout -k 10 300 python -u bench.py --batch 4 $A --no-fp32-leg > gpurun_out/r07y_bench_b4.log 2>&1 || { tail -20 gpurun_out/r07y_bench_b4.log; exit 1; }
timeout -k 10 300 python -u bench.py --config cfg3 $A --no-fp32-leg > gpurun_out/r07y_bench_cfg3.log 2>&1 || { tail -20 gpurun_out/r07y_bench_cfg3.log; exit 1; }
timeout -k 10 300 python -u bench.py --config cfg5 $A --no-fp32-leg > gpurun_out/r07y_bench_cfg5.log 2>&1 || { tail -20 gpurun_out/r07y_bench_cfg5.log; exit 1; }
for f in b4 cfg3 cfg5; do echo "$f $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r07y_bench_$f.log | head -1)"; done
KT_ONLY=1 timeout -k 10 400 bash tools/profile.sh r07y_cfg2 --steps 10 --warmup 3 > gpurun_out/r07y_prof_cfg2.log 2>&1 || { tail -20 gpurun_out/r07y_prof_cfg2.log; exit 1; }
KT_ONLY=1 timeout -k 10 400 bash tools/profile.sh r07y_fp32 --precision fp32 --steps 10 --warmup 3 > gpurun_out/r07y_prof_fp32.log 2>&1 || { tail -20 gpurun_out/r07y_prof_fp32.log; exit 1; }
head -14 gpurun_out/prof_r07y_cfg2/kt_summary.txt
exit $rc
