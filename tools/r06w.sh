#!/bin/bash
# round 5, session w: whole GPU suite on the committed tree, default bench line, cfg2 + fp32 kernel traces
set -o pipefail
export PYTHONDONTWRITEBYTECODE=1
mkdir -p gpurun_out
T="--timeout 300 --timeout-method thread"
timeout -k 10 900 python -u -m pytest tests -m gpu -q $T -rf > gpurun_out/r06w_pytest_gpu.log 2>&1; rc=$?
tail -5 gpurun_out/r06w_pytest_gpu.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 1
timeout -k 10 400 python -u bench.py > gpurun_out/r06w_bench.log 2>&1 || { tail -30 gpurun_out/r06w_bench.log; exit 1; }
grep -o '"ms_per_step": [0-9.]*' gpurun_out/r06w_bench.log | head -3
KT_ONLY=1 timeout -k 10 400 bash tools/profile.sh r06w_cfg2 --steps 10 --warmup 3 > gpurun_out/r06w_prof_cfg2.log 2>&1 || { tail -20 gpurun_out/r06w_prof_cfg2.log; exit 1; }
KT_ONLY=1 timeout -k 10 400 bash tools/profile.sh r06w_fp32 --precision fp32 --steps 10 --warmup 3 > gpurun_out/r06w_prof_fp32.log 2>&1 || { tail -20 gpurun_out/r06w_prof_fp32.log; exit 1; }
head -12 gpurun_out/prof_r06w_cfg2/kt_summary.txt
exit $rc
