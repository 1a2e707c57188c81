#!/bin/bash
# round 5, session t: push-form scatter tests, cfg4 routed fp32 twice (determinism), bench + kernel trace, GPU suite
set -o pipefail
export PYTHONDONTWRITEBYTECODE=1
mkdir -p gpurun_out
T="--timeout 300 --timeout-method thread"
timeout -k 10 300 python -u -m pytest tests/test_scatter_push_gpu.py -q -s $T > gpurun_out/r06t_push.log 2>&1; rc=$?
grep -E "push |passed|failed|Error" gpurun_out/r06t_push.log | head -30
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 1
for r in 1 2; do
  timeout -k 10 300 python -u -m pytest tests/test_partseg.py -q -s -k "cfg4_routed and False" $T > gpurun_out/r06t_cfg4_$r.log 2>&1; rc=$?
  grep -E "Net cfg4|passed|failed" gpurun_out/r06t_cfg4_$r.log | cut -c1-600
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 1
done
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r06t_bench.log 2>&1 || { tail -30 gpurun_out/r06t_bench.log; exit 1; }
grep -o '"ms_per_step": [0-9.]*' gpurun_out/r06t_bench.log | head -3
KT_ONLY=1 timeout -k 10 400 bash tools/profile.sh r06t_cfg2 --steps 10 --warmup 3 > gpurun_out/r06t_prof_cfg2.log 2>&1 || { tail -20 gpurun_out/r06t_prof_cfg2.log; exit 1; }
head -16 gpurun_out/prof_r06t_cfg2/kt_summary.txt
timeout -k 10 900 python -u -m pytest tests -m gpu -q $T > gpurun_out/r06t_pytest_gpu.log 2>&1; rc=$?
tail -8 gpurun_out/r06t_pytest_gpu.log
exit $rc
