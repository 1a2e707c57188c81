#!/bin/bash
# round 5, session r: the AMP cfg4 routed test, kernel traces of the 4-cloud shard and of the fp32 mode
set -o pipefail
export PYTHONDONTWRITEBYTECODE=1
mkdir -p gpurun_out
T="--timeout 300 --timeout-method thread"
timeout -k 10 600 python -u -m pytest tests/test_partseg.py -q -s -k "cfg4_routed" $T > gpurun_out/r06r_pytest_cfg4.log 2>&1; rc=$?
grep -E "Net cfg4|passed|failed|Error" gpurun_out/r06r_pytest_cfg4.log | head -20
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 1
KT_ONLY=1 timeout -k 10 400 bash tools/profile.sh r06r_b4 --batch 4 --steps 10 --warmup 3 > gpurun_out/r06r_prof_b4.log 2>&1 || { tail -20 gpurun_out/r06r_prof_b4.log; exit 1; }
head -25 gpurun_out/prof_r06r_b4/kt_summary.txt
KT_ONLY=1 timeout -k 10 400 bash tools/profile.sh r06r_fp32 --precision fp32 --steps 10 --warmup 3 > gpurun_out/r06r_prof_fp32.log 2>&1 || { tail -20 gpurun_out/r06r_prof_fp32.log; exit 1; }
head -25 gpurun_out/prof_r06r_fp32/kt_summary.txt
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r06r_bench.log 2>&1 || { tail -30 gpurun_out/r06r_bench.log; exit 1; }
tail -c 1200 gpurun_out/r06r_bench.log
KT_ONLY=1 timeout -k 10 400 bash tools/profile.sh r06r_cfg2 --steps 10 --warmup 3 > gpurun_out/r06r_prof_cfg2.log 2>&1 || { tail -20 gpurun_out/r06r_prof_cfg2.log; exit 1; }
head -16 gpurun_out/prof_r06r_cfg2/kt_summary.txt
