#!/bin/bash
# round 5, session v: push-scatter phase lab, fp32 GEMM (BK 32) tests, cfg4 routed modes, fp32 bench
set -o pipefail
export PYTHONDONTWRITEBYTECODE=1
mkdir -p gpurun_out
T="--timeout 300 --timeout-method thread"
timeout -k 10 300 python -u tools/push_lab.py > gpurun_out/r06v_push_lab.log 2>&1 || { tail -20 gpurun_out/r06v_push_lab.log; exit 1; }
cat gpurun_out/r06v_push_lab.log
timeout -k 10 600 python -u -m pytest tests/test_gemm_gpu.py tests/test_pointconv_split_gpu.py tests/test_partseg.py -q -s -k "gemm or f32 or split or cfg4_routed" $T > gpurun_out/r06v_tests.log 2>&1; rc=$?
grep -E "Net cfg4|passed|failed|Error" gpurun_out/r06v_tests.log | cut -c1-400 | head -20
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 1
DGX_SCATTER_PUSH=0 timeout -k 10 300 python -u bench.py --precision fp32 --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/r06v_bench_fp32.log 2>&1 || { tail -30 gpurun_out/r06v_bench_fp32.log; exit 1; }
grep -o '"ms_per_step": [0-9.]*' gpurun_out/r06v_bench_fp32.log | head -2
DGX_SCATTER_PUSH=0 KT_ONLY=1 timeout -k 10 400 bash tools/profile.sh r06v_fp32 --precision fp32 --steps 10 --warmup 3 > gpurun_out/r06v_prof_fp32.log 2>&1 || { tail -20 gpurun_out/r06v_prof_fp32.log; exit 1; }
head -24 gpurun_out/prof_r06v_fp32/kt_summary.txt
