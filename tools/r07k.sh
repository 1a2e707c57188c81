#!/bin/bash
# round 5, session r07k: fp32 GEMM with 128-wide tiles: gemm tests, fp32 routed suites, fp32 bench + trace
set -o pipefail
export PYTHONDONTWRITEBYTECODE=1
mkdir -p gpurun_out
T="--timeout 300 --timeout-method thread"
timeout -k 10 600 python -u -m pytest tests/test_gemm_gpu.py tests/test_edgeconv_gpu.py tests/test_model_gpu.py tests/test_edgemlp_gpu.py -q $T > gpurun_out/r07k_tests.log 2>&1; rc=$?
tail -3 gpurun_out/r07k_tests.log
[ $rc -eq 0 ] || exit 1
for r in 1 2; do
timeout -k 10 300 python -u bench.py --precision fp32 --steps 30 --warmup 5 --no-cpu-baseline --no-eager-baseline --no-edgeconv-leg --no-posemb-leg --no-attention-leg > gpurun_out/r07k_bench_fp32.log 2>&1 || { tail -30 gpurun_out/r07k_bench_fp32.log; exit 1; }
grep -o '"ms_per_step": [0-9.]*' gpurun_out/r07k_bench_fp32.log | head -1
done
KT_ONLY=1 timeout -k 10 400 bash tools/profile.sh r07k_fp32 --precision fp32 --steps 10 --warmup 3 > gpurun_out/r07k_prof_fp32.log 2>&1 || { tail -20 gpurun_out/r07k_prof_fp32.log; exit 1; }
grep gemm32 gpurun_out/prof_r07k_fp32/kt_summary.txt
