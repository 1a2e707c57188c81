#!/bin/bash
# round 5, session r07n: fp32 stacked weights in one launch
# fp32 suites, gemm tests, fp32 bench + trace
set -o pipefail
export PYTHONDONTWRITEBYTECODE=1
mkdir -p gpurun_out
T="--timeout 300 --timeout-method thread"
timeout -k 10 600 python -u -m pytest tests/test_gemm_gpu.py tests/test_edgeconv_gpu.py tests/test_model_gpu.py tests/test_host_ext_gpu.py tests/test_batch1_gpu.py tests/test_edge_mode_gpu.py -q $T > gpurun_out/r07n_tests.log 2>&1; rc=$?
tail -3 gpurun_out/r07n_tests.log
[ $rc -eq 0 ] || exit 1
for r in 1 2; do
timeout -k 10 300 python -u bench.py --precision fp32 --steps 30 --warmup 5 --no-cpu-baseline --no-eager-baseline --no-edgeconv-leg --no-posemb-leg --no-attention-leg > gpurun_out/r07n_bench_fp32.log 2>&1 || { tail -30 gpurun_out/r07n_bench_fp32.log; exit 1; }
grep -o '"ms_per_step": [0-9.]*' gpurun_out/r07n_bench_fp32.log | head -1
done
