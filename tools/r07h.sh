#!/bin/bash
# round 5, session r07h: per-job vectorised slab reduce (tests, bench, trace) + final-tree PMC passes cfg2/cfg3/cfg5
set -o pipefail
export PYTHONDONTWRITEBYTECODE=1
mkdir -p gpurun_out
T="--timeout 300 --timeout-method thread"
timeout -k 10 600 python -u -m pytest tests/test_gemm_gpu.py tests/test_host_ext_gpu.py tests/test_edgeconv_gpu.py tests/test_fused_finalize_gpu.py tests/test_scatter_push_gpu.py tests/test_model_gpu.py -q $T > gpurun_out/r07h_tests.log 2>&1; rc=$?
tail -3 gpurun_out/r07h_tests.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -u bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-eager-baseline --no-edgeconv-leg --no-posemb-leg --no-attention-leg > gpurun_out/r07h_bench.log 2>&1 || { tail -30 gpurun_out/r07h_bench.log; exit 1; }
grep -o '"ms_per_step": [0-9.]*' gpurun_out/r07h_bench.log | head -2
timeout -k 10 900 bash tools/profile.sh r07h_cfg2 --steps 10 --warmup 3 > gpurun_out/r07h_prof_cfg2.log 2>&1 || { tail -20 gpurun_out/r07h_prof_cfg2.log; exit 1; }
grep -E "slab_reduce|sgd_kernel|scatter" gpurun_out/prof_r07h_cfg2/kt_summary.txt
timeout -k 10 900 bash tools/profile.sh r07h_cfg3 --config cfg3 --steps 4 --warmup 2 > gpurun_out/r07h_prof_cfg3.log 2>&1 || { tail -20 gpurun_out/r07h_prof_cfg3.log; exit 1; }
timeout -k 10 900 bash tools/profile.sh r07h_cfg5 --config cfg5 --steps 4 --warmup 2 > gpurun_out/r07h_prof_cfg5.log 2>&1 || { tail -20 gpurun_out/r07h_prof_cfg5.log; exit 1; }
echo done
