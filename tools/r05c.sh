#!/bin/bash
# final tree: full GPU suite + default bench + kernel trace (gpu_suite.sh), then the 4-cloud shard bench line
set -o pipefail
bash tools/gpu_suite.sh r05c || exit 1
timeout -k 10 300 python -u bench.py --batch 4 --no-cpu-baseline --no-eager-baseline --no-fp32-leg --no-edgeconv-leg \
    --no-posemb-leg --no-attention-leg > gpurun_out/r05c_bench_b4.log 2>&1 || { tail -20 gpurun_out/r05c_bench_b4.log; exit 1; }
tail -c 600 gpurun_out/r05c_bench_b4.log
