#!/bin/bash
# B=4 shard (strong-scaling unit): bench line + kernel trace
set -o pipefail
export PYTHONDONTWRITEBYTECODE=1
timeout -k 10 200 python3 bench.py --batch 4 --no-cpu-baseline --no-eager-baseline --no-posemb-leg --no-edgeconv-leg \
    --no-attention-leg --no-fp32-leg --steps 50 --warmup 10 > gpurun_out/r04o_bench_b4.log 2>&1 || { tail gpurun_out/r04o_bench_b4.log; exit 1; }
tail -c 300 gpurun_out/r04o_bench_b4.log
KT_ONLY=1 timeout -k 10 300 bash tools/profile.sh r04o_b4 --batch 4 --steps 5 --warmup 2 > gpurun_out/r04o_prof.log 2>&1 || { tail gpurun_out/r04o_prof.log; exit 1; }
head -40 gpurun_out/prof_r04o_b4/kt_summary.txt
