#!/bin/bash
# round 5, session p: final-tree kernel trace + PMC passes (cfg2), the 4-cloud shard, cfg3 / cfg5 bench lines
set -o pipefail
export PYTHONDONTWRITEBYTECODE=1
mkdir -p gpurun_out
timeout -k 10 900 bash tools/profile.sh r06q_cfg2 --config cfg2 --steps 10 --warmup 3 > gpurun_out/r06q_profile.log 2>&1 || { tail -20 gpurun_out/r06q_profile.log; exit 1; }
tail -3 gpurun_out/r06q_profile.log
FAST="--no-cpu-baseline --no-eager-baseline --no-posemb-leg --no-attention-leg --no-edgeconv-leg --no-fp32-leg"
timeout -k 10 300 python -u bench.py --batch 4 --steps 20 --warmup 5 $FAST > gpurun_out/r06q_bench_b4.log 2>&1 || { tail -20 gpurun_out/r06q_bench_b4.log; exit 1; }
tail -c 600 gpurun_out/r06q_bench_b4.log
timeout -k 10 300 python -u bench.py --config cfg3 --steps 10 --warmup 3 $FAST > gpurun_out/r06q_bench_cfg3.log 2>&1 || { tail -20 gpurun_out/r06q_bench_cfg3.log; exit 1; }
tail -c 600 gpurun_out/r06q_bench_cfg3.log
timeout -k 10 300 python -u bench.py --config cfg5 --steps 10 --warmup 3 $FAST > gpurun_out/r06q_bench_cfg5.log 2>&1 || { tail -20 gpurun_out/r06q_bench_cfg5.log; exit 1; }
tail -c 600 gpurun_out/r06q_bench_cfg5.log
