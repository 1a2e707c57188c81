#!/bin/bash
# round 5, session r07j: final-tree PMC passes (cfg2, cfg3, cfg5) for bench's roofline traffic and the kernel bounds
set -o pipefail
export PYTHONDONTWRITEBYTECODE=1
mkdir -p gpurun_out
timeout -k 10 600 bash tools/profile.sh r07j_cfg2 --steps 10 --warmup 3 > gpurun_out/r07j_prof_cfg2.log 2>&1 || { tail -20 gpurun_out/r07j_prof_cfg2.log; exit 1; }
timeout -k 10 500 bash tools/profile.sh r07j_cfg3 --config cfg3 --steps 4 --warmup 2 > gpurun_out/r07j_prof_cfg3.log 2>&1 || { tail -20 gpurun_out/r07j_prof_cfg3.log; exit 1; }
timeout -k 10 500 bash tools/profile.sh r07j_cfg5 --config cfg5 --steps 4 --warmup 2 > gpurun_out/r07j_prof_cfg5.log 2>&1 || { tail -20 gpurun_out/r07j_prof_cfg5.log; exit 1; }
echo done
