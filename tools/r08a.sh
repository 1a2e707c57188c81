#!/bin/bash
# round 5, session r08a: 4-cloud shard kernel trace (where the strong-scaling step goes)
set -o pipefail
export PYTHONDONTWRITEBYTECODE=1
mkdir -p gpurun_out
KT_ONLY=1 timeout -k 10 400 bash tools/profile.sh r08a_b4 --batch 4 --steps 20 --warmup 3 > gpurun_out/r08a_prof_b4.log 2>&1 || { tail -20 gpurun_out/r08a_prof_b4.log; exit 1; }
head -36 gpurun_out/prof_r08a_b4/kt_summary.txt
