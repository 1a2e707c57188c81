#!/bin/bash
# round 5, session q: whole GPU suite (recorded, not gating), smoke, cfg2 bench, final-tree kernel trace +
# PMC passes, the 4-cloud shard, cfg3 / cfg5 bench lines
set -o pipefail
export PYTHONDONTWRITEBYTECODE=1
mkdir -p gpurun_out
T="--timeout 300 --timeout-method thread"
timeout -k 10 900 python -u -m pytest tests -m gpu -q $T -rf > gpurun_out/r06q_pytest_gpu.log 2>&1; rc=$?
tail -4 gpurun_out/r06q_pytest_gpu.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" || exit 1
timeout -k 10 400 python -u bench.py > gpurun_out/r06q_bench.log 2>&1 || { tail -30 gpurun_out/r06q_bench.log; exit 1; }
tail -c 2500 gpurun_out/r06q_bench.log
bash tools/r06p.sh
