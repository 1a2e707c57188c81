#!/bin/bash
# round 5, session o: round-4 kNN restored; whole GPU suite, smoke, bench
set -o pipefail
export PYTHONDONTWRITEBYTECODE=1
mkdir -p gpurun_out
T="--timeout 300 --timeout-method thread"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q $T > gpurun_out/r06o_pytest_gpu.log 2>&1 || { tail -60 gpurun_out/r06o_pytest_gpu.log; exit 1; }
tail -2 gpurun_out/r06o_pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" || exit 1
timeout -k 10 400 python -u bench.py > gpurun_out/r06o_bench.log 2>&1 || { tail -30 gpurun_out/r06o_bench.log; exit 1; }
tail -c 2500 gpurun_out/r06o_bench.log
