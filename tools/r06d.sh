#!/bin/bash
# round 5, session d: kNN phase lab (clock marks) + the DDP AMP tests
set -o pipefail
export PYTHONDONTWRITEBYTECODE=1
mkdir -p gpurun_out
T="--timeout 300 --timeout-method thread"
timeout -k 10 120 ./tools/knn_lab 20 > gpurun_out/r06d_lab.log 2>&1; rc=$?; cat gpurun_out/r06d_lab.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 600 python -u -m pytest tests/test_ddp_gpu.py -x -q -s $T -k autocast > gpurun_out/r06d_pytest_ddp.log 2>&1 || { tail -40 gpurun_out/r06d_pytest_ddp.log; exit 1; }
grep -E "rel err|passed|failed" gpurun_out/r06d_pytest_ddp.log
