#!/bin/bash
# round 5, session i: kNN v3 selection (value-only top-KL lists + logs + ranking): lab, ragged debug, tests,
# bench + kernel trace; conv5 BN-backward stats kernel at 4 blocks/CU
set -o pipefail
export PYTHONDONTWRITEBYTECODE=1
mkdir -p gpurun_out
T="--timeout 300 --timeout-method thread"
R=$(pwd)
timeout -k 10 120 ./tools/knn_lab 20 > gpurun_out/r06i_lab.log 2>&1; rc=$?; cat gpurun_out/r06i_lab.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -u tools/knn_debug.py > gpurun_out/r06i_debug.log 2>&1; rc=$?; cat gpurun_out/r06i_debug.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 400 python -u -m pytest tests/test_knn_gpu.py tests/test_knn_adversarial_gpu.py tests/test_knn_generic_gpu.py -x -q $T > gpurun_out/r06i_pytest_knn.log 2>&1 || { tail -40 gpurun_out/r06i_pytest_knn.log; exit 1; }
tail -2 gpurun_out/r06i_pytest_knn.log
timeout -k 10 120 python -u tools/knn_bench.py 20 > gpurun_out/r06i_knn_bench.log 2>&1 && cat gpurun_out/r06i_knn_bench.log || exit 1
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r06i_bench.log 2>&1 || { tail -30 gpurun_out/r06i_bench.log; exit 1; }
tail -c 1500 gpurun_out/r06i_bench.log
KT_ONLY=1 timeout -k 10 400 bash tools/profile.sh r06i_cfg2 --steps 10 --warmup 3 > gpurun_out/r06i_prof.log 2>&1 || { tail -20 gpurun_out/r06i_prof.log; exit 1; }
head -30 gpurun_out/prof_r06i_cfg2/kt_summary.txt
