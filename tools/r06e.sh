#!/bin/bash
# round 5, session e: kNN octet merge — lab phases, then the kNN parity tests
set -o pipefail
export PYTHONDONTWRITEBYTECODE=1
mkdir -p gpurun_out
T="--timeout 300 --timeout-method thread"
timeout -k 10 120 ./tools/knn_lab 20 > gpurun_out/r06e_lab.log 2>&1; rc=$?; cat gpurun_out/r06e_lab.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 120 ./tools/knn_lab_pipe 20 > gpurun_out/r06e_lab_pipe.log 2>&1; rc=$?; cat gpurun_out/r06e_lab_pipe.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 400 python -u -m pytest tests/test_knn_gpu.py tests/test_knn_adversarial_gpu.py tests/test_knn_generic_gpu.py -x -q $T > gpurun_out/r06e_pytest_knn.log 2>&1 || { tail -40 gpurun_out/r06e_pytest_knn.log; exit 1; }
tail -2 gpurun_out/r06e_pytest_knn.log
timeout -k 10 120 python -u tools/knn_bench.py 20 > gpurun_out/r06e_knn_bench.log 2>&1 && cat gpurun_out/r06e_knn_bench.log || exit 1
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r06e_bench.log 2>&1 || { tail -30 gpurun_out/r06e_bench.log; exit 1; }
tail -c 1500 gpurun_out/r06e_bench.log
