#!/bin/bash
# round 5, session l: kNN v3 (NaN bounds, rolled fold/compact loops): lab, kNN tests, knn_bench, full bench + kernel trace
set -o pipefail
export PYTHONDONTWRITEBYTECODE=1
mkdir -p gpurun_out
T="--timeout 300 --timeout-method thread"
timeout -k 10 120 ./tools/knn_lab 20 > gpurun_out/r06m_lab.log 2>&1; rc=$?; cat gpurun_out/r06m_lab.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 400 python -u -m pytest tests/test_knn_gpu.py tests/test_knn_adversarial_gpu.py tests/test_knn_generic_gpu.py -q $T > gpurun_out/r06m_pytest_knn.log 2>&1; tail -5 gpurun_out/r06m_pytest_knn.log
timeout -k 10 120 python -u tools/knn_bench.py 20 > gpurun_out/r06m_knn_bench.log 2>&1 && cat gpurun_out/r06m_knn_bench.log || exit 1




