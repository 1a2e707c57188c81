#!/bin/bash
# round 5, session j: kNN v3 structural checks on small ragged shapes (repeated), then the kNN tests
set -o pipefail
export PYTHONDONTWRITEBYTECODE=1
mkdir -p gpurun_out
T="--timeout 300 --timeout-method thread"
timeout -k 10 120 ./tools/knn_lab 3 check > gpurun_out/r06j_lab_check.log 2>&1; rc=$?; cat gpurun_out/r06j_lab_check.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 400 python -u -m pytest tests/test_knn_gpu.py tests/test_knn_adversarial_gpu.py tests/test_knn_generic_gpu.py -q $T > gpurun_out/r06j_pytest_knn.log 2>&1; tail -15 gpurun_out/r06j_pytest_knn.log
