#!/bin/bash
set -o pipefail
export PYTHONDONTWRITEBYTECODE=1
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/knn_debug.py > gpurun_out/r06k_debug.log 2>&1; rc=$?; cat gpurun_out/r06k_debug.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 120 ./tools/knn_lab 20 > gpurun_out/r06k_lab.log 2>&1; rc=$?; cat gpurun_out/r06k_lab.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 120 ./tools/knn_lab 3 check > gpurun_out/r06k_lab_check.log 2>&1; rc=$?; cat gpurun_out/r06k_lab_check.log; [ $rc -eq 0 ] || exit 1
