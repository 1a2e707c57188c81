#!/bin/bash
# round 5, session h: kNN selection by value-only threshold lists + candidate logs ranked by counting
set -o pipefail
export PYTHONDONTWRITEBYTECODE=1
mkdir -p gpurun_out
T="--timeout 300 --timeout-method thread"
for v in n24 n32 nosel; do
  timeout -k 10 120 ./tools/knn_lab_$v 20 > gpurun_out/r06h_lab_$v.log 2>&1; rc=$?; echo "== $v"; cat gpurun_out/r06h_lab_$v.log; [ $rc -eq 0 ] || exit 1
done
timeout -k 10 400 python -u -m pytest tests/test_knn_gpu.py tests/test_knn_adversarial_gpu.py tests/test_knn_generic_gpu.py -x -q $T > gpurun_out/r06h_pytest_knn.log 2>&1 || { tail -40 gpurun_out/r06h_pytest_knn.log; exit 1; }
tail -2 gpurun_out/r06h_pytest_knn.log
timeout -k 10 120 python -u tools/knn_bench.py 20 > gpurun_out/r06h_knn_bench.log 2>&1 && cat gpurun_out/r06h_knn_bench.log || exit 1
