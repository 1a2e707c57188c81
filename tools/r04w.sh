#!/bin/bash
# bf16-filtered kNN (knn_bf_kernel, C = 64/128): kNN parity tests, then standalone timings
set -o pipefail
export PYTHONDONTWRITEBYTECODE=1
timeout -k 10 600 python -u -m pytest tests/test_knn_gpu.py tests/test_knn_adversarial_gpu.py tests/test_knn_generic_gpu.py tests/test_graph_feature_gpu.py -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/r04w_pytest.log 2>&1; rc=$?
tail -40 gpurun_out/r04w_pytest.log
[ $rc -eq 0 ] || exit $rc
DGX_LIB=$(realpath tools/diag/libdgx_bfdiag.so) timeout -k 10 120 python -u tools/knn_bf_diag.py
timeout -k 10 120 python -u tools/knn_bench.py 50
KNN_BENCH_BIG=1 timeout -k 10 120 python -u tools/knn_bench.py 20
