#!/bin/bash
# kNN-only GPU session: parity tests, per-layer kernel timing, flag rates.
# Stops at the first step that crashes or times out.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1
timeout -k 10 300 python -u -m pytest tests/test_knn_gpu.py tests/test_graph_reverse_gpu.py -q -x --timeout 120 \
    --timeout-method thread > gpurun_out/knn_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/knn_tests.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 120 python tools/knn_bench.py 20 || exit $?
DGX_KNN_NOFIX=1 timeout -k 10 120 python tools/knn_flags.py
