#!/bin/bash
# generic-shape kNN tests, then the pending reverse-graph / small-K GEMM variant timings (r04r)
set -o pipefail
export PYTHONDONTWRITEBYTECODE=1
timeout -k 10 600 python -u -m pytest tests/test_edge_mode_gpu.py tests/test_knn_generic_gpu.py tests/test_knn_gpu.py tests/test_graph_feature_gpu.py -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/r04s_pytest.log 2>&1 || { tail -30 gpurun_out/r04s_pytest.log; exit 1; }
tail -2 gpurun_out/r04s_pytest.log
bash tools/r04r.sh
