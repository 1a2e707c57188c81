cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_knn_gpu.py tests/test_graph_reverse_gpu.py -q -x --timeout 120 --timeout-method thread > gpurun_out/knn_tests.log 2>&1; echo "tests rc=$?"; tail -2 gpurun_out/knn_tests.log
timeout -k 10 120 python tools/knn_bench.py 20
DGX_KNN_NOFIX=1 timeout -k 10 120 python tools/knn_flags.py
