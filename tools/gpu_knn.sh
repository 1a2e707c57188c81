#!/bin/bash
# kNN iteration: old vs new kernel timing, GPU parity tests, optional PMC passes.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/knn
export PYTHONDONTWRITEBYTECODE=1
timeout -k 10 600 python -m pytest tests/test_knn_gpu.py -x -q > gpurun_out/knn/pytest_knn.log 2>&1
rc=$?
tail -5 gpurun_out/knn/pytest_knn.log
[ $rc -eq 0 ] || exit $rc
if [ -f tools/libdgx_old.so ]; then
  DGX_LIB=$PWD/tools/libdgx_old.so timeout -k 10 300 python tools/knn_bench.py 20 > gpurun_out/knn/old.log 2>&1 || exit $?
fi
timeout -k 10 300 python tools/knn_bench.py 20 > gpurun_out/knn/new.log 2>&1 || exit $?
cat gpurun_out/knn/old.log gpurun_out/knn/new.log
timeout -k 10 900 python -m pytest tests -m gpu -q > gpurun_out/knn/pytest.log 2>&1
rc=$?
tail -5 gpurun_out/knn/pytest.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
[ "$1" = "pmc" ] && bash tools/gpu_pmc.sh
exit 0
