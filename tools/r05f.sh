#!/bin/bash
# 3-channel kNN pre-pass with 8 tiles per operand chunk (KNN_PRE_PC) vs 4: kNN tests on the variant, selection timings, step A/B
set -o pipefail
export PYTHONDONTWRITEBYTECODE=1
DGX_LIB=$(realpath tools/diag/libdgx_pc8.so) timeout -k 10 300 python -u -m pytest tests/test_knn_gpu.py tests/test_knn_adversarial_gpu.py -m gpu -q -x --timeout 200 --timeout-method thread > gpurun_out/r05f_pytest.log 2>&1 || { tail -20 gpurun_out/r05f_pytest.log; exit 1; }
tail -1 gpurun_out/r05f_pytest.log
for lib in tools/diag/libdgx_pc8.so dgcnn.pytorch_amd/dgx/libdgx.so tools/diag/libdgx_pc8.so dgcnn.pytorch_amd/dgx/libdgx.so; do
  echo "== $(basename $lib)"; DGX_LIB=$(realpath $lib) timeout -k 10 120 python -u tools/knn_bench.py 50 2>/dev/null | grep -E "^C3" || exit 1
done
