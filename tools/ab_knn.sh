#!/bin/bash
# A/B of libdgx variants in abl/ on the kNN micro-benchmark (tools/knn_bench.py),
# interleaved twice; then the bit-exact kNN tests on the LAST variant named.
# usage: tools/ab_knn.sh <variant>...   (abl/libdgx_<variant>.so)
set -o pipefail
for pass in 1 2; do
  for v in "$@"; do
    echo "== $v (pass $pass)"
    DGX_LIB=$PWD/abl/libdgx_$v.so timeout -k 10 120 python3 tools/knn_bench.py 20 2>&1 | grep -v amdgpu.ids || exit 1
  done
done
last=${@: -1}
DGX_LIB=$PWD/abl/libdgx_$last.so timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_knn_gpu.py 2>&1 | tail -3
