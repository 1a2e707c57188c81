#!/bin/bash
# knn_bf_kernel time decomposition: probe builds (1 = no exact phase, 2 = no per-tile refresh, 4 = no selection, 3 = 1+2)
set -o pipefail
export PYTHONDONTWRITEBYTECODE=1
for lib in dgcnn.pytorch_amd/dgx/libdgx.so tools/diag/libdgx_q1.so tools/diag/libdgx_q2.so tools/diag/libdgx_q4.so tools/diag/libdgx_q3.so; do
  echo "== $(basename $lib)"
  DGX_LIB=$(realpath $lib) timeout -k 10 120 python -u tools/knn_bench.py 50 2>&1 | grep -E "^C(64|128) " || exit 1
done
