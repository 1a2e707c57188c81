#!/bin/bash
# kNN time decomposition: probe builds (1 = half Gram chain, 2 = no selection, 3 = both) on tools/knn_bench.py
set -o pipefail
export PYTHONDONTWRITEBYTECODE=1
for lib in dgcnn.pytorch_amd/dgx/libdgx.so tools/diag/libdgx_p1.so tools/diag/libdgx_p2.so tools/diag/libdgx_p3.so; do
  echo "== $(basename $lib)"
  DGX_LIB=$(realpath $lib) timeout -k 10 120 python -u tools/knn_bench.py 50 || exit 1
done
