#!/bin/bash
# Kernel-trace stats of tools/edge_bench.py for the product lib and experiment builds.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/exp
export PYTHONDONTWRITEBYTECODE=1
for v in ${VARIANTS:-0 1 2}; do
  lib=$PWD/dgcnn.pytorch_amd/dgx/libdgx.so
  [ $v -ne 0 ] && lib=$PWD/tools/exp/libdgx_exp$v.so
  DGX_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/exp/v$v -o r --output-format csv -- \
      python3 tools/edge_bench.py 3 > gpurun_out/exp/v$v.log 2>&1 || { tail -5 gpurun_out/exp/v$v.log; exit 1; }
  echo "== variant $v"
  python3 tools/trace_grid.py gpurun_out/exp/v$v/r_kernel_trace.csv edge_
done
