#!/bin/bash
# Phase ablation of the EdgeConv gather/scatter kernels: kernel times with
# tools/libdgx_exp1.so (neighbour loops skipped) and libdgx_exp2.so (LDS staging
# skipped). Results are numerically meaningless; only the timings are read.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
B="python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-eager-baseline --no-fp32-leg --no-edgeconv-leg --no-posemb-leg"
for e in 1 2; do
    DGX_LIB=$PWD/tools/libdgx_exp$e.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/exp$e -o e \
        --output-format csv -- $B > gpurun_out/exp$e.log 2>&1 || exit $?
    echo "--- exp$e"; python3 tools/prof_summary.py gpurun_out/exp$e/e_kernel_stats.csv 12 | grep -E "edge_|total"
done
