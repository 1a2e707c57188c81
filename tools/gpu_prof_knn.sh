#!/bin/bash
# Kernel-trace stats of the standalone kNN driver.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/kprof
export PYTHONDONTWRITEBYTECODE=1
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/kprof -o knn --output-format csv -- \
    python3 tools/knn_bench.py 20 > gpurun_out/kprof/run.log 2>&1 || exit $?
cat gpurun_out/kprof/run.log | grep us/call
python3 tools/prof_summary.py gpurun_out/kprof/knn_kernel_stats.csv
