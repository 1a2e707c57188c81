#!/bin/bash
# A/B of the kNN kernel: current library vs tools/libdgx_old.so (kernel timing only).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1
echo "--- new"; timeout -k 10 120 python tools/knn_bench.py 20 || exit $?

cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/kab -o new --output-format csv -- python3 tools/knn_bench.py 10 > gpurun_out/kab_new.log 2>&1 || exit $?
python3 tools/prof_summary.py gpurun_out/kab/new_kernel_stats.csv 1 2>/dev/null | head -8
