#!/bin/bash
# A/B of the EdgeConv backward scatter kernels (wide vs narrow) inside the bench step.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1
timeout -k 10 300 python -u -m pytest tests/test_edgeconv_gpu.py -q -x --timeout 120 --timeout-method thread > gpurun_out/ab_tests.log 2>&1; echo "tests rc=$?"; tail -1 gpurun_out/ab_tests.log
B="python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-eager-baseline --no-fp32-leg --no-edgeconv-leg --no-posemb-leg"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/abw -o w --output-format csv -- $B > gpurun_out/abw.log 2>&1 && \
DGX_EDGE_BWD_NARROW=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/abn -o n --output-format csv -- $B > gpurun_out/abn.log 2>&1
echo "prof rc=$?"
tail -1 gpurun_out/abw.log | cut -c1-200; tail -1 gpurun_out/abn.log | cut -c1-200
