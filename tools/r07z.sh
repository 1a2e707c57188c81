#!/bin/bash
# round 5, session r07z: final tree sanity after the host cleanup — smoke(), host-op and fp32 suites, default bench line
set -o pipefail
export PYTHONDONTWRITEBYTECODE=1
mkdir -p gpurun_out
T="--timeout 120 --timeout-method thread"
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r07z_smoke.log 2>&1 || { tail -20 gpurun_out/r07z_smoke.log; exit 1; }
tail -1 gpurun_out/r07z_smoke.log
timeout -k 10 500 python -u -m pytest tests/test_host_ext_gpu.py tests/test_edgeconv_gpu.py tests/test_model_gpu.py tests/test_partseg.py tests/test_ddp_gpu.py -q $T > gpurun_out/r07z_tests.log 2>&1 || { tail -30 gpurun_out/r07z_tests.log; exit 1; }
tail -1 gpurun_out/r07z_tests.log
timeout -k 10 400 python -u bench.py > gpurun_out/r07z_bench.log 2>&1 || { tail -30 gpurun_out/r07z_bench.log; exit 1; }
grep -o '"ms_per_step": [0-9.]*' gpurun_out/r07z_bench.log | head -3
