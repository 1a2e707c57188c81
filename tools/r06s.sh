#!/bin/bash
# round 5, session s: cfg4 routed fp32 test twice (determinism of the gradient errors), then the whole GPU suite
set -o pipefail
export PYTHONDONTWRITEBYTECODE=1
mkdir -p gpurun_out
T="--timeout 300 --timeout-method thread"
for r in 1 2; do
  timeout -k 10 300 python -u -m pytest tests/test_partseg.py -q -s -k "cfg4_routed and False" $T > gpurun_out/r06s_cfg4_$r.log 2>&1; rc=$?
  grep -E "Net cfg4|passed|failed" gpurun_out/r06s_cfg4_$r.log | cut -c1-600
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 1
done
timeout -k 10 900 python -u -m pytest tests -m gpu -q $T > gpurun_out/r06s_pytest_gpu.log 2>&1; rc=$?
tail -8 gpurun_out/r06s_pytest_gpu.log
exit $rc
