#!/bin/bash
# Backward on two streams (reverse graphs + weight gradients beside the
# input-gradient chain): the C++-op / graph-replay GPU tests, then an
# interleaved A/B of the cfg2 step with DGX_BWD_STREAMS=0 / 1.
set -o pipefail
export PYTHONDONTWRITEBYTECODE=1
timeout -k 10 600 python -u -m pytest tests/test_host_ext_gpu.py -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/r04n_pytest.log 2>&1 || { tail -20 gpurun_out/r04n_pytest.log; exit 1; }
tail -2 gpurun_out/r04n_pytest.log
for r in 1 2 3; do
  for v in 0 1 2 4; do
    ms=$(DGX_BWD_STREAMS=$v timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-eager-baseline --no-posemb-leg \
         --no-edgeconv-leg --no-attention-leg --no-fp32-leg --no-roofline-leg --steps 50 --warmup 10 2>/dev/null \
         | python3 -c 'import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d["ms_per_step"], d["eager_launch_ms_per_step"])') \
       || { echo "run failed (streams=$v)"; exit 1; }
    echo "round $r streams=$v: $ms (graph, eager ms/step)"
  done
done
