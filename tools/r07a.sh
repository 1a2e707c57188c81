#!/bin/bash
# round 5, session r07a: deterministic graph-feature backward tests; bench with the fp32-mode chain leg;
# SGD fused vs foreach A/B at cfg2 and at the 4-cloud shard
set -o pipefail
export PYTHONDONTWRITEBYTECODE=1
mkdir -p gpurun_out
T="--timeout 300 --timeout-method thread"
timeout -k 10 300 python -u -m pytest tests/test_graph_feature_gpu.py tests/test_library_ops_gpu.py -q $T > gpurun_out/r07a_tests.log 2>&1; rc=$?
tail -3 gpurun_out/r07a_tests.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 400 python -u bench.py --no-cpu-baseline --no-attention-leg --no-posemb-leg > gpurun_out/r07a_bench.log 2>&1 || { tail -30 gpurun_out/r07a_bench.log; exit 1; }
grep -o '"edgeconv_fwd_bwd_ms": {[^}]*}' gpurun_out/r07a_bench.log
for s in fused foreach fused foreach; do
  timeout -k 10 300 python -u bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-eager-baseline --no-edgeconv-leg --no-posemb-leg --no-attention-leg --no-fp32-leg --sgd $s > gpurun_out/r07a_sgd_$s.log 2>&1 || { tail -20 gpurun_out/r07a_sgd_$s.log; exit 1; }
  timeout -k 10 300 python -u bench.py --batch 4 --steps 30 --warmup 5 --no-cpu-baseline --no-eager-baseline --no-edgeconv-leg --no-posemb-leg --no-attention-leg --no-fp32-leg --sgd $s > gpurun_out/r07a_sgd_b4_$s.log 2>&1 || { tail -20 gpurun_out/r07a_sgd_b4_$s.log; exit 1; }
  echo "$s cfg2 $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r07a_sgd_$s.log | head -1) b4 $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r07a_sgd_b4_$s.log | head -1)"
done
