#!/bin/bash
# Interleaved A/B of two builds of the library pair (libdgx.so + libdgx_torch.so)
# on the cfg2 bench step: tools/ab_host.sh <libdgx A> <libdgx_torch A> <libdgx B> <libdgx_torch B> [rounds] [bench args]
set -o pipefail
LA=$1; TA=$2; LB=$3; TB=$4; R=${5:-3}; shift 5
for r in $(seq 1 "$R"); do
    for v in A B; do
        if [ $v = A ]; then L=$LA; T=$TA; else L=$LB; T=$TB; fi
        ms=$(DGX_LIB=$(realpath "$L") DGX_TORCH_LIB=$(realpath "$T") timeout -k 10 200 python3 bench.py --no-cpu-baseline \
             --no-eager-baseline --no-posemb-leg --no-edgeconv-leg --no-attention-leg --no-fp32-leg --no-roofline-leg \
             --steps 50 --warmup 10 "$@" 2>/dev/null \
             | python3 -c 'import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d["ms_per_step"], d["eager_launch_ms_per_step"])') \
            || { echo "run failed ($v)"; exit 1; }
        echo "round $r $v: $ms (graph, eager ms/step)"
    done
done
