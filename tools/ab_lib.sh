#!/bin/bash
# Interleaved A/B of two builds of libdgx.so on the cfg2 bench step (HIP-graph
# replay): tools/ab_lib.sh <lib A> <lib B> [rounds] [bench args...]
# Prints each run's ms_per_step; the per-kernel view comes from rocprofv3.
set -o pipefail
A=$1; B=$2; R=${3:-3}; shift 3
for r in $(seq 1 "$R"); do
    for L in "$A" "$B"; do
        ms=$(DGX_LIB=$(realpath "$L") timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-eager-baseline \
             --no-posemb-leg --no-edgeconv-leg --no-attention-leg --no-fp32-leg --steps 50 --warmup 10 "$@" 2>/dev/null \
             | python3 -c 'import json,sys; print(json.loads(sys.stdin.read().strip().splitlines()[-1])["ms_per_step"])') \
            || { echo "run failed ($L)"; exit 1; }
        echo "round $r $(basename "$L"): $ms ms/step"
    done
done
