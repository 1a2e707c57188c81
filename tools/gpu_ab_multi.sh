#!/bin/bash
# Step time of several libdgx.so builds, interleaved on one box:
# tools/gpu_ab_multi.sh <reps> <lib.so>... ("-" = the in-tree build)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
REPS=$1; shift
B="python bench.py --steps 40 --warmup 10 --no-cpu-baseline --no-eager-baseline --no-fp32-leg --no-edgeconv-leg --no-posemb-leg"
for i in $(seq "$REPS"); do
    line=""
    for lib in "$@"; do
        if [ "$lib" = "-" ]; then env=""; else env="DGX_LIB=$lib"; fi
        ms=$(env $env timeout -k 10 200 $B 2>/dev/null | python -c "import json,sys; print(json.loads(sys.stdin.read())['ms_per_step'])") || exit 1
        line="$line $(basename "$lib")=$ms"
    done
    echo "$line"
done
