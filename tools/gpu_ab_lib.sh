#!/bin/bash
# A/B of two builds of libdgx.so on one box (step times vary box to box):
# tools/gpu_ab_lib.sh <baseline.so> [reps]; the candidate is the in-tree build.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
BASE=$1; REPS=${2:-3}
B="python bench.py --steps 40 --warmup 10 --no-cpu-baseline --no-eager-baseline --no-fp32-leg --no-edgeconv-leg --no-posemb-leg"
ms() { timeout -k 10 200 $B 2>/dev/null | python -c "import json,sys; print(json.loads(sys.stdin.read())['ms_per_step'])"; }
for i in $(seq "$REPS"); do
    a=$(DGX_LIB=$BASE ms) || exit 1
    b=$(ms) || exit 1
    echo "base $a  new $b"
done
