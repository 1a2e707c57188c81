#!/bin/bash
# One GPU-box session: parity tests, bench, rocprof kernel trace.
# Each GPU step has its own time limit; a crash/timeout (anything but a plain
# test failure) stops the script so nothing else touches a bad GPU.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1
step() {  # step <name> <timeout> <cmd...>
    local name=$1 t=$2; shift 2
    echo "=== $name ($(date +%T))"
    timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "=== $name rc=$rc"
    tail -5 "gpurun_out/$name.log"
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "ABORT after $name (rc=$rc)"; exit $rc; fi
    return 0
}
MODE=${1:-all}
if [ "$MODE" = all ] || [ "$MODE" = test ]; then
    step pytest_gpu 900 python -u -m pytest tests -m gpu -q -rf --timeout 120 --timeout-method thread
fi
if [ "$MODE" = all ] || [ "$MODE" = bench ]; then
    step bench 900 python bench.py --steps 20 --warmup 5
fi
if [ "$MODE" = all ] || [ "$MODE" = prof ]; then
    step rocprof 900 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- \
        python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-eager-baseline --no-fp32-leg --no-edgeconv-leg --no-posemb-leg
fi
echo "=== done"
