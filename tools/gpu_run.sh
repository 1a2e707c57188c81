#!/bin/bash
# Run GPU steps in order, each "LOG::COMMAND" under `timeout -k 10 SECS`; stop
# at the first step that faults, aborts, hangs or times out (rc >= 2 other than
# pytest's test-failure rc 1). Logs under gpurun_out/.
#   usage: bash tools/gpu_run.sh SECS "log1::cmd1" ["log2::cmd2" ...]
SECS=${1:?secs}
shift
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$ROOT/gpurun_out"
cd "$ROOT" || exit 1
export PYTHONDONTWRITEBYTECODE=1
for step in "$@"; do
    log=${step%%::*}
    cmd=${step#*::}
    echo "== $log: $cmd"
    timeout -k 10 "$SECS" bash -c "$cmd" > "gpurun_out/$log" 2>&1
    rc=$?
    tail -4 "gpurun_out/$log"
    echo "== $log rc=$rc"
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after rc=$rc"; exit $rc; fi
done
