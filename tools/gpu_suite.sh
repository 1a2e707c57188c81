#!/bin/bash
# One GPU-box pass: the -m gpu suite, the default bench line, and a rocprofv3
# kernel trace of a short cfg2 bench, every step under its own time limit and
# chained so that the first failure ends the call. Outputs: gpurun_out/<tag>_*.
#   usage: bash tools/gpu_suite.sh TAG [pytest-args...]
set -o pipefail
TAG=${1:?tag}
shift
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
cd "$ROOT" || exit 1
export PYTHONDONTWRITEBYTECODE=1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread "$@" \
    > "$OUT/${TAG}_pytest_gpu.log" 2>&1 || { echo "pytest failed rc=$?"; tail -30 "$OUT/${TAG}_pytest_gpu.log"; exit 1; }
tail -2 "$OUT/${TAG}_pytest_gpu.log"
timeout -k 10 300 python -u bench.py > "$OUT/${TAG}_bench.log" 2>&1 || { echo "bench failed rc=$?"; tail -20 "$OUT/${TAG}_bench.log"; exit 1; }
tail -c 400 "$OUT/${TAG}_bench.log"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/${TAG}_prof" -o run -- python3 "$ROOT/bench.py" --steps 10 \
    --warmup 3 --no-cpu-baseline --no-eager-baseline --no-fp32-leg --no-edgeconv-leg --no-posemb-leg \
    --no-attention-leg --no-roofline-leg > "$OUT/${TAG}_prof.log" 2>&1 || { echo "rocprof failed rc=$?"; tail -20 "$OUT/${TAG}_prof.log"; exit 1; }
KS=$(find "$OUT/${TAG}_prof" -name run_kernel_stats.csv -print -quit)
python3 "$ROOT/tools/kt_summary.py" "$(dirname "$KS")" 13 > "$OUT/${TAG}_kernel_stats.txt" && head -12 "$OUT/${TAG}_kernel_stats.txt"
echo done
