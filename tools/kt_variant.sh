#!/bin/bash
# Kernel-trace one command with a libdgx variant (abl/libdgx_NAME.so, "main" =
# the in-tree build) and print the per-kernel summary lines matching PATTERN.
#   usage: tools/kt_variant.sh NAME PATTERN python3 script.py [args...]
set -o pipefail
NAME=$1; PAT=$2; shift 2
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/kt_$NAME
mkdir -p "$OUT"
[ "$NAME" != main ] && export DGX_LIB=$ROOT/abl/libdgx_$NAME.so
export TMPDIR=/tmp
cd /tmp || exit 1
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT" -o run -- "$@" > "$OUT/run.log" 2>&1 \
    || { echo "trace failed"; tail -5 "$OUT/run.log"; exit 2; }
KS=$(find "$OUT" -name run_kernel_stats.csv -print -quit)
python3 "$ROOT/tools/kt_summary.py" "$(dirname "$KS")" > "$OUT/summary.txt"
echo "== $NAME"; grep -E "$PAT" "$OUT/summary.txt"
