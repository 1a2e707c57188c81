#!/bin/bash
# Profile bench.py on the GPU box: one rocprofv3 kernel-trace pass (per-kernel
# durations) and separate PMC passes (HBM bytes, VALU / MFMA / LDS counters),
# each its own run as MI355X_MICROARCH.md's rocprofv3 section prescribes.
# usage: [KT_ONLY=1] tools/profile.sh <tag> [bench args...]     (writes gpurun_out/prof_<tag>/)
set -o pipefail
TAG=$1; shift
REPO=$(pwd)
OUT=$REPO/gpurun_out/prof_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
BENCH=(python3 "$REPO/bench.py" --no-graph --no-cpu-baseline --no-eager-baseline --no-posemb-leg --no-edgeconv-leg --no-attention-leg
       --no-fp32-leg "$@")
cd /tmp || exit 1
echo "== kernel trace: ${BENCH[*]}"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/kt" -o run -- "${BENCH[@]}" \
    > "$OUT/kt.log" 2>&1 || { echo "kernel trace failed"; tail -20 "$OUT/kt.log"; exit 1; }
tail -1 "$OUT/kt.log"
KS=$(find "$OUT/kt" -name run_kernel_stats.csv -print -quit)
python3 "$REPO/tools/kt_summary.py" "$(dirname "$KS")" > "$OUT/kt_summary.txt" && head -40 "$OUT/kt_summary.txt"
if [ -n "$KT_ONLY" ]; then echo "profile done (kernel trace only)"; exit 0; fi
i=0
for pass in "FETCH_SIZE" "WRITE_SIZE" \
            "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE" \
            "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY" \
            "SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR"; do
    i=$((i + 1))
    echo "== pmc pass $i: $pass"
    # shellcheck disable=SC2086
    timeout -s KILL 180 rocprofv3 --pmc $pass --output-format csv -d "$OUT/p$i" -o run -- "${BENCH[@]}" \
        > "$OUT/p$i.log" 2>&1 || { echo "pmc pass $i failed"; tail -5 "$OUT/p$i.log"; exit 1; }
done
echo "profile done"
