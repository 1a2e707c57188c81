#!/bin/bash
# PMC passes over an arbitrary python command (one rocprofv3 run per pass):
# usage: tools/pmc_kernels.sh <tag> <python args...>   -> gpurun_out/pmck_<tag>/
set -o pipefail
TAG=$1; shift
REPO=$(pwd)
OUT=$REPO/gpurun_out/pmck_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp || exit 1
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/kt" -o run -- python3 "$@" \
    > "$OUT/kt.log" 2>&1 || { echo "kernel trace failed"; tail -5 "$OUT/kt.log"; exit 1; }
i=0
for pass in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE" \
            "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE" \
            "FETCH_SIZE" "WRITE_SIZE"; do
    i=$((i + 1))
    # shellcheck disable=SC2086
    timeout -s KILL 120 rocprofv3 --pmc $pass --output-format csv -d "$OUT/p$i" -o run -- python3 "$@" \
        > "$OUT/p$i.log" 2>&1 || { echo "pmc pass $i failed"; tail -5 "$OUT/p$i.log"; exit 1; }
done
echo "pmc done"
