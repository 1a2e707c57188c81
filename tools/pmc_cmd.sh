#!/bin/bash
# PMC passes over an arbitrary command (each pass its own rocprofv3 run, as
# MI355X_MICROARCH.md prescribes): tools/pmc_cmd.sh <outdir> <cmd...>
# Writes <outdir>/p<i>/ and prints per-kernel averages via tools/pmc_avg.py.
set -o pipefail
OUT=$1; shift
mkdir -p "$OUT"
export TMPDIR=/tmp
i=0
for pass in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" \
            "SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES" \
            "FETCH_SIZE" "TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum"; do
    i=$((i + 1))
    # shellcheck disable=SC2086
    (cd /tmp && timeout -s KILL 120 rocprofv3 --pmc $pass --output-format csv -d "$OUT/p$i" -o run -- "$@") \
        > "$OUT/p$i.log" 2>&1 || { echo "pmc pass $i failed"; tail -5 "$OUT/p$i.log"; exit 1; }
done
python3 "$(dirname "$0")/pmc_avg.py" "$OUT"
