#!/bin/bash
# PMC passes over a short bench run (every kernel of the step), each counter
# group in its own rocprofv3 run with kernel-trace only. Table:
#   python tools/pmc_table.py gpurun_out/pmcb <kernel-name-filter>
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/pmcb
mkdir -p $OUT
export PYTHONDONTWRITEBYTECODE=1
CMD="python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-eager-baseline --no-fp32-leg --no-edgeconv-leg --no-posemb-leg"
pass() {
    local name=$1; shift
    timeout -s KILL 180 rocprofv3 --pmc "$@" --kernel-trace -d $OUT/$name -o $name --output-format csv -- $CMD \
        > $OUT/$name.log 2>&1
    local rc=$?
    echo "pass $name rc=$rc"
    return $rc
}
pass p1 SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY && \
pass p2 FETCH_SIZE && \
pass p3 WRITE_SIZE && \
pass p4 SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS
echo "=== done"
