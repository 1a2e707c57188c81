#!/bin/bash
# PMC passes for the kNN selection kernel, each counter group in its own
# rocprofv3 run (kernel-trace only, no other trace domains), plus the counter list.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/pmck
mkdir -p $OUT
export PYTHONDONTWRITEBYTECODE=1
timeout -k 10 120 rocprofv3 -L > $OUT/counters.txt 2>&1 || true
pass() {  # pass <name> <counters...>
    local name=$1; shift
    timeout -s KILL 120 rocprofv3 --pmc "$@" --kernel-trace -d $OUT/$name -o $name --output-format csv -- \
        python3 tools/knn_bench.py 2 > $OUT/$name.log 2>&1
    local rc=$?
    echo "pass $name rc=$rc"
    return $rc
}
pass p1 SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY && \
pass p2 FETCH_SIZE && \
pass p3 WRITE_SIZE && \
pass p4 SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_WAIT_INST_LDS
echo "=== done"
