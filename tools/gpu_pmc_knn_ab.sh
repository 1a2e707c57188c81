#!/bin/bash
# PMC passes over tools/knn_bench.py for the current library and tools/libdgx_old.so.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1
pass() {  # pass <outdir> <name> <counters...>
    local out=$1 name=$2; shift 2
    timeout -s KILL 90 rocprofv3 --pmc "$@" --kernel-trace -d $out/$name -o $name --output-format csv -- \
        python3 tools/knn_bench.py 2 > $out/$name.log 2>&1
    local rc=$?; echo "pass $out/$name rc=$rc"; return $rc
}
P1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY"
P2="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VALU"
mkdir -p gpurun_out/pmck_new gpurun_out/pmck_old
pass gpurun_out/pmck_new p1 $P1 && pass gpurun_out/pmck_new p2 $P2

echo "=== done"
