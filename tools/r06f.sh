#!/bin/bash
# round 5, session f: kNN lab (phases, in-stream flush share), stream-only variant, PMC passes over the lab
set -o pipefail
mkdir -p gpurun_out
R=$(pwd)
timeout -k 10 120 ./tools/knn_lab 20 > gpurun_out/r06f_lab.log 2>&1; rc=$?; cat gpurun_out/r06f_lab.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 120 ./tools/knn_lab_nosel 20 > gpurun_out/r06f_lab_nosel.log 2>&1; rc=$?; cat gpurun_out/r06f_lab_nosel.log; [ $rc -eq 0 ] || exit 1
cd /tmp && export TMPDIR=/tmp
i=0
for pass in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES" \
            "SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE" \
            "SQ_VALU_MFMA_COEXEC_CYCLES SQ_ACTIVE_INST_LDS SQ_INSTS_BRANCH GRBM_GUI_ACTIVE"; do
    i=$((i + 1))
    timeout -s KILL 60 rocprofv3 --pmc $pass --output-format csv -d $R/gpurun_out/r06f_p$i -o run -- $R/tools/knn_lab 3 > $R/gpurun_out/r06f_p$i.log 2>&1 || { echo "pmc pass $i failed"; tail -5 $R/gpurun_out/r06f_p$i.log; exit 1; }
done
echo done
