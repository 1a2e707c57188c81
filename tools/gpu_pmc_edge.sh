#!/bin/bash
# PMC passes over the EdgeConv chain kernels (counters in their own runs, kernel-trace only).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/pmce
export PYTHONDONTWRITEBYTECODE=1
rocprofv3 --list-avail > gpurun_out/pmce/avail.txt 2>&1 || true
i=0
for set in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VMEM" \
           "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $set --kernel-trace -d gpurun_out/pmce/p$i -o p --output-format csv -- \
      python3 tools/edge_bench.py 2 > gpurun_out/pmce/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 gpurun_out/pmce/p$i.log; exit 1; }
done
echo ok
