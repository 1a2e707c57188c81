#!/bin/bash
# PMC passes for the kNN kernel (counters in their own runs, kernel-trace only).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/pmc
export PYTHONDONTWRITEBYTECODE=1
timeout -k 10 300 python tools/knn_bench.py 20 > gpurun_out/pmc/knn_bench.log 2>&1 || exit $?
timeout -k 10 600 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
    --kernel-trace -d gpurun_out/pmc/sq -o sq --output-format csv -- python3 tools/knn_bench.py 2 > gpurun_out/pmc/sq.log 2>&1 || exit $?
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/pmc/fetch -o fetch --output-format csv -- \
    python3 tools/knn_bench.py 2 > gpurun_out/pmc/fetch.log 2>&1 || exit $?
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d gpurun_out/pmc/write -o write --output-format csv -- \
    python3 tools/knn_bench.py 2 > gpurun_out/pmc/write.log 2>&1 || exit $?
cat gpurun_out/pmc/knn_bench.log
ls -R gpurun_out/pmc | head -30
