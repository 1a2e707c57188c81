#!/bin/bash
# round 5, session z: pull scatter with LDS row starts + prefetched id batches (tests, bench, trace);
# PMC of the four-wave and the pair PositionEmbedding backward kernels
set -o pipefail
export PYTHONDONTWRITEBYTECODE=1
mkdir -p gpurun_out
T="--timeout 300 --timeout-method thread"
timeout -k 10 600 python -u -m pytest tests/test_fused_finalize_gpu.py tests/test_scatter_push_gpu.py tests/test_edgeconv_gpu.py tests/test_graph_reverse_gpu.py -q $T > gpurun_out/r06z_tests.log 2>&1; rc=$?
tail -3 gpurun_out/r06z_tests.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -u bench.py --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/r06z_bench.log 2>&1 || { tail -30 gpurun_out/r06z_bench.log; exit 1; }
grep -o '"ms_per_step": [0-9.]*' gpurun_out/r06z_bench.log | head -2
KT_ONLY=1 timeout -k 10 400 bash tools/profile.sh r06z_cfg2 --steps 10 --warmup 3 > gpurun_out/r06z_prof_cfg2.log 2>&1 || { tail -20 gpurun_out/r06z_prof_cfg2.log; exit 1; }
grep -E "scatter|knn_kernel<16" gpurun_out/prof_r06z_cfg2/kt_summary.txt | head -3
timeout -k 10 600 bash tools/pmc_kernels.sh r06z_emb4 tools/posemb_once.py 1 3 > gpurun_out/r06z_pmc4.log 2>&1 || { tail -10 gpurun_out/r06z_pmc4.log; exit 1; }
DGX_EMLP_BWD_PAIR=1 timeout -k 10 600 bash tools/pmc_kernels.sh r06z_emb2 tools/posemb_once.py 1 3 > gpurun_out/r06z_pmc2.log 2>&1 || { tail -10 gpurun_out/r06z_pmc2.log; exit 1; }
echo done
