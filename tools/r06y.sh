#!/bin/bash
# round 5, session x: four-wave PositionEmbedding backward kernel: parity tests, posemb leg A/B, kernel trace
set -o pipefail
export PYTHONDONTWRITEBYTECODE=1
mkdir -p gpurun_out
T="--timeout 300 --timeout-method thread"
timeout -k 10 600 python -u -m pytest tests/test_edgemlp_fused_bwd_gpu.py tests/test_edgemlp_gpu.py -q $T > gpurun_out/r06y_tests.log 2>&1; rc=$?
tail -5 gpurun_out/r06y_tests.log
[ $rc -eq 0 ] || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_r06y_pe -o run -- python3 $GRAFT_REPO_ROOT/tools/posemb_once.py 1 5 > $GRAFT_REPO_ROOT/gpurun_out/r06y_prof.log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/gpurun_out/r06y_prof.log; exit 1; }
KS=$(find $GRAFT_REPO_ROOT/gpurun_out/prof_r06y_pe -name run_kernel_stats.csv -print -quit)
python3 $GRAFT_REPO_ROOT/tools/kt_summary.py "$(dirname "$KS")" > $GRAFT_REPO_ROOT/gpurun_out/prof_r06y_pe/kt_summary.txt && head -14 $GRAFT_REPO_ROOT/gpurun_out/prof_r06y_pe/kt_summary.txt
