#!/bin/bash
# conv5 BN-backward stats pass, pipelined: GPU tests of the path, then A/B of the
# step against the previous build (tools/diag/libdgx_head.so) and the RS_LT=4 build.
set -o pipefail
export PYTHONDONTWRITEBYTECODE=1
timeout -k 10 600 python -u -m pytest tests/test_model_gpu.py tests/test_host_ext_gpu.py -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/r04l_pytest.log 2>&1 || { tail -20 gpurun_out/r04l_pytest.log; exit 1; }
tail -2 gpurun_out/r04l_pytest.log
timeout -k 10 400 bash tools/ab_lib.sh tools/diag/libdgx_head.so dgcnn.pytorch_amd/dgx/libdgx.so 3 > gpurun_out/r04l_ab.log 2>&1 || { cat gpurun_out/r04l_ab.log; exit 1; }
cat gpurun_out/r04l_ab.log
timeout -k 10 400 bash tools/ab_lib.sh tools/diag/libdgx_rs4.so dgcnn.pytorch_amd/dgx/libdgx.so 2 > gpurun_out/r04l_ab2.log 2>&1 || { cat gpurun_out/r04l_ab2.log; exit 1; }
cat gpurun_out/r04l_ab2.log
KT_ONLY=1 timeout -k 10 300 bash tools/profile.sh r04l --steps 5 --warmup 2 > gpurun_out/r04l_prof.log 2>&1 || { tail gpurun_out/r04l_prof.log; exit 1; }
grep -E "bwd16|apply16" gpurun_out/prof_r04l/kt_summary.txt
