#!/bin/bash
# full GPU suite + bench + kernel trace (r04y), then A/B of one 128-point tile per conv5 BN-stats block (RS_LT 1)
set -o pipefail
bash tools/gpu_suite.sh r04y || exit 1
timeout -k 10 400 bash tools/ab_lib.sh dgcnn.pytorch_amd/dgx/libdgx.so tools/diag/libdgx_rs1.so 3 > gpurun_out/r04z_ab.log 2>&1 || { cat gpurun_out/r04z_ab.log; exit 1; }
cat gpurun_out/r04z_ab.log
