#!/bin/bash
# conv5 GEMMs: 256x256 tiles vs the 128x128 LDS kernel, forward (stats16 epilogue) and input gradient (store)
set -o pipefail
timeout -k 10 600 bash tools/ab_lib.sh tools/diag/libdgx_g3nofwd.so dgcnn.pytorch_amd/dgx/libdgx.so 2 > gpurun_out/r05d_ab1.log 2>&1 || { cat gpurun_out/r05d_ab1.log; exit 1; }
cat gpurun_out/r05d_ab1.log
timeout -k 10 600 bash tools/ab_lib.sh tools/diag/libdgx_g3nostore.so dgcnn.pytorch_amd/dgx/libdgx.so 2 > gpurun_out/r05d_ab2.log 2>&1 || { cat gpurun_out/r05d_ab2.log; exit 1; }
cat gpurun_out/r05d_ab2.log

DGX_LIB=$(realpath tools/diag/libdgx_g3r2.so) timeout -k 10 300 python -u -m pytest tests/test_gemm_gpu.py -m gpu -q -x --timeout 200 --timeout-method thread > gpurun_out/r05d_pytest_r2.log 2>&1 || { tail -20 gpurun_out/r05d_pytest_r2.log; exit 1; }
tail -1 gpurun_out/r05d_pytest_r2.log
timeout -k 10 600 bash tools/ab_lib.sh tools/diag/libdgx_g3r2.so dgcnn.pytorch_amd/dgx/libdgx.so 3 > gpurun_out/r05d_ab3.log 2>&1 || { cat gpurun_out/r05d_ab3.log; exit 1; }
cat gpurun_out/r05d_ab3.log
