#!/bin/bash
# one slab-sum launch per backward in the C++ op: equality tests, A/B vs the previous build, kernel trace
set -o pipefail
export PYTHONDONTWRITEBYTECODE=1
timeout -k 10 600 python -u -m pytest tests/test_host_ext_gpu.py -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/r04q_pytest.log 2>&1 || { tail -20 gpurun_out/r04q_pytest.log; exit 1; }
tail -2 gpurun_out/r04q_pytest.log
timeout -k 10 600 bash tools/ab_host.sh dgcnn.pytorch_amd/dgx/libdgx.so tools/diag/libdgx_torch_head.so dgcnn.pytorch_amd/dgx/libdgx.so dgcnn.pytorch_amd/dgx/libdgx_torch.so 3 > gpurun_out/r04q_ab.log 2>&1 || { cat gpurun_out/r04q_ab.log; exit 1; }
cat gpurun_out/r04q_ab.log
