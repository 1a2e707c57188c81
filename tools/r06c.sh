#!/bin/bash
# round 5, session b: the 32x32x2-MFMA kNN selection kernel + the unified C++ schedule:
# bench + kernel trace first, then the DDP tests and the whole -m gpu suite, smoke
set -o pipefail
export PYTHONDONTWRITEBYTECODE=1
mkdir -p gpurun_out
T="--timeout 300 --timeout-method thread"
R=$(pwd)
timeout -k 10 300 python -u -m pytest tests/test_knn_gpu.py tests/test_knn_adversarial_gpu.py -x -q $T > gpurun_out/r06c_pytest_knn.log 2>&1 || { tail -40 gpurun_out/r06c_pytest_knn.log; exit 1; }
timeout -k 10 120 python -u tools/knn_bench.py 20 > gpurun_out/r06c_knn_bench.log 2>&1 && cat gpurun_out/r06c_knn_bench.log || exit 1
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r06c_bench.log 2>&1 || { tail -30 gpurun_out/r06c_bench.log; exit 1; }
tail -c 2500 gpurun_out/r06c_bench.log
cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r06c_prof -o run -- python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-eager-baseline --no-posemb-leg --no-attention-leg --no-edgeconv-leg --no-fp32-leg > $R/gpurun_out/r06c_prof.log 2>&1 || { tail -20 $R/gpurun_out/r06c_prof.log; exit 1; }
cd $R
timeout -k 10 600 python -u -m pytest tests/test_ddp_gpu.py -x -q -s $T > gpurun_out/r06c_pytest_ddp.log 2>&1 || { tail -60 gpurun_out/r06c_pytest_ddp.log; exit 1; }
tail -2 gpurun_out/r06c_pytest_ddp.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q $T > gpurun_out/r06c_pytest_gpu.log 2>&1 || { tail -60 gpurun_out/r06c_pytest_gpu.log; exit 1; }
tail -2 gpurun_out/r06c_pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" || exit 1
