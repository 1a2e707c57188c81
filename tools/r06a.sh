#!/bin/bash
# round 5, session a: the unified C++ schedule (dgx_host::chain_* / pointconv_* / dgcnn),
# autocast rule, SyncBN from C++; new tests first, then the whole -m gpu suite, smoke, bench
set -o pipefail
export PYTHONDONTWRITEBYTECODE=1
mkdir -p gpurun_out
timeout -k 10 60 ./tools/knn32_probe > gpurun_out/r06a_knn32_probe.log 2>&1; cat gpurun_out/r06a_knn32_probe.log
timeout -k 10 600 python -u -m pytest tests/test_host_ext_gpu.py tests/test_amp_bn_gpu.py tests/test_ddp_gpu.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r06a_pytest_new.log 2>&1 || { tail -80 gpurun_out/r06a_pytest_new.log; exit 1; }
tail -2 gpurun_out/r06a_pytest_new.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r06a_pytest_gpu.log 2>&1 || { tail -60 gpurun_out/r06a_pytest_gpu.log; exit 1; }
tail -2 gpurun_out/r06a_pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" || exit 1
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r06a_bench.log 2>&1 || { tail -30 gpurun_out/r06a_bench.log; exit 1; }
tail -c 3000 gpurun_out/r06a_bench.log
