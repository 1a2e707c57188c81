#!/bin/bash
# final tree check: the -m gpu suite and smoke()
set -o pipefail
export PYTHONDONTWRITEBYTECODE=1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r05e_pytest_gpu.log 2>&1 || { tail -30 gpurun_out/r05e_pytest_gpu.log; exit 1; }
tail -1 gpurun_out/r05e_pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" || exit 1
