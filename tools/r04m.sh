#!/bin/bash
# kNN ring-depth check: the kNN GPU tests on the new build, then an interleaved
# A/B of the cfg2 step (tools/diag/libdgx_head.so = two-slot ring) and a
# kernel trace of the new build.
set -o pipefail
export PYTHONDONTWRITEBYTECODE=1
timeout -k 10 600 python -u -m pytest tests/test_knn_gpu.py tests/test_knn_adversarial_gpu.py tests/test_edgeconv_gpu.py -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/r04m_pytest.log 2>&1 || { tail -20 gpurun_out/r04m_pytest.log; exit 1; }
tail -2 gpurun_out/r04m_pytest.log
timeout -k 10 600 bash tools/ab_lib.sh tools/diag/libdgx_head.so dgcnn.pytorch_amd/dgx/libdgx.so 3 > gpurun_out/r04m_ab.log 2>&1 || { cat gpurun_out/r04m_ab.log; exit 1; }
cat gpurun_out/r04m_ab.log
KT_ONLY=1 timeout -k 10 300 bash tools/profile.sh r04m --steps 5 --warmup 2 > gpurun_out/r04m_prof.log 2>&1 || { tail gpurun_out/r04m_prof.log; exit 1; }
grep knn_kernel gpurun_out/prof_r04m/kt_summary.txt
