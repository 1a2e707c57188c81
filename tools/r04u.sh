#!/bin/bash
# kNN variant v2 (two-group kernel keeps the per-candidate j < N check): trace + A/B vs the tail-split build and the base
set -o pipefail
export PYTHONDONTWRITEBYTECODE=1
DGX_LIB=$(realpath tools/diag/libdgx_v2.so) timeout -k 10 300 python -u -m pytest tests/test_knn_gpu.py -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/r04u_pytest.log 2>&1 || { tail -30 gpurun_out/r04u_pytest.log; exit 1; }
tail -1 gpurun_out/r04u_pytest.log
for lib in tools/diag/libdgx_v2.so dgcnn.pytorch_amd/dgx/libdgx.so tools/diag/libdgx_base.so; do
  tag=r04u_$(basename $lib .so)
  DGX_LIB=$(realpath $lib) KT_ONLY=1 timeout -k 10 200 bash tools/profile.sh $tag --steps 20 --warmup 2 > gpurun_out/$tag.log 2>&1 || { tail gpurun_out/$tag.log; exit 1; }
  echo "== $tag"; grep -E "knn_kernel" gpurun_out/prof_$tag/kt_summary.txt
done
timeout -k 10 300 bash tools/ab_lib.sh tools/diag/libdgx_v2.so dgcnn.pytorch_amd/dgx/libdgx.so 3 > gpurun_out/r04u_ab.log 2>&1 || { cat gpurun_out/r04u_ab.log; exit 1; }
cat gpurun_out/r04u_ab.log
