#!/bin/bash
# kNN FIFO as packed (value, index) pairs + padding check only on the tail tile:
# kNN parity tests, kernel traces of both builds, interleaved step A/B
set -o pipefail
export PYTHONDONTWRITEBYTECODE=1
timeout -k 10 600 python -u -m pytest tests/test_knn_gpu.py tests/test_knn_adversarial_gpu.py tests/test_knn_generic_gpu.py tests/test_graph_feature_gpu.py tests/test_host_ext_gpu.py -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/r04t_pytest.log 2>&1 || { tail -30 gpurun_out/r04t_pytest.log; exit 1; }
tail -2 gpurun_out/r04t_pytest.log
for lib in dgcnn.pytorch_amd/dgx/libdgx.so tools/diag/libdgx_base.so; do
  tag=r04t_$(basename $lib .so)
  DGX_LIB=$(realpath $lib) KT_ONLY=1 timeout -k 10 200 bash tools/profile.sh $tag --steps 5 --warmup 2 > gpurun_out/$tag.log 2>&1 || { tail gpurun_out/$tag.log; exit 1; }
  echo "== $tag"; grep -E "knn" gpurun_out/prof_$tag/kt_summary.txt
done
timeout -k 10 600 bash tools/ab_lib.sh dgcnn.pytorch_amd/dgx/libdgx.so tools/diag/libdgx_base.so 3 > gpurun_out/r04t_ab.log 2>&1 || { cat gpurun_out/r04t_ab.log; exit 1; }
cat gpurun_out/r04t_ab.log
