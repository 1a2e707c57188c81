#!/bin/bash
# reverse graphs with 2 ranges per cloud (RG_CAP 20480) vs 4: reverse-graph tests on the variant, kernel traces, step A/B
set -o pipefail
export PYTHONDONTWRITEBYTECODE=1
DGX_LIB=$(realpath tools/diag/libdgx_rgp2.so) timeout -k 10 300 python -u -m pytest tests/test_graph_reverse_gpu.py tests/test_host_ext_gpu.py -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/r04r_pytest.log 2>&1 || { tail -20 gpurun_out/r04r_pytest.log; exit 1; }
tail -2 gpurun_out/r04r_pytest.log
for lib in dgcnn.pytorch_amd/dgx/libdgx.so tools/diag/libdgx_rgp2.so; do
  tag=r04r_$(basename $lib .so)
  DGX_LIB=$(realpath $lib) KT_ONLY=1 timeout -k 10 200 bash tools/profile.sh $tag --steps 5 --warmup 2 > gpurun_out/$tag.log 2>&1 || { tail gpurun_out/$tag.log; exit 1; }
  echo "== $tag"; grep -E "rev_graph" gpurun_out/prof_$tag/kt_summary.txt
done
timeout -k 10 600 bash tools/ab_lib.sh dgcnn.pytorch_amd/dgx/libdgx.so tools/diag/libdgx_rgp2.so 3 > gpurun_out/r04r_ab.log 2>&1 || { cat gpurun_out/r04r_ab.log; exit 1; }
cat gpurun_out/r04r_ab.log
DGX_LIB=$(realpath tools/diag/libdgx_sk16.so) KT_ONLY=1 timeout -k 10 200 bash tools/profile.sh r04r_sk16 --steps 5 --warmup 2 > gpurun_out/r04r_sk16.log 2>&1 || { tail gpurun_out/r04r_sk16.log; exit 1; }
echo "== sk16"; grep -E "smallk" gpurun_out/prof_r04r_sk16/kt_summary.txt; grep -E "smallk" gpurun_out/prof_r04r_libdgx/kt_summary.txt
