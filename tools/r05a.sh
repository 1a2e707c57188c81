#!/bin/bash
# kNN split kernel (four candidate parts for small grids): kNN parity tests, B=4 kernel timings, B=4 and B=32 bench
set -o pipefail
export PYTHONDONTWRITEBYTECODE=1
timeout -k 10 600 python -u -m pytest tests/test_knn_gpu.py tests/test_knn_adversarial_gpu.py tests/test_knn_generic_gpu.py tests/test_edgeconv_gpu.py tests/test_host_ext_gpu.py -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/r05a_pytest.log 2>&1 || { tail -30 gpurun_out/r05a_pytest.log; exit 1; }
tail -2 gpurun_out/r05a_pytest.log
for lib in dgcnn.pytorch_amd/dgx/libdgx.so tools/diag/libdgx_base.so; do
  echo "== $(basename $lib) B=4"
  DGX_LIB=$(realpath $lib) timeout -k 10 200 python3 bench.py --batch 4 --no-cpu-baseline --no-eager-baseline --no-posemb-leg --no-edgeconv-leg --no-attention-leg --no-fp32-leg --steps 50 --warmup 10 2>/dev/null | python3 -c 'import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d["ms_per_step"], d.get("roofline",{}).get("knn_ms_by_layer"))' || exit 1
done
timeout -k 10 400 bash tools/ab_lib.sh dgcnn.pytorch_amd/dgx/libdgx.so tools/diag/libdgx_base.so 2 > gpurun_out/r05a_ab.log 2>&1 || { cat gpurun_out/r05a_ab.log; exit 1; }
cat gpurun_out/r05a_ab.log
