cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1
for s in 1 2 3 4; do DGX_LIB=$PWD/tools/diag/libdgx_kg$s.so timeout -k 10 60 python -u tools/kg_stage.py || exit 1; done
timeout -k 10 60 python -u tools/kg_stage.py || exit 1
timeout -k 10 600 python -u -m pytest tests/test_knn_grid_gpu.py tests/test_knn_gpu.py -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/r04e_pytest.log 2>&1; tail -3 gpurun_out/r04e_pytest.log; grep -E "^FAILED|Error" gpurun_out/r04e_pytest.log | head
