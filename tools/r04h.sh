export PYTHONDONTWRITEBYTECODE=1
timeout -k 10 600 python -u -m pytest tests/test_library_ops_gpu.py tests/test_host_ext_gpu.py tests/test_partseg.py -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/r04h_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/r04h_pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 150 python -u tools/host_profile.py 20 > gpurun_out/r04h_host.log 2>&1 || exit $?
head -3 gpurun_out/r04h_host.log
timeout -k 10 300 python -u bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-eager-baseline --no-fp32-leg --no-edgeconv-leg --no-posemb-leg --no-attention-leg > gpurun_out/r04h_bench.log 2>&1 || exit $?
tail -c 600 gpurun_out/r04h_bench.log
