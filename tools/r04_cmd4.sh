mkdir -p gpurun_out; export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 200 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_dist.py -v -s -m gpu -k "error_flag or two_ranks" --timeout 150 --timeout-method thread > gpurun_out/r04d_occ.log 2>&1; rc=$?
echo "occ rc=$rc"; grep -E "PASS|FAIL|assert|branch|rank " gpurun_out/r04d_occ.log | tail -20
[ $rc -eq 0 ] || exit 1
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/r04c_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; grep -E "FAILED|ERROR|passed|failed" gpurun_out/r04c_tests.log | tail -8
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r04c_smoke.log 2>&1; echo "smoke rc=$?"; grep smoke gpurun_out/r04c_smoke.log
timeout -k 10 900 python -u bench.py > gpurun_out/r04c_bench.log 2>&1; echo "bench rc=$?"; grep '^{' gpurun_out/r04c_bench.log | tail -1 | cut -c1-3000
