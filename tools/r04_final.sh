mkdir -p gpurun_out; export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/r04h_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; grep -E "FAILED|ERROR|passed|failed" gpurun_out/r04h_tests.log | tail -8
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r04h_smoke.log 2>&1; rc=$?; echo "smoke rc=$rc"; grep smoke gpurun_out/r04h_smoke.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 900 python -u bench.py > gpurun_out/r04h_bench.log 2>&1; rc=$?; echo "bench rc=$rc"; grep '^{' gpurun_out/r04h_bench.log | tail -1 | cut -c1-1500
[ $rc -eq 0 ] || exit 1
PHASES="dwconv_gln_bwd" bash tools/pmc_traffic.sh gpurun_out/r04h_pmc gpurun_out/r04h_traffic.json > gpurun_out/r04h_pmc.log 2>&1; echo "pmc rc=$?"; tail -3 gpurun_out/r04h_pmc.log
