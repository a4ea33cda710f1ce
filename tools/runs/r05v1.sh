# round-5 validation, part 1: every -m gpu test and smoke()
mkdir -p gpurun_out; export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 1000 python -u -m pytest tests -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/r05v1_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; grep -E "FAILED|ERROR|passed|failed" gpurun_out/r05v1_tests.log | tail -12
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r05v1_smoke.log 2>&1; rc2=$?; echo "smoke rc=$rc2"; tail -3 gpurun_out/r05v1_smoke.log
exit $rc
