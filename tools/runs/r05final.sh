# round-5 final validation on one MI355X: every -m gpu test, smoke(), the default bench line (headline + secondaries),
# the headline's rocprof windows, PMC traffic of the scan kernels as the model now calls them (delta_softplus = 2)
mkdir -p gpurun_out; export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 1000 python -u -m pytest tests -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/r05h2_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; grep -E "FAILED|ERROR|passed|failed" gpurun_out/r05h2_tests.log | tail -8
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r05h2_smoke.log 2>&1; r2=$?; echo "smoke rc=$r2"; grep "smoke ok" gpurun_out/r05h2_smoke.log
[ $r2 -eq 0 ] || exit $r2
timeout -k 10 900 python -u bench.py > gpurun_out/r05h2_bench.log 2>&1; r3=$?; echo "bench rc=$r3"; grep '^{' gpurun_out/r05h2_bench.log | tail -1 | cut -c1-400
[ $r3 -eq 0 ] || exit $r3
timeout -k 10 400 bash tools/profile_bench.sh gpurun_out/r05h2_prof_avse1 10; r4=$?; echo "prof rc=$r4"
[ $r4 -eq 0 ] || exit $r4
echo "pmc: unchanged scan kernels, see profiles/r05g_traffic.json"
exit $rc
