# final tree after the padded-row split fix and the avse4 1x1-conv GEMM rates in the bench line: every -m gpu test,
# smoke(), the default bench line
mkdir -p gpurun_out; export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 1000 python -u -m pytest tests -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/r05z6_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; grep -E "FAILED|ERROR|passed|failed" gpurun_out/r05z6_tests.log | tail -8
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r05z6_smoke.log 2>&1; r2=$?; echo "smoke rc=$r2"; grep "smoke ok" gpurun_out/r05z6_smoke.log
[ $r2 -eq 0 ] || exit $r2
timeout -k 10 900 python -u bench.py > gpurun_out/r05z6_bench.log 2>&1; r3=$?; echo "bench rc=$r3"; grep '^{' gpurun_out/r05z6_bench.log | tail -1 | cut -c1-300
exit $r3
