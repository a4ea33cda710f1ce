# round-6 final validation on one MI355X: every -m gpu test, smoke(), the default bench line (headline + secondaries
# with their parity legs), the headline's rocprof windows
mkdir -p gpurun_out; export HSA_ENABLE_IPC_MODE_LEGACY=0
tag=${1:-r06final}
timeout -k 10 1100 python -u -m pytest tests -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/${tag}_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; grep -E "FAILED|ERROR|passed|failed" gpurun_out/${tag}_tests.log | tail -8
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${tag}_smoke.log 2>&1; r2=$?; echo "smoke rc=$r2"; tail -2 gpurun_out/${tag}_smoke.log
[ $r2 -eq 0 ] || exit $r2
timeout -k 10 1000 python -u bench.py > gpurun_out/${tag}_bench.log 2>&1; r3=$?; echo "bench rc=$r3"; grep '^{' gpurun_out/${tag}_bench.log | tail -1 | cut -c1-400
[ $r3 -eq 0 ] || exit $r3
exit $rc
