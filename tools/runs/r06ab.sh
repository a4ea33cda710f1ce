# round 6 (ab): the shortcut input-gradient GEMM alone (library vs split GEMM); the C5 projections casting once under
# autocast: Mamba / C5 tests and the C5 line (r06t: 59.82 utt/s)
mkdir -p gpurun_out; export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 120 python -u tools/lstm_gemm_probe.py > gpurun_out/r06ab_gemm_probe.jsonl 2>&1; r=$?; cat gpurun_out/r06ab_gemm_probe.jsonl; [ $r -eq 0 ] || exit $r
timeout -k 10 700 python -u -m pytest tests -k "mamba or avmamba or dpmamba or bimamba or masknet or dropin or projgemm" -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/r06ab_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; grep -E "FAILED|ERROR|passed|failed" gpurun_out/r06ab_tests.log | tail -6
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py --workload avmamba --steps 4 --warmup 1 --no-cpu-baseline --no-roofline-hip --no-parity > gpurun_out/r06ab_c5.log 2>&1; r=$?
echo "c5 rc=$r"; grep '^{' gpurun_out/r06ab_c5.log | tail -1 | cut -c1-200
exit $r
