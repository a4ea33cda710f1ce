# round 6 (ac): bf16 RMSNorm rows in the C5 Block (norm output in bf16 under autocast, the mixer's bf16 output read as
# it is): the whole -m gpu suite, C5 and C3 lines
mkdir -p gpurun_out; export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 900 python -u -m pytest tests -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/r06ac_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; grep -E "FAILED|ERROR|passed|failed" gpurun_out/r06ac_tests.log | tail -6
[ $rc -eq 0 ] || exit $rc
for w in avmamba mamba; do
  timeout -k 10 400 python -u bench.py --workload $w --steps 4 --warmup 1 --no-cpu-baseline --no-roofline-hip > gpurun_out/r06ac_$w.log 2>&1; r=$?
  echo "$w rc=$r"; grep '^{' gpurun_out/r06ac_$w.log | tail -1 | python -c "import json,sys; r=json.loads(sys.stdin.read()); print(r['value'], r['ms_per_step'], json.dumps(r.get('parity'))[:400])"
  [ $r -eq 0 ] || exit $r
done
