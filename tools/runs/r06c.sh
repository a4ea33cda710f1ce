# round 6: every -m gpu test on the tree without the env switches; then C5 with the direction streams off / on
mkdir -p gpurun_out; export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 1000 python -u -m pytest tests -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/r06c_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; grep -E "FAILED|ERROR|passed|failed" gpurun_out/r06c_tests.log | tail -12
[ $rc -eq 0 ] || exit $rc
for ds in off on off on; do
  timeout -k 10 400 python -u bench.py --workload avmamba --steps 4 --warmup 1 --secondary "" --no-cpu-baseline --no-roofline-hip --no-parity --direction-streams $ds > gpurun_out/r06c_c5_$ds.log 2>&1; r=$?
  echo "c5 streams $ds rc=$r"; [ $r -eq 0 ] || exit $r
  grep '^{' gpurun_out/r06c_c5_$ds.log | tail -1 | python -c "import json,sys; r=json.loads(sys.stdin.read()); ro=r['roofline'] or {}; print(r['value'], r['ms_per_step'], ro.get('avg_ms'), ro.get('frac'), (ro.get('in_step_fwd') or {}).get('frac'))"
done
