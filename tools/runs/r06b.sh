# round 6: bench line with the parity legs (headline avse1 + C1, secondaries C3 / C4 / C5)
mkdir -p gpurun_out; export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 1000 python -u bench.py --steps 5 --warmup 2 --no-roofline-hip > gpurun_out/r06b_bench.log 2>&1; rc=$?
echo "bench rc=$rc"; grep '^{' gpurun_out/r06b_bench.log | tail -1 | python -c "import json,sys; r=json.loads(sys.stdin.read()); print(r['value'], json.dumps(r['parity'])); [print(s['workload'], s.get('value'), json.dumps(s.get('parity')), s.get('error')) for s in r.get('secondary', [])]"
exit $rc
