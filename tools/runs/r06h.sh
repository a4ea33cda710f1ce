# round 6: the default bench line (headline + parity + secondaries, as the driver runs it), then a rocprofv3 kernel
# trace of the avse1 step (timed window + serial-branch roofline window)
mkdir -p gpurun_out; export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 900 python -u bench.py > gpurun_out/r06h_bench.log 2>&1; r=$?
echo "bench rc=$r"; grep '^{' gpurun_out/r06h_bench.log | tail -1 | python -c "
import json,sys; r=json.loads(sys.stdin.read()); ro=r['roofline']
print(r['value'], r['ms_per_step'], ro['avg_ms'], ro['frac'], json.dumps(r['parity'])[:300])
print('cpu', r['cpu_baseline']['value'], r['cpu_baseline']['cores'])
for s in r.get('secondary', []): print(s['workload'], s.get('value'), s.get('ms_per_step'), (s.get('roofline') or {}).get('frac'), json.dumps(s.get('parity'))[:200], s.get('error'))"
[ $r -eq 0 ] || exit $r
timeout -k 10 800 bash tools/profile_bench.sh gpurun_out/r06h_prof 10 > gpurun_out/r06h_prof.log 2>&1; r=$?
echo "profile rc=$r"; head -25 gpurun_out/r06h_prof/window_stats.csv | cut -c1-160
exit $r
