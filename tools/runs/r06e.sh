# round 6: (1) the 8-wave dconv weight gradient's tests, (2) every -m gpu test on the tree without the env switches,
# (3) old vs new dconv weight gradient at the C2 shape, (4) C5 with the direction streams off / on
mkdir -p gpurun_out; export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py -v -m gpu --timeout 300 --timeout-method thread -k "dconv or dilated or audiofeat" > gpurun_out/r06e_dconv_tests.log 2>&1; rc=$?
echo "dconv tests rc=$rc"; grep -E "FAILED|ERROR|passed|failed" gpurun_out/r06e_dconv_tests.log | tail -6
[ $rc -eq 0 ] || exit $rc
for v in base new base new; do
  if [ $v = base ]; then lib=tools/variants/base_r06.so; else lib=avse_challenge_amd/libavse_hip.so; fi
  AVSE_HIP_LIB=$lib timeout -k 10 300 python -u tools/dconv_bench.py --no-miopen > gpurun_out/r06e_dbench_$v.log 2>&1; r=$?
  echo "dconv bench $v rc=$r"; [ $r -eq 0 ] || exit $r
  python -c "
import json
for l in open('gpurun_out/r06e_dbench_$v.log'):
    if l.startswith('{'):
        r = json.loads(l); print('$v', r['dilation'], 'wgrad16', r['split_wgrad16']['ms'], 'fwd conv', r['split_conv_only']['ms'])"
done
timeout -k 10 1000 python -u -m pytest tests -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/r06e_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; grep -E "FAILED|ERROR|passed|failed" gpurun_out/r06e_tests.log | tail -12
[ $rc -eq 0 ] || exit $rc
for ds in off on; do
  timeout -k 10 400 python -u bench.py --workload avmamba --steps 4 --warmup 1 --secondary "" --no-cpu-baseline --no-roofline-hip --no-parity --direction-streams $ds > gpurun_out/r06e_c5_$ds.log 2>&1; r=$?
  echo "c5 streams $ds rc=$r"; [ $r -eq 0 ] || exit $r
  grep '^{' gpurun_out/r06e_c5_$ds.log | tail -1 | python -c "import json,sys; r=json.loads(sys.stdin.read()); ro=r['roofline'] or {}; print(r['value'], r['ms_per_step'], ro.get('avg_ms'), ro.get('frac'), (ro.get('in_step_fwd') or {}).get('frac'))"
done
timeout -k 10 400 python -u bench.py --steps 10 --warmup 2 --secondary "" --no-cpu-baseline --no-roofline-hip --no-parity > gpurun_out/r06e_c2.log 2>&1; r=$?
echo "c2 rc=$r"; grep '^{' gpurun_out/r06e_c2.log | tail -1 | python -c "import json,sys; r=json.loads(sys.stdin.read()); ro=r['roofline']; print(r['value'], r['ms_per_step'], ro['kernel'][:20], ro['avg_ms'], ro['frac'], ro['in_step_serial'], [ (o['kernel'][:20], o['avg_ms'], o['frac']) for o in ro['other_conv_kernels']])"
exit $r
