# round 6: sconv forward with a precomputed DMA plan, flat planes split with a tail row: tests, old vs new, C2 step
mkdir -p gpurun_out; export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests/test_gpu_sconv.py tests/test_gpu_projgemm.py tests/test_gpu_kernels.py -v -m gpu --timeout 300 --timeout-method thread -k "sconv or trunk or gemm or split or add_max or planes" > gpurun_out/r06m_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; grep -E "FAILED|ERROR|passed|failed" gpurun_out/r06m_tests.log | tail -6
[ $rc -eq 0 ] || exit $rc
for v in base new base new; do
  if [ $v = base ]; then lib=tools/variants/pre_addmax_r06.so; else lib=avse_challenge_amd/libavse_hip.so; fi
  AVSE_HIP_LIB=$lib timeout -k 10 300 python -u tools/split_bench.py > gpurun_out/r06m_split_$v.log 2>&1 || exit 1
  AVSE_HIP_LIB=$lib timeout -k 10 300 python -u tools/sconv_bench.py --no-miopen > gpurun_out/r06m_sbench_$v.log 2>&1 || exit 1
  echo "bench $v"; grep '^{' gpurun_out/r06m_split_$v.log | cut -c1-120
  python -c "
import json
for l in open('gpurun_out/r06m_sbench_$v.log'):
    if l.startswith('{'):
        r = json.loads(l); print('$v', r['shape'], 'fwd', r['split_fwd']['ms'], 'dgrad', (r.get('split_dgrad') or {}).get('ms'), 'wgrad', r['split_wgrad']['ms'])"
done
timeout -k 10 400 python -u bench.py --steps 10 --warmup 2 --secondary "" --no-cpu-baseline --no-roofline-hip --no-parity > gpurun_out/r06m_c2.log 2>&1; r=$?
echo "c2 rc=$r"; grep '^{' gpurun_out/r06m_c2.log | tail -1 | python -c "import json,sys; r=json.loads(sys.stdin.read()); ro=r['roofline']; print(r['value'], r['ms_per_step'], ro['kernel'][:20], ro['avg_ms'], ro['frac'], ro['in_step_serial'])"
exit $r
