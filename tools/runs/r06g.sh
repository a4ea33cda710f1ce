# round 6: conflict-free transposed-read swizzles in the dconv / sconv weight gradients: tests, A/B, PMC, C2 step
mkdir -p gpurun_out; export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_sconv.py -v -m gpu --timeout 300 --timeout-method thread -k "dconv or dilated or audiofeat or sconv or trunk" > gpurun_out/r06g_tests.log 2>&1; rc=$?
echo "conv tests rc=$rc"; grep -E "FAILED|ERROR|passed|failed" gpurun_out/r06g_tests.log | tail -6
[ $rc -eq 0 ] || exit $rc
for v in base new base new; do
  if [ $v = base ]; then lib=tools/variants/wgrad8_r06.so; else lib=avse_challenge_amd/libavse_hip.so; fi
  AVSE_HIP_LIB=$lib timeout -k 10 300 python -u tools/dconv_bench.py --no-miopen > gpurun_out/r06g_dbench_$v.log 2>&1; r=$?
  [ $r -eq 0 ] || exit $r
  AVSE_HIP_LIB=$lib timeout -k 10 300 python -u tools/sconv_bench.py --no-miopen > gpurun_out/r06g_sbench_$v.log 2>&1; r=$?
  echo "bench $v rc=$r"; [ $r -eq 0 ] || exit $r
  python -c "
import json
for f in ('gpurun_out/r06g_dbench_$v.log', 'gpurun_out/r06g_sbench_$v.log'):
    for l in open(f):
        if l.startswith('{'):
            r = json.loads(l)
            print('$v', r.get('dilation', r.get('shape')), 'wgrad', (r.get('split_wgrad16') or r.get('split_wgrad'))['ms'])"
done
for v in nw4 cur nw4 cur; do
  if [ $v = nw4 ]; then lib=tools/variants/dfwd_nw4.so; else lib=avse_challenge_amd/libavse_hip.so; fi
  AVSE_HIP_LIB=$lib timeout -k 10 300 python -u tools/dconv_bench.py --no-miopen > gpurun_out/r06g_fwd_$v.log 2>&1; r=$?
  [ $r -eq 0 ] || exit $r
  python -c "
import json
for l in open('gpurun_out/r06g_fwd_$v.log'):
    if l.startswith('{'):
        r = json.loads(l); print('$v', r['dilation'], 'fwd conv', r['split_conv_only']['ms'])"
done
timeout -k 10 400 bash tools/pmc_cmd.sh gpurun_out/r06g_pmc_dconv tools/dconv_bench.py --no-miopen --dils 4 --iters 3 > gpurun_out/r06g_pmc_dconv.log 2>&1; r=$?
echo "pmc rc=$r"; grep -A3 "dcf::wgrad_kernel" gpurun_out/r06g_pmc_dconv/summary.txt; grep -A16 "dcf::wgrad_kernel" gpurun_out/r06g_pmc_dconv/summary.txt | grep "BANK\|IDX_ACT\|MFMA_BUSY\|GRBM"
timeout -k 10 400 python -u bench.py --steps 10 --warmup 2 --secondary "" --no-cpu-baseline --no-roofline-hip --no-parity > gpurun_out/r06g_c2.log 2>&1; r=$?
echo "c2 rc=$r"; grep '^{' gpurun_out/r06g_c2.log | tail -1 | python -c "import json,sys; r=json.loads(sys.stdin.read()); ro=r['roofline']; print(r['value'], r['ms_per_step'], ro['kernel'][:20], ro['avg_ms'], ro['frac'], ro['in_step_serial'], [ (o['kernel'][:20], o['avg_ms'], o['frac']) for o in ro['other_conv_kernels']])"
exit $r
