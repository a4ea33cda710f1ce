# round 6: the 8-wave dconv weight gradient: its tests, then old vs new kernel at the C2 shape (one box)
mkdir -p gpurun_out; export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py -v -m gpu --timeout 300 --timeout-method thread -k "dconv or dilated or audiofeat" > gpurun_out/r06d_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; grep -E "FAILED|ERROR|passed|failed|wgrad16 vs" gpurun_out/r06d_tests.log | tail -12
[ $rc -eq 0 ] || exit $rc
for v in base new base new; do
  if [ $v = base ]; then lib=tools/variants/base_r06.so; else lib=avse_challenge_amd/libavse_hip.so; fi
  AVSE_HIP_LIB=$lib timeout -k 10 300 python -u tools/dconv_bench.py --no-miopen > gpurun_out/r06d_bench_$v.log 2>&1; r=$?
  echo "bench $v rc=$r"; [ $r -eq 0 ] || exit $r
  python -c "
import json
for l in open('gpurun_out/r06d_bench_$v.log'):
    if l.startswith('{'):
        r = json.loads(l); print('$v', r['dilation'], 'wgrad16', r['split_wgrad16']['ms'], 'fwd conv', r['split_conv_only']['ms'])"
done
