# round 6: C3 (fp32) on BiMambaSerial with producer-side maxima (one atomic per workgroup / a row-max pass), A/B vs add_max
mkdir -p gpurun_out; export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 900 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_models.py tests/test_gpu_avmamba.py tests/test_gpu_fullsize.py -v -m gpu --timeout 300 --timeout-method thread -k "accumulate or mamba or trainer or graph" > gpurun_out/r06s_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; grep -E "FAILED|ERROR|passed|failed" gpurun_out/r06s_tests.log | tail -6
[ $rc -eq 0 ] || exit $rc
for v in new old new old; do
  flag=""; [ $v = old ] && flag="--old"
  timeout -k 10 500 python -u tools/c5_serial_ab.py $flag -- --workload mamba --steps 4 --warmup 2 --secondary "" --no-cpu-baseline --no-roofline-hip --no-parity > gpurun_out/r06s_c3_$v.log 2>&1; r=$?
  echo "c3 $v rc=$r"; [ $r -eq 0 ] || exit $r
  grep '^{' gpurun_out/r06s_c3_$v.log | tail -1 | python -c "
import json,sys; r=json.loads(sys.stdin.read()); ro=r['roofline']; print('$v', r['value'], r['ms_per_step'], 'bwd', ro['avg_ms'], ro['per_launch_ms'], 'fwd', ro['in_step_fwd']['avg_ms'])"
done
exit 0
