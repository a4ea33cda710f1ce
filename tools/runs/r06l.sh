# round 6: add_max without the per-float4 modulo, flat planes split for short rows: tests, old vs new
mkdir -p gpurun_out; export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests/test_gpu_projgemm.py tests/test_gpu_kernels.py -v -m gpu --timeout 300 --timeout-method thread -k "gemm or split or add_max or planes or dtproj or scan_mode2" > gpurun_out/r06l_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; grep -E "FAILED|ERROR|passed|failed" gpurun_out/r06l_tests.log | tail -6
[ $rc -eq 0 ] || exit $rc
for v in base new base new; do
  if [ $v = base ]; then lib=tools/variants/pre_addmax_r06.so; else lib=avse_challenge_amd/libavse_hip.so; fi
  AVSE_HIP_LIB=$lib timeout -k 10 300 python -u tools/split_bench.py > gpurun_out/r06l_bench_$v.log 2>&1; r=$?
  echo "bench $v rc=$r"; [ $r -eq 0 ] || exit $r
  grep '^{' gpurun_out/r06l_bench_$v.log | cut -c1-200
done
timeout -k 10 300 python -u tools/dtproj_bench.py > gpurun_out/r06l_dtproj.log 2>&1 || exit 1
grep '^{' gpurun_out/r06l_dtproj.log | cut -c1-200
timeout -k 10 600 python -u bench.py --workload mamba --steps 4 --warmup 2 --secondary "" --no-cpu-baseline --no-roofline-hip --no-parity > gpurun_out/r06l_c3.log 2>&1; r=$?
echo "c3 rc=$r"; grep '^{' gpurun_out/r06l_c3.log | cut -c1-200
[ $r -eq 0 ] || exit $r
timeout -k 10 600 python -u bench.py --workload avmamba --steps 4 --warmup 2 --secondary "" --no-cpu-baseline --no-roofline-hip --no-parity > gpurun_out/r06l_c5.log 2>&1; r=$?
echo "c5 rc=$r"; grep '^{' gpurun_out/r06l_c5.log | cut -c1-200
exit $r
