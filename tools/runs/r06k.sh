# round 6: dt_proj epilogue writing whole rows (swapped MFMA operands): tests, old vs new, the Mamba model tests
mkdir -p gpurun_out; export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py -v -m gpu --timeout 300 --timeout-method thread -k "dtproj or scan_mode2" > gpurun_out/r06k_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; grep -E "FAILED|ERROR|passed|failed" gpurun_out/r06k_tests.log | tail -6
[ $rc -eq 0 ] || exit $rc
for v in base new base new; do
  if [ $v = base ]; then lib=tools/variants/pre_dtproj_r06.so; else lib=avse_challenge_amd/libavse_hip.so; fi
  AVSE_HIP_LIB=$lib timeout -k 10 300 python -u tools/dtproj_bench.py > gpurun_out/r06k_bench_$v.log 2>&1; r=$?
  echo "bench $v rc=$r"; [ $r -eq 0 ] || exit $r
  grep '^{' gpurun_out/r06k_bench_$v.log | cut -c1-250
done
timeout -k 10 800 python -u -m pytest tests/test_gpu_models.py tests/test_gpu_dropin.py tests/test_gpu_avmamba.py -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/r06k_models.log 2>&1; rc=$?
echo "model tests rc=$rc"; grep -E "FAILED|ERROR|passed|failed" gpurun_out/r06k_models.log | tail -6
exit $rc
