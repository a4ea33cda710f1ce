# A/B of the NHWC PReLU slope reduction (expso/prelu_old.so = the previous single-workgroup reduce) in the avse1 step,
# plus the avse1 model tests on the new one
mkdir -p gpurun_out; export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_models.py -k "avse1" > gpurun_out/prelu_test.log 2>&1 || { tail -30 gpurun_out/prelu_test.log; exit 1; }
tail -1 gpurun_out/prelu_test.log
for v in new old new old; do
  if [ $v = new ]; then lib=avse_challenge_amd/libavse_hip.so; else lib=expso/prelu_old.so; fi
  AVSE_HIP_LIB=$lib timeout -k 10 400 python -u bench.py --secondary "" --no-cpu-baseline --no-roofline-hip --no-roofline > gpurun_out/prelu_bench.log 2>&1 || exit 1
  echo "$v $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/prelu_bench.log)"
done
