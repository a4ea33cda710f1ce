# add_max: 4 float4 pairs in flight, no column mask when the rows are unpadded (the avse4 residual sum); parity tests,
# then the C4 / C3 steps
mkdir -p gpurun_out; export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests/test_gpu_projgemm.py tests/test_gpu_models.py tests/test_gpu_kernels.py -v -m gpu -k "add_max or avse4 or mamba or masknet or bimamba or f32s" --timeout 300 --timeout-method thread > gpurun_out/r05z5_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; grep -E "FAILED|ERROR|passed|failed" gpurun_out/r05z5_tests.log | tail -12
[ $rc -eq 0 ] || exit $rc
for w in avse4 mamba; do
  timeout -k 10 400 python -u bench.py --workload $w --steps 6 --warmup 2 --no-cpu-baseline --no-roofline-hip > gpurun_out/r05z5_bench_$w.log 2>&1 || exit $?
  echo "$w: $(grep '^{' gpurun_out/r05z5_bench_$w.log | tail -1 | cut -c100-220)"
done
