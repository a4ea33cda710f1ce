# fewer same-word atomics in the absmax / producer-max passes (projgemm planes, dconv split16, rmsnorm outputs):
# parity tests of those kernels, then the C3 / C4 / C2 steps
mkdir -p gpurun_out; export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests/test_gpu_projgemm.py tests/test_gpu_kernels.py -v -m gpu -k "rmsnorm or dconv or split or f32s or gemm or planes or pointwise" --timeout 300 --timeout-method thread > gpurun_out/r05z3_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; grep -E "FAILED|ERROR|passed|failed" gpurun_out/r05z3_tests.log | tail -12
[ $rc -eq 0 ] || exit $rc
for w in avse4 mamba; do
  timeout -k 10 400 python -u bench.py --workload $w --steps 6 --warmup 2 --no-cpu-baseline --no-roofline-hip > gpurun_out/r05z3_bench_$w.log 2>&1 || exit $?
  echo "$w: $(grep '^{' gpurun_out/r05z3_bench_$w.log | tail -1 | cut -c1-220)"
done
timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-roofline-hip --secondary '' > gpurun_out/r05z3_bench_avse1.log 2>&1 || exit $?
echo "avse1: $(grep '^{' gpurun_out/r05z3_bench_avse1.log | tail -1 | cut -c1-220)"
