# A/B: the split GEMM's fp32 outputs straight from the accumulators (epilogue 1) instead of LDS-staged lines
mkdir -p gpurun_out; export HSA_ENABLE_IPC_MODE_LEGACY=0
V=tools/variants/libavse_hip_epi1.so
AVSE_HIP_LIB=$V timeout -k 10 300 python -u -m pytest tests/test_gpu_projgemm.py -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/r05e1_tests.log 2>&1; rc=$?
echo "variant tests rc=$rc"; tail -2 gpurun_out/r05e1_tests.log
[ $rc -eq 0 ] || exit $rc
for w in avse4 mamba; do
  for lib in $V avse_challenge_amd/libavse_hip.so; do
    AVSE_HIP_LIB=$lib timeout -k 10 400 python -u bench.py --workload $w --steps 6 --warmup 2 --no-cpu-baseline --no-roofline-hip > gpurun_out/r05e1_bench.log 2>&1 || exit $?
    echo "$w $lib: $(grep '^{' gpurun_out/r05e1_bench.log | tail -1 | cut -c100-190)"
  done
done
