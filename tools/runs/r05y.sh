# avse4 1x1 Conv1d on avse_gemm_f32s (padded-row planes, the DS-conv gLN writing its GEMM's planes): parity tests, then
# the C4 step A/B (AVSE_AVSE4_PW_SPLIT=0: hipBLASLt fp32 bmm) and a kernel-trace profile of the new step
mkdir -p gpurun_out; export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests/test_gpu_projgemm.py tests/test_gpu_models.py tests/test_gpu_fullsize.py tests/test_gpu_kernels.py -v -m gpu -k "conv3d or avse4 or f32s or split or pointwise or planes or gln or dwconv or tblock or separator" --timeout 300 --timeout-method thread > gpurun_out/r05y6_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; grep -E "FAILED|ERROR|passed|failed" gpurun_out/r05y6_tests.log | tail -12
[ $rc -eq 0 ] || exit $rc
for v in 1; do
  AVSE_AVSE4_PW_SPLIT=$v timeout -k 10 300 python -u bench.py --workload avse4 --steps 10 --warmup 3 --no-cpu-baseline --no-roofline-hip > gpurun_out/r05y6_bench_$v.log 2>&1 || exit $?
  echo "split=$v: $(grep '^{' gpurun_out/r05y6_bench_$v.log | tail -1 | cut -c1-200)"
done
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r05y6_prof -o r05y -- python3 bench.py --workload avse4 --steps 3 --warmup 1 --no-cpu-baseline --no-roofline-hip > gpurun_out/r05y6_prof.log 2>&1; echo "prof rc=$?"
