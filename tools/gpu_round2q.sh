#!/bin/bash
# fused BatchNorm -> [+res] -> act: kernel parity, avse1 model parity, then the C2 step rate with / without it
set -u
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -k "bnact" -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/t14.log 2>&1
rc=$?; grep -E "PASSED|FAILED" gpurun_out/t14.log | cut -c1-120; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests/test_gpu_models.py tests/test_gpu_fullsize.py -k "avse1" -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/t15.log 2>&1
rc=$?; grep -E "PASSED|FAILED" gpurun_out/t15.log | cut -c1-120; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for b in 1 0; do
  AVSE_BNACT=$b timeout -k 10 400 python bench.py --steps 10 --warmup 3 --no-roofline-hip --no-cpu-baseline --no-roofline > gpurun_out/bench_bnact$b.log 2>&1; rc=$?
  echo "bnact=$b: $(grep -E '^\[bench\] warmup 1' gpurun_out/bench_bnact$b.log) $(grep '^{' gpurun_out/bench_bnact$b.log | cut -c60-150)"; [ $rc -eq 0 ] || exit $rc
done
