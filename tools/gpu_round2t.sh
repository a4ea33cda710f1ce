#!/bin/bash
# maxpool plane kernels + two-stage BN finalize: parity, then avse1 / avse4 step rates
set -u
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 900 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_models.py tests/test_gpu_fullsize.py -k "maxpool or bnact or avse1 or avse4" -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/t18.log 2>&1
rc=$?; tail -2 gpurun_out/t18.log; grep -E "FAILED" gpurun_out/t18.log | cut -c1-150; grep -v "MIOpen(HIP)" gpurun_out/t18.log | grep -E "^E  " | head -8; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for w in avse1 avse4; do
  timeout -k 10 400 python bench.py --workload $w --steps 10 --warmup 3 --no-roofline-hip --no-cpu-baseline --no-roofline > gpurun_out/bench_$w.log 2>&1; rc=$?
  echo "$w: $(grep '^{' gpurun_out/bench_$w.log | cut -c40-170)"; [ $rc -eq 0 ] || exit $rc
done
