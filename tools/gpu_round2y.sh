#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests/test_gpu_dpmamba.py tests/test_gpu_kernels.py -k "dpmamba or cconv or short" -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/t22.log 2>&1
rc=$?; tail -1 gpurun_out/t22.log; [ $rc -eq 0 ] || exit $rc
for w in dpmamba avse2; do
  timeout -k 10 600 python bench.py --workload $w --steps 5 --warmup 2 --no-roofline-hip > gpurun_out/bench_full_$w.log 2>&1; rc=$?
  echo "$w rc=$rc: $(grep '^{' gpurun_out/bench_full_$w.log | cut -c1-150)"; [ $rc -eq 0 ] || exit $rc
done
