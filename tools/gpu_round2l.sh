#!/bin/bash
# avse1 lip branch on a second stream: equality test, then the C2 bench with and without it
set -u
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u -m pytest tests/test_gpu_models.py -k "branch_streams" -v --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/t9.log 2>&1
rc=$?; tail -4 gpurun_out/t9.log; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for s in 1 0 1; do
  AVSE_AVSE1_STREAMS=$s timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-roofline-hip --no-cpu-baseline > gpurun_out/bench_avse1_s$s.log 2>&1; rc=$?
  echo "streams=$s"; grep '^{' gpurun_out/bench_avse1_s$s.log | cut -c1-160; [ $rc -eq 0 ] || exit $rc
done
