#!/bin/bash
# full bench lines (roofline, cpu_baseline) for the non-default workloads
set -u
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
for w in mamba avmamba dpmamba avse2 avse4; do
  timeout -k 10 600 python bench.py --workload $w --steps 5 --warmup 2 --no-roofline-hip > gpurun_out/bench_full_$w.log 2>&1; rc=$?
  echo "$w rc=$rc: $(grep '^{' gpurun_out/bench_full_$w.log | cut -c1-150)"; [ $rc -eq 0 ] || exit $rc
done
