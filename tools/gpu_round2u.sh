#!/bin/bash
# eager vs captured step rate (the N > 1 path runs forward/backward eagerly)
set -u
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
for w in avse1 avse4; do
  for g in "" "--no-graph"; do
    timeout -k 10 400 python bench.py --workload $w --steps 10 --warmup 3 --no-roofline-hip --no-cpu-baseline --no-roofline $g > gpurun_out/bench_eg.log 2>&1; rc=$?
    echo "$w $g: $(grep '^{' gpurun_out/bench_eg.log | cut -c40-160)"; [ $rc -eq 0 ] || exit $rc
  done
done
