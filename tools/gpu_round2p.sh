#!/bin/bash
# NHWC lip ResNet trunk, immediate mode (no find-db records for its shapes): first-step time and step rate
set -u
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
for cl in 1 0; do
  AVSE_LIP_CHANNELS_LAST=$cl timeout -k 10 500 python bench.py --steps 10 --warmup 3 --no-roofline-hip --no-cpu-baseline --no-roofline > gpurun_out/bench_lipcl$cl.log 2>&1; rc=$?
  echo "lip_cl=$cl: $(grep -E '^\[bench\] warmup' gpurun_out/bench_lipcl$cl.log | tr '\n' ' ') $(grep '^{' gpurun_out/bench_lipcl$cl.log | cut -c60-150)"; [ $rc -eq 0 ] || exit $rc
done
