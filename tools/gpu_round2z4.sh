#!/bin/bash
# NHWC lip ResNet trunk with MIOpen find-db records for ITS shapes: find pass (cudnn.benchmark) with the trunk
# channels-last, then the A/B of both layouts on the extended db; the db comes back under gpurun_out/miopen_db
set -u
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
rm -rf gpurun_out/miopen_db && cp -r avse_challenge_amd/miopen_db gpurun_out/miopen_db
MIOPEN_FIND_MODE=${FIND_MODE:-5} AVSE_LIP_CHANNELS_LAST=1 AVSE_MIOPEN_FIND=1 MIOPEN_USER_DB_PATH=$PWD/gpurun_out/miopen_db timeout -k 10 600 python bench.py --steps 2 --warmup 2 --no-roofline-hip --no-cpu-baseline --no-roofline > gpurun_out/bench_find_cl.log 2>&1; rc=$?
grep -E '^\[bench\] warm|^\{' gpurun_out/bench_find_cl.log | cut -c1-120; [ $rc -eq 0 ] || exit $rc
for cl in 1 0 1; do
  MIOPEN_USER_DB_PATH=$PWD/gpurun_out/miopen_db AVSE_LIP_CHANNELS_LAST=$cl timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-roofline-hip --no-cpu-baseline --no-roofline > gpurun_out/bench_lipcl$cl.log 2>&1; rc=$?
  echo "lip_cl=$cl: $(grep -E '^\[bench\] warmup 1' gpurun_out/bench_lipcl$cl.log) $(grep '^{' gpurun_out/bench_lipcl$cl.log | cut -c60-150)"; [ $rc -eq 0 ] || exit $rc
done
