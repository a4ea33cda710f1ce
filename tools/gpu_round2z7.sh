#!/bin/bash
# avse1 lip Conv3d forward folded into a Conv2d over frames: probe (immediate / find), then the bench A/B
set -u
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
rm -rf gpurun_out/miopen_db && cp -r avse_challenge_amd/miopen_db gpurun_out/miopen_db
export MIOPEN_USER_DB_PATH=$PWD/gpurun_out/miopen_db
timeout -k 10 400 python tools/conv3d_fold_probe.py > gpurun_out/fold_probe.log 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/fold_probe.log | tail -4; [ $rc -eq 0 ] || exit $rc
for f in 1 0 1; do
  AVSE_CONV3D_FOLD=$f timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-roofline-hip --no-cpu-baseline --no-roofline > gpurun_out/bench_fold$f.log 2>&1; rc=$?
  echo "fold=$f: $(grep '^{' gpurun_out/bench_fold$f.log | cut -c60-130)"; [ $rc -eq 0 ] || exit $rc
done
