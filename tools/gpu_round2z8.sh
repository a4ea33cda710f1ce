#!/bin/bash
# folded lip Conv3d forward on by default: full GPU suite, avse4 find pass + A/B (Cin = 1 variant), default bench line
set -u
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --timeout 400 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu_fold.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_gpu_fold.log; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
rm -rf gpurun_out/miopen_db && cp -r avse_challenge_amd/miopen_db gpurun_out/miopen_db
AVSE_MIOPEN_FIND=1 MIOPEN_USER_DB_PATH=$PWD/gpurun_out/miopen_db timeout -k 10 400 python bench.py --workload avse4 --steps 2 --warmup 2 --no-roofline-hip --no-cpu-baseline --no-roofline > gpurun_out/bench_find_avse4.log 2>&1; rc=$?
grep '^{' gpurun_out/bench_find_avse4.log | cut -c60-130; [ $rc -eq 0 ] || exit $rc
for f in 1 0 1; do
  MIOPEN_USER_DB_PATH=$PWD/gpurun_out/miopen_db AVSE_CONV3D_FOLD=$f timeout -k 10 300 python bench.py --workload avse4 --steps 10 --warmup 3 --no-roofline-hip --no-cpu-baseline --no-roofline > gpurun_out/bench_a4fold$f.log 2>&1; rc=$?
  echo "avse4 fold=$f: $(grep '^{' gpurun_out/bench_a4fold$f.log | cut -c60-130)"; [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 600 python bench.py --steps 10 --warmup 3 > gpurun_out/bench_default_fold.log 2>&1; rc=$?
grep '^{' gpurun_out/bench_default_fold.log | cut -c1-200; exit $rc
