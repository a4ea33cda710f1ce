#!/bin/bash
# NHWC lip ResNet trunk: PReLU NHWC + avse1 parity, MIOpen find-db records for the NHWC shapes, then the A/B
set -u
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 500 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_models.py -k "prelu or avse1_full_golden or avse1_wave_frontend" -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/t13.log 2>&1
rc=$?; grep -E "PASSED|FAILED" gpurun_out/t13.log | cut -c1-120; [ $rc -eq 0 ] || exit $rc
rm -rf gpurun_out/miopen_db && cp -r avse_challenge_amd/miopen_db gpurun_out/miopen_db
AVSE_MIOPEN_FIND=1 MIOPEN_USER_DB_PATH=$PWD/gpurun_out/miopen_db timeout -k 10 700 python bench.py --steps 2 --warmup 2 --no-roofline-hip --no-cpu-baseline --no-roofline > gpurun_out/bench_find.log 2>&1; rc=$?
grep -E '^\[bench\] warm|^\{' gpurun_out/bench_find.log | cut -c1-120; [ $rc -eq 0 ] || exit $rc
for cl in 1 0 1; do
  MIOPEN_USER_DB_PATH=$PWD/gpurun_out/miopen_db AVSE_LIP_CHANNELS_LAST=$cl timeout -k 10 400 python bench.py --steps 10 --warmup 3 --no-roofline-hip --no-cpu-baseline --no-roofline > gpurun_out/bench_lipcl$cl.log 2>&1; rc=$?
  echo "lip_cl=$cl: $(grep -E '^\[bench\] warmup 1' gpurun_out/bench_lipcl$cl.log) $(grep '^{' gpurun_out/bench_lipcl$cl.log | cut -c60-150)"; [ $rc -eq 0 ] || exit $rc
done
