#!/bin/bash
# fused BN -> ReLU in the avse4 lip front-end / ResNet: avse4 parity, avse1 C1 test, then avse4 step rate on / off
set -u
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 700 python -u -m pytest tests/test_gpu_models.py tests/test_gpu_fullsize.py tests/test_gpu_ckpt_io.py -k "avse4 or avse1_audio_only" -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/t17.log 2>&1
rc=$?; grep -E "PASSED|FAILED" gpurun_out/t17.log | cut -c1-120; grep -v "MIOpen(HIP)" gpurun_out/t17.log | grep -E "^E  " | head -8; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for b in 1 0; do
  AVSE_BNACT=$b timeout -k 10 400 python bench.py --workload avse4 --steps 10 --warmup 3 --no-roofline-hip --no-cpu-baseline --no-roofline > gpurun_out/bench_avse4_bnact$b.log 2>&1; rc=$?
  echo "avse4 bnact=$b: $(grep '^{' gpurun_out/bench_avse4_bnact$b.log | cut -c40-150)"; [ $rc -eq 0 ] || exit $rc
done
