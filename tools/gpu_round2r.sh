#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 700 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_models.py -k "bnact or avse1_wave or avse1_audio_only or avse1_full" -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/t16.log 2>&1
rc=$?; grep -E "PASSED|FAILED" gpurun_out/t16.log | cut -c1-120; grep -v "MIOpen(HIP)" gpurun_out/t16.log | grep -E "^E  " | head -12; exit $rc
