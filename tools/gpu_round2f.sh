#!/bin/bash
# HIP LSTM parity + avse1/avse2 model tests, then the avse1 bench (graph-captured) and Mamba C3/C5 benches
set -u
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_models.py tests/test_gpu_avse2.py tests/test_gpu_fullsize.py -k "lstm or avse1 or avse2" -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/t6.log 2>&1
rc=$?; grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/t6.log | tail -30; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 400 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-roofline-hip > gpurun_out/bench_avse1.log 2>&1; rc=$?
grep '^{' gpurun_out/bench_avse1.log | cut -c1-700; [ $rc -eq 0 ] || { tail -5 gpurun_out/bench_avse1.log; exit $rc; }
bash tools/gpu_round2e.sh
