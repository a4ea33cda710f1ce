#!/bin/bash
# fused TCN kernels: parity, avse4 model tests, avse4 bench + roofline_hip list
set -u
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_models.py tests/test_gpu_fullsize.py -k "dwconv or gln or avse4" -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/t7.log 2>&1
rc=$?; grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/t7.log | tail -30; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 500 python bench.py --workload avse4 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/bench_avse4.log 2>&1; rc=$?
grep '^{' gpurun_out/bench_avse4.log > gpurun_out/lines_r2j.jsonl; cut -c1-400 gpurun_out/lines_r2j.jsonl; exit $rc
