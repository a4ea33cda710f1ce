#!/bin/bash
# 128-B aligned time stride on the Mamba path: Mamba / C5 / DPMamba / drop-in tests, then C3 and C5 benches
set -u
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 700 python -u -m pytest tests/test_gpu_models.py tests/test_gpu_avmamba.py tests/test_gpu_dpmamba.py tests/test_gpu_dropin.py tests/test_gpu_fullsize.py -k "mamba or bimamba or masknet or dpmamba or dropin or block or rms or avmamba" -q --timeout 400 --timeout-method thread -p no:cacheprovider > gpurun_out/t8.log 2>&1
rc=$?; tail -3 gpurun_out/t8.log; grep FAILED gpurun_out/t8.log | head; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python bench.py --workload mamba --steps 4 --warmup 2 --no-roofline-hip --no-cpu-baseline > gpurun_out/bench_mamba_al.log 2>&1; rc=$?
grep '^{' gpurun_out/bench_mamba_al.log | cut -c1-200; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --workload avmamba --steps 5 --warmup 2 --no-roofline-hip --no-cpu-baseline > gpurun_out/bench_avmamba_al.log 2>&1; rc=$?
grep '^{' gpurun_out/bench_avmamba_al.log | cut -c1-200; exit $rc
