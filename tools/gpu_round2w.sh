#!/bin/bash
# padded-storage adds in BiMamba (direction sum, xz gradient): Mamba parity, then C3 / C5 step rates
set -u
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 900 python -u -m pytest tests/test_gpu_models.py tests/test_gpu_dropin.py tests/test_gpu_avmamba.py tests/test_gpu_dpmamba.py tests/test_gpu_fullsize.py -k "mamba or bimamba or dropin or masknet or dpmamba or block or rms or graph" -q --timeout 400 --timeout-method thread -p no:cacheprovider > gpurun_out/t21.log 2>&1
rc=$?; tail -2 gpurun_out/t21.log; grep FAILED gpurun_out/t21.log | head; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 400 python bench.py --workload mamba --steps 4 --warmup 2 --no-roofline-hip --no-cpu-baseline --no-roofline > gpurun_out/bench_m.log 2>&1; rc=$?
echo "mamba: $(grep '^{' gpurun_out/bench_m.log | cut -c60-170)"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --workload avmamba --steps 5 --warmup 2 --no-roofline-hip --no-cpu-baseline --no-roofline > gpurun_out/bench_am.log 2>&1; rc=$?
echo "avmamba: $(grep '^{' gpurun_out/bench_am.log | cut -c60-170)"; exit $rc
