#!/bin/bash
# vectorised causal-conv rows: parity (kernel + Mamba model tests), then the C3 conv timings
set -u
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 900 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_models.py tests/test_gpu_dropin.py tests/test_gpu_avmamba.py tests/test_gpu_dpmamba.py -k "cconv or conv1d or mamba or bimamba or dropin or masknet or dpmamba or block or rms" -q --timeout 400 --timeout-method thread -p no:cacheprovider > gpurun_out/t20.log 2>&1
rc=$?; tail -2 gpurun_out/t20.log; grep FAILED gpurun_out/t20.log | head; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 200 python tools/scan_bench.py --pad --cfg 64,1024,3999 16,1024,3999 --iters 10 2>&1 | grep cfg
