#!/bin/bash
# scan v3b: parity, A/B vs round 1
set -u
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_dropin.py tests/test_gpu_models.py -k "scan or cconv or bimamba or masknet or mamba or block or dropin or rms" -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/t5.log 2>&1
rc=$?; tail -4 gpurun_out/t5.log; [ $rc -eq 0 ] || exit $rc
bash tools/ab_scan.sh "r1=expso/base.so v3b=avse_challenge_amd/libavse_hip.so" --cfg 64,1024,3999 --no-conv || exit 1
bash tools/ab_scan.sh "r1bf=expso/base.so v3bbf=avse_challenge_amd/libavse_hip.so" --cfg 32,1024,5999 --dtype bf16 || exit 1
