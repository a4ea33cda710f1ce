#!/bin/bash
# round-2 check: C1 / C5 GPU tests, then scan A/B of experiment builds (bwd parts compiled out, aligned strides)
set -u
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_models.py tests/test_gpu_fullsize.py tests/test_gpu_kernels.py tests/test_gpu_avmamba.py -k "audio_only or c5 or production" -v --timeout 400 --timeout-method thread -p no:cacheprovider -s > gpurun_out/t3.log 2>&1
rc=$?; grep -E "PASSED|FAILED|Error|passed|failed|C5 n_mamba|RMS" gpurun_out/t3.log | tail -20; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
bash tools/ab_scan.sh "base=expso/base.so noadjexp=expso/noadjexp.so nopass1=expso/nopass1.so nored=expso/nored.so" --cfg 64,1024,3999 --no-conv || exit 1
echo "== padded inputs, aligned outputs (base)"
AVSE_TIME_ALIGN_BYTES=128 AVSE_HIP_LIB=$PWD/expso/base.so timeout -k 10 200 python tools/scan_bench.py --cfg 64,1024,3999 --pad > gpurun_out/ab_pad.log 2>&1 && cat gpurun_out/ab_pad.log
echo "== bf16 C5 base / padded"
AVSE_HIP_LIB=$PWD/expso/base.so timeout -k 10 200 python tools/scan_bench.py --cfg 32,1024,5999 --dtype bf16 > gpurun_out/ab_bf.log 2>&1 && cat gpurun_out/ab_bf.log
AVSE_TIME_ALIGN_BYTES=128 AVSE_HIP_LIB=$PWD/expso/base.so timeout -k 10 200 python tools/scan_bench.py --cfg 32,1024,5999 --dtype bf16 --pad > gpurun_out/ab_bfpad.log 2>&1 && cat gpurun_out/ab_bfpad.log
