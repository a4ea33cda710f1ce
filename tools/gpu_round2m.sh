#!/bin/bash
# forward scan at 4 workgroups per CU (40 KB swizzled LDS): parity with each build, then A/B vs HEAD
set -u
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
for v in fwd4u4 fwd4u8; do
  AVSE_HIP_LIB=$PWD/expso/$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -k "scan" -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/t10_$v.log 2>&1
  rc=$?; echo "$v: $(tail -1 gpurun_out/t10_$v.log)"; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
done
bash tools/ab_scan.sh "head=expso/head.so u4=expso/fwd4u4.so u8=expso/fwd4u8.so" --pad --no-conv --cfg 64,1024,3999 16,1024,3999 --iters 10 || exit 1
bash tools/ab_scan.sh "head=expso/head.so u4=expso/fwd4u4.so u8=expso/fwd4u8.so" --pad --no-conv --dtype bf16 --cfg 32,1024,5999 --iters 10
