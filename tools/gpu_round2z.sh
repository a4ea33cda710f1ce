#!/bin/bash
# round 2 (session 3): forward pipelining / early z, backward lam*dA reuse — parity per variant, then A/B
set -u
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 AVSE_TIME_ALIGN_BYTES=128
for v in p2ze p3 lda; do
  AVSE_HIP_LIB=$PWD/expso/$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -k "scan" -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/t_$v.log 2>&1
  rc=$?; echo "$v: $(tail -1 gpurun_out/t_$v.log)"; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
done
bash tools/ab_scan.sh "base=expso/base.so ze=expso/ze.so p2=expso/p2.so p2ze=expso/p2ze.so p3=expso/p3.so lda=expso/lda.so" --cfg 64,1024,3999 --no-conv --pad || exit 1
bash tools/ab_scan.sh "base=expso/base.so p2ze=expso/p2ze.so p3=expso/p3.so lda=expso/lda.so" --cfg 32,1024,5999 --dtype bf16 --pad --no-conv || exit 1
