#!/bin/bash
# scan backward scheduling fences: sched_barrier masks that let VALU / SALU / transcendentals cross step
# boundaries (replay R, adjoint A) — parity per variant, then A/B at C3 fp32 and C5 bf16
set -u
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 AVSE_TIME_ALIGN_BYTES=128
for v in r406 a406 ra406 ra606 ra7ff; do
  AVSE_HIP_LIB=$PWD/expso/$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -k "scan" -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/t_$v.log 2>&1
  rc=$?; echo "$v: $(tail -1 gpurun_out/t_$v.log)"; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
done
bash tools/ab_scan.sh "base=expso/base.so r406=expso/r406.so a406=expso/a406.so ra406=expso/ra406.so ra606=expso/ra606.so ra7ff=expso/ra7ff.so" --cfg 64,1024,3999 --no-conv --pad || exit 1
bash tools/ab_scan.sh "base=expso/base.so ra406=expso/ra406.so ra606=expso/ra606.so ra7ff=expso/ra7ff.so" --cfg 32,1024,5999 --dtype bf16 --pad --no-conv || exit 1
