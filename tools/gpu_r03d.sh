#!/bin/bash
# scan forward layouts A/B at C3 (fp32) and C5 (bf16) + the scan tests
set -u
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_kernels.py -k "scan" > gpurun_out/r03d_scan_tests.log 2>&1 || { tail -30 gpurun_out/r03d_scan_tests.log; exit 1; }
tail -2 gpurun_out/r03d_scan_tests.log
for g in 4 2; do
  AVSE_SCAN_G=$g timeout -k 10 200 python -u tools/scan_bench.py --cfg 64,1024,3999 --pad --no-conv > gpurun_out/r03d_g$g.log 2>&1 || exit 1
  AVSE_SCAN_G=$g timeout -k 10 200 python -u tools/scan_bench.py --cfg 32,1024,5999 --dtype bf16 --pad --no-conv > gpurun_out/r03d_g${g}_bf16.log 2>&1 || exit 1
  echo "G=$g"; grep cfg gpurun_out/r03d_g$g.log gpurun_out/r03d_g${g}_bf16.log
done
