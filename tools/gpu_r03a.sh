#!/bin/bash
# round 3 session 1: avse1 per-site gradient diagnosis, new GPU tests, scan forward layout A/B
set -u
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
T="timeout -k 10"
$T 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_kernels.py -k "scan or lstm" > gpurun_out/r03a_scan_tests.log 2>&1 || { tail -30 gpurun_out/r03a_scan_tests.log; exit 1; }
tail -3 gpurun_out/r03a_scan_tests.log
for g in 4 2; do AVSE_SCAN_G=$g $T 200 python -u tools/scan_bench.py --cfg 64,1024,3999 --pad --no-conv > gpurun_out/r03a_scanbench_g$g.log 2>&1 || { tail -20 gpurun_out/r03a_scanbench_g$g.log; exit 1; }; grep -v amdgpu.ids gpurun_out/r03a_scanbench_g$g.log | tail -4; done
$T 400 python -u tools/avse1_site_diag.py cl > gpurun_out/site_diag_cl.log 2>&1 || { tail -30 gpurun_out/site_diag_cl.log; exit 1; }
grep -v -e amdgpu.ids -e MIOpen gpurun_out/site_diag_cl.log | tail -50
$T 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_dist.py > gpurun_out/r03a_dist_test.log 2>&1; rc=$?
tail -5 gpurun_out/r03a_dist_test.log
exit $rc
