#!/bin/bash
# trunk conv weight-gradient kernel: tests + HIP vs MIOpen at the avse1 C2 trunk shapes
set -u
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_kernels.py -k "rconv or trunk or dconv or dilated" > gpurun_out/r03h_tests.log 2>&1 || { tail -40 gpurun_out/r03h_tests.log; exit 1; }
tail -2 gpurun_out/r03h_tests.log
timeout -k 10 400 python -u tools/rconv_bench.py > gpurun_out/r03h_bench.log 2>&1; rc=$?
grep cin gpurun_out/r03h_bench.log; exit $rc
