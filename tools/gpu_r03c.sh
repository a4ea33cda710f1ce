#!/bin/bash
# avse1 train-step tests against the masked fp64 oracle (incl. the benchmarked graph step), then scan fwd PMC A/B
set -u
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 500 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread tests/test_gpu_models.py -k "avse1_bench_step" > gpurun_out/r03c_avse1_tests.log 2>&1; rc=$?
grep -E "PASS|FAIL|Error|error|avse1 grads|passed|failed" gpurun_out/r03c_avse1_tests.log | tail -30
[ $rc -eq 0 ] || exit $rc
bash tools/gpu_r03b.sh
