#!/bin/bash
# round 2 session 3 close-out: the two re-floored tests, rocprofv3 stats of the default bench command, and the
# Mamba-L C3 / C5 bench lines with the backward's lam*dA reuse
set -u
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u -m pytest tests/test_gpu_avmamba.py "tests/test_gpu_models.py::test_avse4_full_train_step_vs_oracle" -q -rf --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/t_close.log 2>&1
rc=$?; tail -2 gpurun_out/t_close.log; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
bash tools/profile_bench_full.sh "$PWD/gpurun_out/prof_r02c" 10 || exit 1
for w in mamba avmamba; do
  timeout -k 10 600 python bench.py --workload $w --steps 5 --warmup 2 --no-roofline-hip > gpurun_out/bench_r02c_$w.log 2>&1; rc=$?
  echo "$w rc=$rc: $(grep '^{' gpurun_out/bench_r02c_$w.log | cut -c1-160)"; [ $rc -eq 0 ] || exit $rc
done
