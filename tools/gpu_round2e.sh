#!/bin/bash
# step-level benches of the Mamba workloads (C3, C5) with the scan v3 kernels (+ their CPU baselines)
set -u
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 420 python bench.py --workload mamba --steps 4 --warmup 2 --no-roofline-hip > gpurun_out/bench_mamba.log 2>&1; rc=$?
grep '^{' gpurun_out/bench_mamba.log | cut -c1-400; [ $rc -eq 0 ] || exit $rc
timeout -k 10 420 python bench.py --workload avmamba --steps 4 --warmup 2 --no-roofline-hip > gpurun_out/bench_avmamba.log 2>&1; rc=$?
grep '^{' gpurun_out/bench_avmamba.log | cut -c1-400; exit $rc
