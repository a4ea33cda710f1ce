#!/bin/bash
# Mamba C3 (B=64, captured) and C5 (B=32) bench lines with CPU baselines
set -u
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 500 python bench.py --workload avmamba --steps 5 --warmup 2 --no-roofline-hip > gpurun_out/bench_avmamba.log 2>&1; rc=$?
grep '^{' gpurun_out/bench_avmamba.log > gpurun_out/lines_r2h.jsonl; cut -c1-300 gpurun_out/lines_r2h.jsonl; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python bench.py --workload mamba --steps 4 --warmup 2 --no-roofline-hip > gpurun_out/bench_mamba.log 2>&1; rc=$?
grep '^{' gpurun_out/bench_mamba.log >> gpurun_out/lines_r2h.jsonl; tail -1 gpurun_out/lines_r2h.jsonl | cut -c1-300; exit $rc
