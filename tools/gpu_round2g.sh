#!/bin/bash
# Mamba-L C3 B=64: eager (2 streams) vs captured (1 stream); C5 avmamba default
set -u
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python bench.py --workload mamba --steps 4 --warmup 2 --no-roofline-hip --no-cpu-baseline --no-graph > gpurun_out/bench_mamba_eager.log 2>&1; rc=$?
grep '^{' gpurun_out/bench_mamba_eager.log | cut -c1-200; grep -o '"hip_graph[^}]*' gpurun_out/bench_mamba_eager.log; [ $rc -eq 0 ] || exit $rc
AVSE_BIMAMBA_STREAMS=0 timeout -k 10 300 python bench.py --workload mamba --steps 4 --warmup 2 --no-roofline-hip --no-cpu-baseline > gpurun_out/bench_mamba_graph1s.log 2>&1; rc=$?
grep '^{' gpurun_out/bench_mamba_graph1s.log | cut -c1-200; grep -o '"hip_graph[^}]*' gpurun_out/bench_mamba_graph1s.log; grep "capture failed" gpurun_out/bench_mamba_graph1s.log | cut -c1-100
timeout -k 10 420 python bench.py --workload avmamba --steps 4 --warmup 2 --no-roofline-hip > gpurun_out/bench_avmamba.log 2>&1; rc=$?
grep '^{' gpurun_out/bench_avmamba.log | cut -c1-200; grep -o '"hip_graph[^}]*' gpurun_out/bench_avmamba.log; grep -o '"cpu_baseline.*' gpurun_out/bench_avmamba.log; exit $rc
