#!/bin/bash
# HIP graph packet capture off (package default) vs on: avse1 stream test, avse1 / mamba / avmamba step rate
set -u
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u -m pytest tests/test_gpu_models.py -k "branch_streams or graph or bimamba_direction" -v --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/t11.log 2>&1
rc=$?; grep -E "PASSED|FAILED" gpurun_out/t11.log | cut -c1-120; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for pc in 0 1; do
  for w in avse1 avmamba; do
    DEBUG_CLR_GRAPH_PACKET_CAPTURE=$pc timeout -k 10 300 python bench.py --workload $w --steps 8 --warmup 3 --no-roofline-hip --no-cpu-baseline --no-roofline > gpurun_out/bench_${w}_pc$pc.log 2>&1; rc=$?
    echo "packet_capture=$pc $w: $(grep '^{' gpurun_out/bench_${w}_pc$pc.log | cut -c60-150)"; [ $rc -eq 0 ] || exit $rc
  done
done
