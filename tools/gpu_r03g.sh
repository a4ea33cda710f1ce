#!/bin/bash
# avse1 model tests (masked-oracle parity incl. the benchmarked graph step) + the default bench line
set -u
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
tag=${1:-r03g}
timeout -k 10 500 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread tests/test_gpu_models.py -k "avse1" > gpurun_out/${tag}_avse1_tests.log 2>&1; rc=$?
grep -E "avse1 grads|passed|failed|FAILED" gpurun_out/${tag}_avse1_tests.log | tail -12
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 > gpurun_out/${tag}_bench.log 2>&1; rc=$?
grep '^{' gpurun_out/${tag}_bench.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print({k: d[k] for k in ('value','ms_per_step')}, d['roofline'], d.get('cpu_baseline',{}).get('value'))"
exit $rc
