#!/bin/bash
# the round-end checks as the driver runs them: every GPU test (-x), then smoke()
set -u
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
tag=${1:-full}
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/${tag}_pytest_gpu.log 2>&1; rc=$?
grep -E "FAILED|ERROR|passed|failed" gpurun_out/${tag}_pytest_gpu.log | tail -8
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${tag}_smoke.log 2>&1; rc=$?
tail -2 gpurun_out/${tag}_smoke.log
exit $rc
