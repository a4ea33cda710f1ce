#!/bin/bash
# GPU-box round check: parity tests, smoke, short bench. Stops at the first GPU-level failure
# (timeout / abort / segfault); a plain test failure (pytest rc 1) still lets smoke + bench run.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 1100 python -u -m pytest tests -m gpu -q -rf --timeout 400 --timeout-method thread -p no:cacheprovider "$@" > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/pytest_gpu.log
tail -5 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; tail -3 gpurun_out/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python bench.py --steps 5 --warmup 2 > gpurun_out/bench.log 2>&1
rc=$?; tail -3 gpurun_out/bench.log; exit $rc
