#!/bin/bash
# the default bench command under rocprofv3 (kernel trace + stats): per-kernel averages to check the bench line's
# live roofline / roofline_hip timings against
set -u
root="${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p "$root/gpurun_out/prof_default"
cd "$root/gpurun_out/prof_default" || exit 1
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 700 rocprofv3 --kernel-trace --stats --output-format csv -d . -o run -- python3 "$root/bench.py" --steps 5 --warmup 2 > bench.log 2>&1
rc=$?
grep '^{' bench.log | cut -c1-300
rm -f run_kernel_trace.csv
ls
exit $rc
