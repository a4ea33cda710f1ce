#!/bin/bash
# rocprofv3 kernel trace of bench.py's timed steps. usage: tools/profile_bench.sh OUTDIR STEPS [bench args...]
# Writes OUTDIR/{bench.log,window_stats.csv,post_window_stats.csv,roofline_window_stats.csv,run_kernel_stats.csv}
# (the big trace is deleted).  The bench runs with its roofline (avse1: 3 eager steps between markers 3 and 4) and
# without the CPU baseline / roofline_hip / secondary configs.  MARK=roof: the markers bracket the last eager warm-up
# step instead (the in-step roofline of the C3 / C4 / C5 workloads), whose summary is then window_stats.csv.
set -u
out=$1; steps=$2; shift 2
root="${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p "$out"
cd "$out" || exit 1
export TMPDIR=/tmp AVSE_PROFILE_MARK=${MARK:-1}
timeout -k 10 700 rocprofv3 --kernel-trace --stats --output-format csv -d . -o run -- \
    python "$root/bench.py" --steps "$steps" --no-cpu-baseline --no-roofline-hip --secondary "" "$@" > bench.log 2>&1
rc=$?
[ $rc -eq 0 ] && python "$root/tools/ktrace_window.py" run_kernel_trace.csv "$steps" window_stats.csv \
    post_window_stats.csv roofline_window_stats.csv
rm -f run_kernel_trace.csv
grep metric bench.log | cut -c1-220
exit $rc
