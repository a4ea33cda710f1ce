#!/bin/bash
# rocprofv3 kernel trace + stats of the DEFAULT bench command (roofline, roofline_hip and cpu_baseline included).
# usage: tools/profile_bench_full.sh OUTDIR STEPS [bench args...]
# Writes OUTDIR/{bench.log, run_kernel_stats.csv (whole run), window_stats.csv (timed steps),
# post_window_stats.csv (the isolated roofline measurements after the timed steps)}; the big trace is deleted.
set -u
out=$1; steps=$2; shift 2
root="${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p "$out"
cd "$out" || exit 1
export TMPDIR=/tmp AVSE_PROFILE_MARK=1
timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d . -o run -- \
    python "$root/bench.py" --steps "$steps" "$@" > bench.log 2>&1
rc=$?
[ $rc -eq 0 ] && python "$root/tools/ktrace_window.py" run_kernel_trace.csv "$steps" window_stats.csv post_window_stats.csv
rm -f run_kernel_trace.csv
grep metric bench.log | cut -c1-220
exit $rc
