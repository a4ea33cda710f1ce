#!/bin/bash
# round-2 final: the round-end checks (GPU suite, smoke, bench) and the rocprofv3 stats of the default bench
set -u
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
bash tools/gpu_check.sh || exit $?
bash tools/profile_bench_full.sh "$PWD/gpurun_out/prof_r02d" 10 || exit 1
