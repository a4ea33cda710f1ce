#!/bin/bash
# Round measurement on one MI355X: the bench line of every workload + the rocprofv3 kernel-trace
# stats of the default bench command.  usage: tools/round_bench.sh TAG   (outputs gpurun_out/TAG/)
set -u
tag=$1
root="${GRAFT_REPO_ROOT:-$(pwd)}"
out="$root/gpurun_out/$tag"
mkdir -p "$out"
export HSA_ENABLE_IPC_MODE_LEGACY=0
for w in avse1 mamba avse4; do
  timeout -k 10 600 python "$root/bench.py" --workload $w --steps 10 --warmup 3 > "$out/bench_$w.log" 2>&1
  rc=$?; grep '"metric"' "$out/bench_$w.log" | cut -c1-400; [ $rc -eq 0 ] || { echo "bench $w rc=$rc"; tail -5 "$out/bench_$w.log"; exit $rc; }
done
bash "$root/tools/profile_bench.sh" "$out/prof_avse1" 5 --workload avse1 || exit 1
python "$root/tools/kstats.py" "$out/prof_avse1/window_stats.csv" 5 40 > "$out/prof_avse1/window_stats.txt" 2>/dev/null || true
