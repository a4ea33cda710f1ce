#!/bin/bash
# Bench lines of the §8f / C5 workloads (DPMamba-L, AV Mamba-TasNet-L bf16, avse2) + the C5 kernel-trace window.
# usage: tools/round_bench_more.sh TAG   (outputs gpurun_out/TAG/)
set -u
tag=$1
root="${GRAFT_REPO_ROOT:-$(pwd)}"
out="$root/gpurun_out/$tag"
mkdir -p "$out"
export HSA_ENABLE_IPC_MODE_LEGACY=0
for w in dpmamba avmamba avse2; do
  timeout -k 10 600 python "$root/bench.py" --workload $w --steps 5 --warmup 2 > "$out/bench_$w.log" 2>&1
  rc=$?; grep '"metric"' "$out/bench_$w.log" | cut -c1-400; [ $rc -eq 0 ] || { echo "bench $w rc=$rc"; tail -5 "$out/bench_$w.log"; exit $rc; }
done
bash "$root/tools/profile_bench.sh" "$out/prof_avmamba" 3 --workload avmamba || exit 1
python "$root/tools/kstats.py" "$out/prof_avmamba/window_stats.csv" 3 40 > "$out/prof_avmamba/window_stats.txt" 2>/dev/null || true
