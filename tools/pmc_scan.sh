#!/bin/bash
# PMC passes over the scan / conv micro-bench (one counter group per pass; gfx950 slot limits).
# usage: tools/pmc_scan.sh OUTDIR [scan_bench args...]
set -u
out=$1; shift
root="${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p "$out"
export TMPDIR=/tmp
i=0
PASSES=("SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS"
        "FETCH_SIZE" "WRITE_SIZE" "SQ_INSTS_SALU SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES SQ_BUSY_CYCLES")
# PMC_PASSES="A B C;D E" replaces the passes (';' separates passes)
if [ -n "${PMC_PASSES:-}" ]; then IFS=';' read -r -a PASSES <<< "$PMC_PASSES"; fi
for grp in "${PASSES[@]}"; do
    i=$((i + 1))
    timeout -k 10 300 rocprofv3 --pmc $grp --output-format csv -d "$out/p$i" -o run -- \
        python "$root/tools/scan_bench.py" "$@" > "$out/p$i.log" 2>&1 || { echo "pass $i failed"; exit 1; }
done
python "$root/tools/pmc_summary.py" "$out" > "$out/summary.txt"
cat "$out/summary.txt"
