#!/bin/bash
# PMC passes (one counter group per pass; gfx950 slot limits) over an arbitrary python command; per-kernel summary.
# usage: tools/pmc_cmd.sh OUTDIR script.py [args...]     (the script runs as `python script.py args...`)
set -u
out=$1; shift
mkdir -p "$out"
export TMPDIR=/tmp
i=0
PASSES=("SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"
        "TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_WR")
for grp in "${PASSES[@]}"; do
    i=$((i + 1))
    timeout -s KILL 180 rocprofv3 --pmc $grp --output-format csv -d "$out/p$i" -o run -- python "$@" > "$out/p$i.log" 2>&1 \
        || { echo "pass $i failed"; tail -3 "$out/p$i.log"; exit 1; }
done
python tools/pmc_summary.py "$out" > "$out/summary.txt"
cat "$out/summary.txt"
