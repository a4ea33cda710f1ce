#!/bin/bash
# HBM traffic per launch of the bench's roofline kernels from rocprofv3 PMC passes (one counter per
# pass: FETCH_SIZE needs 3 TCC slots, WRITE_SIZE 2 — MI355X_MICROARCH.md 'rocprofv3 PMC slots').
# usage: tools/pmc_traffic.sh OUTDIR [JSON_OUT]   -> JSON_OUT (default OUTDIR/traffic.json)
set -u
out=$1; json=${2:-$1/traffic.json}
root="${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p "$out"
export TMPDIR=/tmp
for ph in ${PHASES:-cconv scan scan_bwd scan_c5 scan_bwd_c5 dwconv dwconv_gln dwconv_gln_bwd prelu_gln prelu_gln_bwd dconv_wgrad}; do
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 240 rocprofv3 --pmc $c --output-format csv -d "$out/$ph/$c" -o run -- \
        python "$root/tools/roofline_kernels.py" $ph > "$out/$ph.$c.log" 2>&1 || { echo "$ph $c failed"; tail -3 "$out/$ph.$c.log"; exit 1; }
  done
done
python "$root/tools/traffic_summary.py" "$out" > "$json" && cat "$json"
