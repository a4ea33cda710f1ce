#!/bin/bash
# A/B the scan kernels of several builds: tools/ab_scan.sh "NAME=LIB ..." [scan_bench args]
# (main = the in-tree library); prints fwd/bwd ms per config for each build.
set -u
libs=$1; shift
mkdir -p gpurun_out
for spec in $libs; do
  n=${spec%%=*}; lib=${spec#*=}
  AVSE_HIP_LIB=$PWD/$lib timeout -k 10 200 python tools/scan_bench.py "$@" > gpurun_out/ab_$n.log 2>&1 || { echo "$n failed"; tail -5 gpurun_out/ab_$n.log; exit 1; }
  echo "== $n"
  grep cfg gpurun_out/ab_$n.log | python -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); print(d['cfg'], {k: v['ms'] for k, v in d.items() if k.startswith('scan')})"
done
