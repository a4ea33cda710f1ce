#!/bin/bash
# One GPU session as a list of steps, each under its own time limit, stopping at the first failure (gpurun rules: no
# retries, nothing more on the GPU after a fault / abort / timeout).  Logs: gpurun_out/<tag>_<n>_<kind>.log.
#
# usage (on the box, via gpurun):  bash tools/gpu_steps.sh TAG STEP [STEP ...]
#   test:EXPR          python -m pytest tests -m gpu -x -v -k "EXPR"   (EXPR "all": every GPU test, then smoke())
#   bench:ARGS         python bench.py ARGS   (ARGS comma-separated, e.g. bench:--workload,mamba,--steps,10)
#   tool:SCRIPT,ARGS   python tools/SCRIPT ARGS (comma-separated)
#   pmc:PASSES,ARGS    tools/pmc_scan.sh over tools/scan_bench.py ARGS with PMC_PASSES (';' between passes)
# env: STEP_TIMEOUT (seconds per step, default 600)
set -u
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
tag=$1; shift
lim=${STEP_TIMEOUT:-600}
n=0
for step in "$@"; do
    n=$((n + 1))
    kind=${step%%:*}; arg=${step#*:}
    log=gpurun_out/${tag}_${n}_${kind}.log
    echo "== step $n: $step"
    case $kind in
        test)
            if [ "$arg" = "all" ]; then
                timeout -k 10 "$lim" python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > "$log" 2>&1 \
                    && timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" >> "$log" 2>&1
            else
                timeout -k 10 "$lim" python -u -m pytest tests -x -v -s -m gpu -k "$arg" --timeout 300 --timeout-method thread > "$log" 2>&1
            fi
            rc=$?
            grep -E "FAILED|ERROR|passed|failed|smoke ok|avse1 grads|rank .* rel err" "$log" | tail -15 ;;
        bench)
            timeout -k 10 "$lim" python -u bench.py ${arg//,/ } > "$log" 2>&1; rc=$?
            grep '^{' "$log" | tail -1 | cut -c1-1500 ;;
        tool)
            script=${arg%%,*}; rest=""; [ "$arg" != "$script" ] && rest=${arg#*,}
            timeout -k 10 "$lim" python -u "tools/$script" ${rest//,/ } > "$log" 2>&1; rc=$?
            grep -v -e amdgpu.ids -e "MIOpen(HIP): Warning" "$log" | tail -25 ;;
        pmc)
            passes=${arg%%,*}; rest=""; [ "$arg" != "$passes" ] && rest=${arg#*,}
            PMC_PASSES="$passes" timeout -k 10 "$lim" bash tools/pmc_scan.sh "gpurun_out/${tag}_${n}_pmc" ${rest//,/ } > "$log" 2>&1; rc=$?
            tail -40 "$log" ;;
        *) echo "unknown step kind: $kind"; exit 2 ;;
    esac
    if [ $rc -ne 0 ]; then echo "step $n failed (rc $rc): $log"; tail -30 "$log"; exit $rc; fi
done
