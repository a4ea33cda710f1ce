# Full GPU validation of the tree on one MI355X: every -m gpu test, smoke(), the default bench line, PMC traffic of
# the fused dwconv/gLN backward.  usage (from the repo root, through gpurun): bash tools/gpu_validate.sh
mkdir -p gpurun_out; export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/validate_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; grep -E "FAILED|ERROR|passed|failed" gpurun_out/validate_tests.log | tail -8
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/validate_smoke.log 2>&1; rc=$?; echo "smoke rc=$rc"; grep smoke gpurun_out/validate_smoke.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 900 python -u bench.py > gpurun_out/validate_bench.log 2>&1; rc=$?; echo "bench rc=$rc"; grep '^{' gpurun_out/validate_bench.log | tail -1 | cut -c1-1500
[ $rc -eq 0 ] || exit 1
PHASES="cconv dwconv_gln dwconv_gln_bwd" bash tools/pmc_traffic.sh gpurun_out/validate_pmc gpurun_out/validate_traffic.json > gpurun_out/validate_pmc.log 2>&1; echo "pmc rc=$?"; tail -3 gpurun_out/validate_pmc.log
