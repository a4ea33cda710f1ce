set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_projgemm.py > gpurun_out/pg_test.log 2>&1; rc=$?
tail -5 gpurun_out/pg_test.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/gemm_probe.py --reps 20 > gpurun_out/pg_probe.jsonl 2>&1; rc=$?
cat gpurun_out/pg_probe.jsonl
exit $rc
