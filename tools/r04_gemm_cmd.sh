set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_projgemm.py tests/test_gpu_avmamba.py "tests/test_gpu_dropin.py::test_block_v2_dropins_under_bf16_autocast" > gpurun_out/pg_test.log 2>&1; rc=$?
tail -5 gpurun_out/pg_test.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/gemm_probe.py --reps 20 > gpurun_out/pg_probe.jsonl 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/pg_probe.jsonl | cut -c1-260
[ $rc -eq 0 ] || exit $rc
if [ "${1:-}" = bench ]; then
  for g in 1 0; do
    AVSE_PROJ_GEMM=$g timeout -k 10 300 python -u bench.py --workload avmamba --steps 4 --warmup 1 --no-cpu-baseline --no-roofline-hip > gpurun_out/pg_c5_$g.log 2>&1 || exit 1
    echo "PROJ_GEMM=$g $(grep -o '"value": [0-9.]*, "unit": "[^"]*", "n_gpus": 1, "steps": 4, "warmup": 1, "ms_per_step": [0-9.]*' gpurun_out/pg_c5_$g.log)"
  done
fi
