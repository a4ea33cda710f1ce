set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 python -u -m pytest -x -q --timeout 60 --timeout-method thread tests/test_gpu_projgemm.py > gpurun_out/pg_test.log 2>&1 || { tail -20 gpurun_out/pg_test.log; exit 1; }
echo "test: $(tail -1 gpurun_out/pg_test.log)"
bash tools/r04_gemm_abl.sh
