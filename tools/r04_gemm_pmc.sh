set -o pipefail
mkdir -p gpurun_out
for v in base bk64 n3 n5; do
  if [ $v = base ]; then lib=avse_challenge_amd/libavse_hip.so; else lib=expso/pg_$v.so; fi
  AVSE_HIP_LIB=$lib timeout -k 10 120 python -u -m pytest -x -q --timeout 60 --timeout-method thread tests/test_gpu_projgemm.py > gpurun_out/pg_test_$v.log 2>&1 || { echo "test $v failed"; tail -20 gpurun_out/pg_test_$v.log; exit 1; }
  echo "test $v: $(tail -1 gpurun_out/pg_test_$v.log)"
done
bash tools/r04_gemm_abl.sh && bash tools/pmc_gemm.sh gpurun_out/pmc_inproj2 --case "in_proj fwd"
