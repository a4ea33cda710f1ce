# correctness + probe of the experimental 16x16x32-MFMA GEMM build (expso/pg_m16.so from tools/pg_mfma16.patch)
mkdir -p gpurun_out
AVSE_HIP_LIB=expso/pg_m16.so timeout -k 10 120 python -u -m pytest -x -q --timeout 60 --timeout-method thread tests/test_gpu_projgemm.py > gpurun_out/pg_m16_test.log 2>&1 || { tail -30 gpurun_out/pg_m16_test.log; exit 1; }
echo "test m16: $(tail -1 gpurun_out/pg_m16_test.log)"
for v in base m16 base m16; do
  if [ $v = base ]; then lib=avse_challenge_amd/libavse_hip.so; else lib=expso/pg_$v.so; fi
  echo "== $v"
  AVSE_HIP_LIB=$lib timeout -k 10 120 python -u tools/gemm_probe.py --reps 10 --no-lib 2>&1 | grep '^{' | python -c "
import sys, json
for l in sys.stdin:
    d=json.loads(l); print(d['gemm'], d.get('hip_ms'), d.get('hip_frac'))
"
done
