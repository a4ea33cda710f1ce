# round 6: sconv weight gradient with 64 o x 32 i waves and a precomputed DMA plan: tests, old vs new
mkdir -p gpurun_out; export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests/test_gpu_sconv.py tests/test_gpu_kernels.py -v -m gpu --timeout 300 --timeout-method thread -k "sconv or trunk" > gpurun_out/r06j_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; grep -E "FAILED|ERROR|passed|failed" gpurun_out/r06j_tests.log | tail -6
[ $rc -eq 0 ] || exit $rc
for v in base new base new; do
  if [ $v = base ]; then lib=tools/variants/pre_sconvw_r06.so; else lib=avse_challenge_amd/libavse_hip.so; fi
  AVSE_HIP_LIB=$lib timeout -k 10 300 python -u tools/sconv_bench.py --no-miopen > gpurun_out/r06j_sbench_$v.log 2>&1; r=$?
  echo "bench $v rc=$r"; [ $r -eq 0 ] || exit $r
  python -c "
import json
for l in open('gpurun_out/r06j_sbench_$v.log'):
    if l.startswith('{'):
        r = json.loads(l); print('$v', r['shape'], 'wgrad', r['split_wgrad']['ms'], 'fwd', r['split_fwd']['ms'])"
done
for wl in avse4 mamba avmamba; do
  MARK=roof timeout -k 10 800 bash tools/profile_bench.sh gpurun_out/r06j_$wl 3 --workload $wl --warmup 2 --no-parity > gpurun_out/r06j_$wl.log 2>&1; r=$?
  echo "$wl rc=$r"; [ $r -eq 0 ] || exit $r
  head -14 gpurun_out/r06j_$wl/window_stats.csv | cut -c1-150
done
