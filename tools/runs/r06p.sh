# round 6: lip Conv3d weight gradient as a sliding window over output rows (ring of staged input rows): tests, bench, steps
mkdir -p gpurun_out; export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 900 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_models.py tests/test_gpu_avmamba.py -v -m gpu --timeout 300 --timeout-method thread -k "conv3d or lip or avse4 or avse1 or frontend or avmamba" > gpurun_out/r06p_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; grep -E "FAILED|ERROR|passed|failed" gpurun_out/r06p_tests.log | tail -8
grep -E "of sum\|terms\|" gpurun_out/r06p_tests.log | head -20
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/conv3d_bench.py --avse4 > gpurun_out/r06p_c3bench4.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/conv3d_bench.py --no-miopen > gpurun_out/r06p_c3bench1.log 2>&1 || exit 1
grep '^{' gpurun_out/r06p_c3bench4.log gpurun_out/r06p_c3bench1.log | cut -c1-420
timeout -k 10 400 python -u bench.py --steps 10 --warmup 2 --secondary "" --no-cpu-baseline --no-roofline-hip --no-parity > gpurun_out/r06p_c2.log 2>&1; r=$?
echo "c2 rc=$r"; grep '^{' gpurun_out/r06p_c2.log | tail -1 | cut -c1-250
[ $r -eq 0 ] || exit $r
timeout -k 10 600 python -u bench.py --workload avse4 --steps 6 --warmup 2 --secondary "" --no-cpu-baseline --no-roofline-hip > gpurun_out/r06p_c4.log 2>&1; r=$?
echo "c4 rc=$r"; grep '^{' gpurun_out/r06p_c4.log | tail -1 | python -c "
import json,sys; r=json.loads(sys.stdin.read()); ro=r['roofline']; print(r['value'], r['ms_per_step']); print(json.dumps(ro)[:1500])"
exit $r
