# round 6: Conv3d wgrad ring without per-pair divisions, one resident round; scan forward out_z accumulate (C5)
mkdir -p gpurun_out; export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 900 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_models.py tests/test_gpu_avmamba.py -v -m gpu --timeout 300 --timeout-method thread -k "conv3d or lip or avse4 or frontend or avmamba or scan or mamba or cconv or dropin" > gpurun_out/r06q_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; grep -E "FAILED|ERROR|passed|failed" gpurun_out/r06q_tests.log | tail -8
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/conv3d_bench.py --avse4 > gpurun_out/r06q_c3bench4.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/conv3d_bench.py --no-miopen > gpurun_out/r06q_c3bench1.log 2>&1 || exit 1
grep '^{' gpurun_out/r06q_c3bench4.log gpurun_out/r06q_c3bench1.log | cut -c1-420
timeout -k 10 600 python -u bench.py --workload avmamba --steps 4 --warmup 2 --secondary "" --no-cpu-baseline --no-roofline-hip > gpurun_out/r06q_c5.log 2>&1; r=$?
echo "c5 rc=$r"; grep '^{' gpurun_out/r06q_c5.log | tail -1 | python -c "
import json,sys; r=json.loads(sys.stdin.read()); print(r['value'], r['ms_per_step'], json.dumps(r.get('parity'))[:300]); print(json.dumps(r['roofline'])[:600])"
exit $r
