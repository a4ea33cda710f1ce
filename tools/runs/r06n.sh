# round 6: lip Conv3d fp32 frames on the split-fp16 MFMA (forward and weight gradient): tests, bench, C4 / C5 steps
mkdir -p gpurun_out; export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_models.py tests/test_gpu_avmamba.py -v -m gpu --timeout 300 --timeout-method thread -k "avse4_full_train_step_vs_oracle" > gpurun_out/r06n_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; grep -E "FAILED|ERROR|passed|failed" gpurun_out/r06n_tests.log | tail -8
grep -E "of sum\|terms\|" gpurun_out/r06n_tests.log | head -20
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/conv3d_bench.py --avse4 > gpurun_out/r06n_c3bench4.log 2>&1 || exit 1
grep '^{' gpurun_out/r06n_c3bench4.log
timeout -k 10 300 python -u tools/conv3d_bench.py --no-miopen > gpurun_out/r06n_c3bench1.log 2>&1 || exit 1
grep '^{' gpurun_out/r06n_c3bench1.log
timeout -k 10 600 python -u bench.py --workload avse4 --steps 6 --warmup 2 --secondary "" --no-cpu-baseline --no-roofline-hip > gpurun_out/r06n_c4.log 2>&1; r=$?
echo "c4 rc=$r"; grep '^{' gpurun_out/r06n_c4.log | tail -1 | cut -c1-400
[ $r -eq 0 ] || exit $r
timeout -k 10 600 python -u bench.py --workload avmamba --steps 4 --warmup 2 --secondary "" --no-cpu-baseline --no-roofline-hip --no-parity > gpurun_out/r06n_c5.log 2>&1; r=$?
echo "c5 rc=$r"; grep '^{' gpurun_out/r06n_c5.log | tail -1 | cut -c1-300
exit $r
