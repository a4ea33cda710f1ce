# round 6 (z): the lip-shortcut input gradient on the split GEMM: its tests, the avse1 / avse4 model tests, the step's
# remaining library GEMMs, C2 and C4 lines (r06t: C2 440.1, C4 186.4 utt/s)
mkdir -p gpurun_out; export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 700 python -u -m pytest tests -k "pointwise or avse1 or avse4 or trunk or aonly or fullsize" -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/r06z_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; grep -E "FAILED|ERROR|passed|failed" gpurun_out/r06z_tests.log | tail -6
[ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python -u tools/avse1_op_profile.py --kernels "Cijk/gemm_kernel/planes_" --top 30 > gpurun_out/r06z_avse1_ops.log 2>&1; r=$?
echo "op profile rc=$r"; grep -v "^alive" gpurun_out/r06z_avse1_ops.log | grep -E "ms|kernels matching" | cut -c1-240 | head -80
[ $r -eq 0 ] || exit $r
timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 --secondary "" --no-cpu-baseline --no-roofline-hip --no-parity > gpurun_out/r06z_c2.log 2>&1; r=$?
echo "c2 rc=$r"; grep '^{' gpurun_out/r06z_c2.log | tail -1 | cut -c1-200
[ $r -eq 0 ] || exit $r
timeout -k 10 400 python -u bench.py --workload avse4 --steps 6 --warmup 2 --no-cpu-baseline --no-roofline-hip --no-parity > gpurun_out/r06z_c4.log 2>&1; r=$?
echo "c4 rc=$r"; grep '^{' gpurun_out/r06z_c4.log | tail -1 | cut -c1-200
[ $r -eq 0 ] || exit $r
timeout -k 10 500 python -u tools/avse1_op_profile.py --workload avmamba --kernels "copy_kernel/Cijk" --top 25 > gpurun_out/r06z_c5_ops.log 2>&1; r=$?
echo "c5 op profile rc=$r"; grep -v "^alive" gpurun_out/r06z_c5_ops.log | grep -E "ms|kernels matching" | cut -c1-230 | head -50
exit $r
