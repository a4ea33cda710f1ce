# round 6 (m): the avse1 TCN weight / input gradients and the lip-shortcut weight gradients on the split GEMM
# (avse_gemm_f32s): their tests, the step's remaining library GEMMs, the C2 line
mkdir -p gpurun_out; export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests/test_gpu_projgemm.py tests/test_gpu_kernels.py -k "f32s or rows_tn or time_conv1d or pointwise or convf or trunk or conv1" -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/r06m_pg_tests.log 2>&1; rc=$?
echo "projgemm tests rc=$rc"; grep -E "FAILED|ERROR|passed|failed|rows_tn" gpurun_out/r06m_pg_tests.log | tail -12
[ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python -u tools/avse1_op_profile.py --kernels "Cijk/gemm_kernel/igemm/cvf::" --top 30 > gpurun_out/r06m_avse1_ops.log 2>&1; r=$?
echo "op profile rc=$r"; grep -v "^alive" gpurun_out/r06m_avse1_ops.log | grep -E "ms|kernels matching" | cut -c1-200 | head -60
[ $r -eq 0 ] || exit $r
timeout -k 10 400 python -u bench.py --steps 10 --warmup 2 --secondary "" --no-cpu-baseline --no-roofline-hip --no-parity > gpurun_out/r06m_c2.log 2>&1; r=$?
echo "c2 rc=$r"; grep '^{' gpurun_out/r06m_c2.log | tail -1 | python -c "import json,sys; r=json.loads(sys.stdin.read()); ro=r['roofline']; print(r['value'], r['ms_per_step'], ro['kernel'][:20], ro['avg_ms'], ro['frac'], ro['in_step_serial'])"
exit $r
