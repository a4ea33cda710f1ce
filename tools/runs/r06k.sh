# round 6 (k): the stride-2 trunk input gradient on csrc/sconv.hip (avse_sconv_dgrad2): its tests, its rate vs MIOpen
# at the C2 lip-trunk shapes, every -m gpu test, the C2 line without secondaries
mkdir -p gpurun_out; export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests/test_gpu_sconv.py -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/r06k_sconv_tests.log 2>&1; rc=$?
echo "sconv tests rc=$rc"; grep -E "FAILED|ERROR|passed|failed|dgrad2" gpurun_out/r06k_sconv_tests.log | tail -20
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/sconv_bench.py > gpurun_out/r06k_sconv_bench.log 2>&1; r=$?
echo "sconv bench rc=$r"; [ $r -eq 0 ] || exit $r
python -c "
import json
for l in open('gpurun_out/r06k_sconv_bench.log'):
    if l.startswith('{'):
        r = json.loads(l); print(r['shape'], 'fwd', r['split_fwd']['ms'], 'dgrad', r['split_dgrad']['ms'], r['split_dgrad']['frac_f16x3'], 'miopen dgrad', r['miopen_dgrad']['ms'], 'wgrad', r['split_wgrad']['ms'])"
timeout -k 10 1000 python -u -m pytest tests -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/r06k_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; grep -E "FAILED|ERROR|passed|failed" gpurun_out/r06k_tests.log | tail -12
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py --steps 10 --warmup 2 --secondary "" --no-cpu-baseline --no-roofline-hip --no-parity > gpurun_out/r06k_c2.log 2>&1; r=$?
echo "c2 rc=$r"; grep '^{' gpurun_out/r06k_c2.log | tail -1 | python -c "import json,sys; r=json.loads(sys.stdin.read()); ro=r['roofline']; print(r['value'], r['ms_per_step'], ro['kernel'][:20], ro['avg_ms'], ro['frac'], ro['in_step_serial'])"
exit $r
