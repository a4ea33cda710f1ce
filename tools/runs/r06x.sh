# round 6 (x) = (v) + (w) in one call: the avse1 LSTM GEMMs one by one and the per-sequence dw_hh (avse1 tests, C2
# line); the x_proj input gradient on csrc/lowrank.hip (its tests, the Mamba model tests, C3 / C5 lines; A/B against
# r06t: C2 440.1, C3 68.66, C5 59.82 utt/s)
mkdir -p gpurun_out; export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 120 python -u tools/lstm_gemm_probe.py > gpurun_out/r06x_lstm_gemm.jsonl 2>&1; r=$?; cat gpurun_out/r06x_lstm_gemm.jsonl; [ $r -eq 0 ] || exit $r
timeout -k 10 900 python -u -m pytest tests -k "lowrank or lstm or avse1 or fusion or aonly or mamba or avmamba or dpmamba or bimamba or masknet or dropin or encdec or fullsize" -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/r06x_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; grep -E "FAILED|ERROR|passed|failed" gpurun_out/r06x_tests.log | tail -6
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 --secondary "" --no-cpu-baseline --no-roofline-hip --no-parity > gpurun_out/r06x_c2.log 2>&1; r=$?
echo "c2 rc=$r"; grep '^{' gpurun_out/r06x_c2.log | tail -1 | cut -c1-200
[ $r -eq 0 ] || exit $r
for w in mamba avmamba; do
  timeout -k 10 400 python -u bench.py --workload $w --steps 4 --warmup 1 --no-cpu-baseline --no-roofline-hip --no-parity > gpurun_out/r06x_$w.log 2>&1; r=$?
  echo "$w rc=$r"; grep '^{' gpurun_out/r06x_$w.log | tail -1 | cut -c1-260
  [ $r -eq 0 ] || exit $r
done
