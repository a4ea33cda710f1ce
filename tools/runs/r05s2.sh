# which split-fp16 operand splits still run an absmax pass in one eager C3 / C4 step (tools/split_sites.py)
mkdir -p gpurun_out; export HSA_ENABLE_IPC_MODE_LEGACY=0
for w in mamba avse4; do
  timeout -k 10 300 python -u tools/split_sites.py $w > gpurun_out/r05s2_$w.log 2>&1 || { echo "$w failed"; tail -5 gpurun_out/r05s2_$w.log; exit 1; }
  echo "== $w"; cat gpurun_out/r05s2_$w.log | grep -v Warning | tail -30
done
