# dist masked test repeated (split-output BatchNorm on / off) + the bnact flag diagnostic
mkdir -p gpurun_out; export HSA_ENABLE_IPC_MODE_LEGACY=0
for i in 1 2 3; do
  timeout -k 10 300 python -u -m pytest tests/test_gpu_dist.py -x -v -s -m gpu --timeout 280 -k "avse1" > gpurun_out/r05z2_dist_q1_$i.log 2>&1; echo "q1 run $i rc=$?"; grep -E "total rel err" gpurun_out/r05z2_dist_q1_$i.log
done
for i in 1 2; do
  AVSE_BNACT_Q=0 timeout -k 10 300 python -u -m pytest tests/test_gpu_dist.py -x -v -s -m gpu --timeout 280 -k "avse1" > gpurun_out/r05z2_dist_q0_$i.log 2>&1; echo "q0 run $i rc=$?"; grep -E "total rel err" gpurun_out/r05z2_dist_q0_$i.log
done
timeout -k 10 200 python tools/bnact_q_check.py > gpurun_out/r05z2_flags.log 2>&1; echo "flags rc=$?"; grep '"fwd"' gpurun_out/r05z2_flags.log | head -30
