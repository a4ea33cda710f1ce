# round 6 (y): lowrank vs baddbmm in isolation; the avse1 step's library GEMM launches with their call sites
mkdir -p gpurun_out; export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 120 python -u tools/lowrank_bench.py > gpurun_out/r06y_lowrank.jsonl 2>&1; r=$?; cat gpurun_out/r06y_lowrank.jsonl; [ $r -eq 0 ] || exit $r
timeout -k 10 500 python -u tools/avse1_op_profile.py --kernels "Cijk" --top 30 > gpurun_out/r06y_avse1_ops.log 2>&1; r=$?
echo "op profile rc=$r"; grep -v "^alive" gpurun_out/r06y_avse1_ops.log | grep -E "ms|kernels matching" | cut -c1-260 | head -40
exit $r
