# round 6 (u): rocprofv3 kernel windows of the final tree: avse1 C2 timed window + roofline window, the C5 / C3 in-step
# windows (per-kernel time to pick the next target)
mkdir -p gpurun_out; export HSA_ENABLE_IPC_MODE_LEGACY=0
bash tools/profile_bench.sh gpurun_out/r06u_avse1 10; r=$?; echo "avse1 rc=$r"; [ $r -eq 0 ] || exit $r
MARK=roof bash tools/profile_bench.sh gpurun_out/r06u_c5 3 --workload avmamba --warmup 2; r=$?; echo "c5 rc=$r"; [ $r -eq 0 ] || exit $r
MARK=roof bash tools/profile_bench.sh gpurun_out/r06u_c3 3 --workload mamba --warmup 2; r=$?; echo "c3 rc=$r"; exit $r
