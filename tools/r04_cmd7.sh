# PMC traffic of the roofline kernels (current tree) + rocprofv3 kernel-trace window of the default bench
mkdir -p gpurun_out; export HSA_ENABLE_IPC_MODE_LEGACY=0
bash tools/pmc_traffic.sh gpurun_out/r04_pmc gpurun_out/r04_traffic.json > gpurun_out/r04_pmc.log 2>&1; echo "pmc rc=$?"; tail -5 gpurun_out/r04_pmc.log
bash tools/profile_bench.sh gpurun_out/r04_prof 10 > gpurun_out/r04_prof.log 2>&1; echo "prof rc=$?"; cat gpurun_out/r04_prof.log | tail -3
find gpurun_out/r04_prof -name "*kernel_stats.csv" -o -name "*window*.csv" | head
