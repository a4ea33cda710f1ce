# in-step roofline windows (MARK=roof: the markers bracket the last eager warm-up step) for C3 / C4 / C5
mkdir -p gpurun_out; export HSA_ENABLE_IPC_MODE_LEGACY=0
MARK=roof timeout -k 10 400 bash tools/profile_bench.sh gpurun_out/r05s3_roof_avse4 3 --workload avse4 --warmup 2 && \
MARK=roof timeout -k 10 500 bash tools/profile_bench.sh gpurun_out/r05s3_roof_avmamba 3 --workload avmamba --warmup 2 && \
MARK=roof timeout -k 10 500 bash tools/profile_bench.sh gpurun_out/r05s3_roof_mamba 3 --workload mamba --warmup 2
