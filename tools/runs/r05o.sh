bash tools/gpu_steps.sh r05o "dtproj or mode2 or bimamba_block" \
  "timeout -k 10 300 python bench.py --workload mamba --steps 3 --warmup 2 --no-cpu-baseline" \
  "MARK=roof timeout -k 10 350 bash tools/profile_bench.sh gpurun_out/r05o_prof_avmamba 3 --workload avmamba --warmup 2" \
  "MARK=roof timeout -k 10 300 bash tools/profile_bench.sh gpurun_out/r05o_prof_avse4 6 --workload avse4 --warmup 2"
