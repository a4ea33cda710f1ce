B="python bench.py --steps 10 --warmup 2 --secondary '' --no-cpu-baseline --no-roofline-hip --no-roofline"
bash tools/gpu_steps.sh r05n "conv1_module" \
  "timeout -k 10 200 $B" \
  "timeout -k 10 300 bash tools/profile_bench.sh gpurun_out/r05n_prof_avse1 10" \
  "timeout -k 10 300 python bench.py --workload avmamba --steps 3 --warmup 2 --no-cpu-baseline --no-roofline"
