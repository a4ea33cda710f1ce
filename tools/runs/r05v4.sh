# the fork's gradient sum with its max (in_proj backward split without absmax): Mamba tests + C3; the avse1 roofline
# measured with the lip branch serialized, against its rocprof window
bash tools/gpu_steps.sh r05v4 "mamba or bimamba or dropin or add_max" \
  "timeout -k 10 300 python bench.py --workload mamba --steps 3 --warmup 2 --no-cpu-baseline --no-roofline" \
  "timeout -k 10 400 bash tools/profile_bench.sh gpurun_out/r05v4_prof_avse1 10"
