B="python bench.py --steps 10 --warmup 2 --secondary '' --no-cpu-baseline --no-roofline-hip --no-roofline"
bash tools/gpu_steps.sh r05l "sconv or trunk_conv2d or dtproj or mode2 or bnact_vs_fp64 or avse1 or avse4_full_train_step_vs_masked or dconv or audiofeat" \
  "python tools/sconv_bench.py --no-miopen" \
  "$B" \
  "python bench.py --workload avse4 --steps 6 --warmup 2 --no-cpu-baseline --no-roofline --no-roofline-hip" \
  "python bench.py --workload mamba --steps 3 --warmup 1 --no-cpu-baseline --no-roofline"
