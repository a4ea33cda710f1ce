B="python bench.py --steps 10 --warmup 2 --secondary '' --no-cpu-baseline --no-roofline-hip --no-roofline"
bash tools/gpu_steps.sh r05k "sconv or trunk_conv2d or dtproj or mode2 or bimamba_block or masknet or avse4_full_train_step_vs_masked" \
  "python tools/sconv_bench.py --no-miopen" \
  "$B" \
  "python bench.py --workload mamba --steps 4 --warmup 2 --no-cpu-baseline --no-roofline" \
  "python bench.py --workload avse4 --steps 6 --warmup 2 --no-cpu-baseline --no-roofline --no-roofline-hip" \
  "AVSE_SCONV=0 python bench.py --workload avse4 --steps 6 --warmup 2 --no-cpu-baseline --no-roofline --no-roofline-hip"
