B="python bench.py --steps 10 --warmup 2 --secondary '' --no-cpu-baseline --no-roofline-hip --no-roofline"
bash tools/gpu_steps.sh r05k "sconv or trunk_conv2d or avse1_visualfeat or avse1_bench_step or avse1_full" \
  "python tools/sconv_bench.py" \
  "$B" "AVSE_SCONV=0 $B"
