B="python bench.py --steps 10 --warmup 2 --secondary '' --no-cpu-baseline --no-roofline-hip --no-roofline"
bash tools/gpu_steps.sh r05j "sconv or trunk_conv2d or f32s or bimamba_block" \
  "python tools/sconv_bench.py" \
  "python tools/gemm_f32s_probe.py" \
  "$B" "AVSE_SCONV=0 $B" "AVSE_AVSE1_SIDE_PRIO=-1 $B" \
  "python bench.py --workload mamba --steps 4 --warmup 2 --no-cpu-baseline --no-roofline --no-roofline-hip" \
  "bash tools/profile_bench.sh gpurun_out/r05j_prof_avse1 10"
