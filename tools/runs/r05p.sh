B="python bench.py --steps 10 --warmup 2 --secondary '' --no-cpu-baseline --no-roofline-hip --no-roofline"
bash tools/gpu_steps.sh r05p "conv3d or conv1 or sconv or dtproj" \
  "timeout -k 10 200 $B" \
  "AVSE_C3F_F16=0 timeout -k 10 200 $B" \
  "AVSE_AVSE1_STREAMS=0 timeout -k 10 200 $B" \
  "timeout -k 10 300 bash tools/profile_bench.sh gpurun_out/r05p_prof_avse1 10"
