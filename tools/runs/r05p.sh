B="python bench.py --steps 10 --warmup 2 --secondary '' --no-cpu-baseline --no-roofline-hip --no-roofline"
bash tools/gpu_steps.sh r05p "conv3d or conv1 or sconv or dtproj or mode2 or bnact_vs_fp64" \
  "timeout -k 10 200 $B" \
  "AVSE_C3F_F16=0 AVSE_C3W_F16=0 timeout -k 10 200 $B" \
  "timeout -k 10 300 bash tools/profile_bench.sh gpurun_out/r05p_prof_avse1 10" \
  "timeout -k 10 300 python bench.py --workload mamba --steps 3 --warmup 2 --no-cpu-baseline --no-roofline" \
  "timeout -k 10 200 python tools/gemm_probe.py --reps 20" \
  "AVSE_HIP_LIB=tools/variants/libavse_hip_pgv1.so timeout -k 10 200 python tools/gemm_probe.py --reps 20 --no-lib"
