# C3 producer-side maxima (add+RMSNorm fwd/bwd, direction-sum add) + the bf16 lip-encoder GEMM conv fix: tests, C3 / C5
bash tools/gpu_steps.sh r05v2 "avmamba or rmsnorm or add_max or mamba or gemm_f32s or projgemm or dropin or avse4" \
  "timeout -k 10 300 python bench.py --workload mamba --steps 3 --warmup 2 --no-cpu-baseline --no-roofline" \
  "timeout -k 10 300 python bench.py --workload avmamba --steps 4 --warmup 2 --no-cpu-baseline --no-roofline"
