# split-output BatchNorm passes: kernel + module + avse1 model tests (no dist), bench A/B
B="python bench.py --steps 10 --warmup 2 --secondary '' --no-cpu-baseline --no-roofline-hip --no-roofline"
bash tools/gpu_steps.sh r05x "(bnact or split or dilated or sconv or avse1 or conv1) and not two_ranks" \
  "timeout -k 10 200 $B" \
  "AVSE_BNACT_Q=0 timeout -k 10 200 $B" \
  "timeout -k 10 200 $B" \
  "AVSE_BNACT_Q=0 timeout -k 10 200 $B"
