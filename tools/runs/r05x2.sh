# split-output BatchNorm in the avse4 ResNet: tests + C4 bench A/B
B="python bench.py --workload avse4 --steps 5 --warmup 2 --no-cpu-baseline --no-roofline"
bash tools/gpu_steps.sh r05x2 "avse4 or bnact" \
  "timeout -k 10 300 $B" \
  "AVSE_BNACT_Q=0 timeout -k 10 300 $B" \
  "timeout -k 10 300 $B"
