# C5 step time with the projection GEMM routing modes (AVSE_PROJ_GEMM = 1 | all | 0), two interleaved rounds
mkdir -p gpurun_out
for g in 1 all 0 1 all 0; do
  AVSE_PROJ_GEMM=$g timeout -k 10 300 python -u bench.py --workload avmamba --steps 4 --warmup 1 --no-cpu-baseline --no-roofline-hip > gpurun_out/c5ab_$g.log 2>&1 || exit 1
  echo "PROJ_GEMM=$g $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/c5ab_$g.log)"
done
