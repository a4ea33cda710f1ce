set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python -u tools/gemm_probe.py --reps 10 > gpurun_out/pg_probe_lib.jsonl 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/pg_probe_lib.jsonl | python -c "
import sys, json
for l in sys.stdin:
    d=json.loads(l); print(d['gemm'], 'hip', d.get('hip_ms'), d.get('hip_frac'), 'lib', d.get('lib_ms'), d.get('lib_frac'))
"
for g in 1 0 1 0; do
  AVSE_PROJ_GEMM=$g timeout -k 10 300 python -u bench.py --workload avmamba --steps 4 --warmup 1 --no-cpu-baseline --no-roofline-hip > gpurun_out/pg_c5_$g.log 2>&1 || exit 1
  echo "PROJ_GEMM=$g $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/pg_c5_$g.log)"
done
