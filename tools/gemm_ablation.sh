# Ablation runner for the projection GEMM: tools/gemm_probe.py against libavse_hip.so and expso/pg_<V>.so variants built
# by tools/build_exp.sh from tools/pg_exp.patch (e.g. -DPG_NOLOAD -DPG_NOEPI -DPG_NOBAR).  usage: bash tools/gemm_ablation.sh
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/pg_abl.jsonl
for v in base LE LEB; do
  if [ $v = base ]; then lib=avse_challenge_amd/libavse_hip.so; else lib=expso/pg_$v.so; fi
  echo "== $v" >> gpurun_out/pg_abl.jsonl
  AVSE_HIP_LIB=$lib timeout -k 10 120 python -u tools/gemm_probe.py --reps 10 --no-lib >> gpurun_out/pg_abl.jsonl 2>&1 || exit 1
done
grep -v amdgpu.ids gpurun_out/pg_abl.jsonl | python -c "
import sys, json
for l in sys.stdin:
    l=l.strip()
    if l.startswith('=='): print(l); continue
    try: d=json.loads(l)
    except Exception: print(l); continue
    print(d['gemm'], d.get('hip_ms'), d.get('hip_frac'), d.get('fold', ''))
"
