#!/bin/bash
# max pool k3 s2 p1 backward on 2x2 input blocks: parity (kernel + lip front-end models), then the default bench line
set -u
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 500 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_models.py -k "maxpool or avse1_full_golden or avse1_wave_frontend or avse4_visual_frontend or avse4_full" -q -rf --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/t_mp.log 2>&1
rc=$?; tail -2 gpurun_out/t_mp.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/bench_mp.log 2>&1; rc=$?
python - <<'PY'
import json
l = json.loads([x for x in open("gpurun_out/bench_mp.log") if x.startswith("{")][0])
print(l["value"], l["ms_per_step"])
for e in l["roofline_hip"]:
    if "maxpool" in e["kernel"]: print(e["kernel"], e["avg_ms"], e["frac"])
PY
exit $rc
