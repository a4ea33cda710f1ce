set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 python -u -m pytest -x -q --timeout 60 --timeout-method thread tests/test_gpu_projgemm.py > gpurun_out/pg_test.log 2>&1 || { tail -30 gpurun_out/pg_test.log; exit 1; }
echo "test: $(tail -1 gpurun_out/pg_test.log)"
timeout -k 10 200 python -u tools/gemm_probe.py --reps 10 > gpurun_out/pg_probe_lib2.jsonl 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/pg_probe_lib2.jsonl | python -c "
import sys, json
for l in sys.stdin:
    d=json.loads(l); print(d['gemm'], 'hip', d.get('hip_ms'), d.get('hip_frac'), 'lib', d.get('lib_ms'), d.get('lib_frac'))
"
