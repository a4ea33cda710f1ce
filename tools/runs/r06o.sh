# round 6: C4 line with the split GEMM as its in-step roofline
mkdir -p gpurun_out; export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u bench.py --workload avse4 --steps 6 --warmup 2 --secondary "" --no-cpu-baseline --no-roofline-hip --no-parity > gpurun_out/r06o_c4.log 2>&1; r=$?
echo "c4 rc=$r"; grep '^{' gpurun_out/r06o_c4.log | tail -1 | python -c "
import json,sys; r=json.loads(sys.stdin.read()); ro=r['roofline']; print(r['value'], r['ms_per_step']); print(json.dumps(ro)[:1500])"
exit $r
