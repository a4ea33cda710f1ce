mkdir -p gpurun_out; export HSA_ENABLE_IPC_MODE_LEGACY=0
for i in 1 2; do
AVSE_HIP_LIB=expso/old_gln.so timeout -k 10 120 python -u tools/gln_bench.py > gpurun_out/r04e_gln_old.log 2>&1 || { echo old_fail; tail -5 gpurun_out/r04e_gln_old.log; exit 1; }
echo "old: $(grep '^{' gpurun_out/r04e_gln_old.log)"
timeout -k 10 120 python -u tools/gln_bench.py > gpurun_out/r04e_gln_new.log 2>&1 || { echo new_fail; tail -5 gpurun_out/r04e_gln_new.log; exit 1; }
echo "new: $(grep '^{' gpurun_out/r04e_gln_new.log)"
done
timeout -k 10 300 python -u -m pytest tests -x -v -m gpu -k "gln or tblock or avse4" --timeout 200 --timeout-method thread > gpurun_out/r04e_gln_tests.log 2>&1; rc=$?
echo "gln tests rc=$rc"; grep -E "FAILED|ERROR|passed|failed" gpurun_out/r04e_gln_tests.log | tail -5
[ $rc -eq 0 ] || exit 1
bash tools/r04_cmd4.sh
