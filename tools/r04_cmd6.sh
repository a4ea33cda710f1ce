mkdir -p gpurun_out; export HSA_ENABLE_IPC_MODE_LEGACY=0
for i in 1 2; do
AVSE_HIP_LIB=expso/old_gln.so timeout -k 10 120 python -u tools/gln_bench.py > gpurun_out/r04f_gln_old.log 2>&1 || { echo old_fail; tail -5 gpurun_out/r04f_gln_old.log; exit 1; }
echo "old: $(grep '^{' gpurun_out/r04f_gln_old.log)"
timeout -k 10 120 python -u tools/gln_bench.py > gpurun_out/r04f_gln_new.log 2>&1 || { echo new_fail; tail -5 gpurun_out/r04f_gln_new.log; exit 1; }
echo "new: $(grep '^{' gpurun_out/r04f_gln_new.log)"
done
bash tools/r04_cmd4.sh
