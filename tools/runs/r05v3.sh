# round-5 validation, part 2: the default bench line (headline + secondary configs, roofline, CPU baseline) and a
# rocprofv3 window of the headline's timed steps
mkdir -p gpurun_out; export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 900 python -u bench.py > gpurun_out/r05v3_bench.log 2>&1; rc=$?; echo "bench rc=$rc"; grep '^{' gpurun_out/r05v3_bench.log | tail -1 | cut -c1-600
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 bash tools/profile_bench.sh gpurun_out/r05v3_prof_avse1 10; echo "prof rc=$?"
