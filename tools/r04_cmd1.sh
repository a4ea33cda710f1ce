mkdir -p gpurun_out; export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 500 python -u tools/avse1_stream_diag.py > gpurun_out/r04a_diag.log 2>&1 || { echo DIAG_FAIL; exit 1; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -v -k "lstm or variants" --timeout 150 --timeout-method thread > gpurun_out/r04a_kt.log 2>&1; echo "kt rc=$?"
tail -4 gpurun_out/r04a_kt.log
timeout -k 10 200 python -u tools/scan_fwd_ab.py > gpurun_out/r04a_ab.log 2>&1; echo "ab rc=$?"; cat gpurun_out/r04a_ab.log | grep -v amdgpu.ids
grep -v -e amdgpu.ids -e "MIOpen(HIP)" gpurun_out/r04a_diag.log | tail -190
