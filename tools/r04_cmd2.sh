mkdir -p gpurun_out; export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u tools/avse1_stream_diag.py serial serial stream_nohold stream serial > gpurun_out/r04b_diag.log 2>&1 || { echo DIAG_FAIL; tail -30 gpurun_out/r04b_diag.log; exit 1; }
grep -E "^\[|grad trunk.layer4|pgrad net_visualfeat.tcn" gpurun_out/r04b_diag.log
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu -k "avse1 or lstm or two_ranks or variants" --timeout 300 --timeout-method thread > gpurun_out/r04b_tests.log 2>&1; echo "tests rc=$?"
grep -E "PASS|FAIL|ERROR|passed|failed|branch|rank" gpurun_out/r04b_tests.log | tail -60
timeout -k 10 200 python -u tools/scan_fwd_ab.py > gpurun_out/r04b_ab.log 2>&1; echo "ab rc=$?"; grep -v amdgpu.ids gpurun_out/r04b_ab.log
