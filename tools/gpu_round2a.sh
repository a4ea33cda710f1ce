set -u
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_dropin.py tests/test_gpu_models.py tests/test_gpu_fullsize.py tests/test_gpu_kernels.py tests/test_gpu_avmamba.py -k "audio_only or c5 or production" -x -v --timeout 400 --timeout-method thread -p no:cacheprovider -s > gpurun_out/t2.log 2>&1
rc=$?; tail -30 gpurun_out/t2.log; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 600 python bench.py --steps 5 --warmup 2 > gpurun_out/bench2.log 2>&1; rc2=$?
tail -2 gpurun_out/bench2.log; exit $rc2
