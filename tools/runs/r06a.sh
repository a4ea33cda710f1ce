# round 6: the 2-rank avse1 dist test with the new diagnostics (twice), then every -m gpu test without -x
mkdir -p gpurun_out; export HSA_ENABLE_IPC_MODE_LEGACY=0
for i in 1 2; do
  timeout -k 10 600 python -u -m pytest tests/test_gpu_dist.py -v -s -m gpu --timeout 500 --timeout-method thread -k avse1 > gpurun_out/r06a_dist$i.log 2>&1; rc=$?
  echo "dist$i rc=$rc"; grep -E "diagnostics|total rel err|branch|passed|failed" gpurun_out/r06a_dist$i.log | cut -c1-1500
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
done
timeout -k 10 1000 python -u -m pytest tests -v -m gpu --timeout 300 --timeout-method thread --deselect "tests/test_gpu_dist.py::test_two_ranks_one_gpu_side_stream_buckets[avse1]" > gpurun_out/r06a_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; grep -E "FAILED|ERROR|passed|failed" gpurun_out/r06a_tests.log | tail -8
exit $rc
