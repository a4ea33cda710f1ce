mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread "tests/test_gpu_kernels.py::test_dwconv_prelu_gln_fused_vs_fp64" "tests/test_gpu_models.py::test_avse4_tblock_golden_fwd_and_grads" "tests/test_gpu_models.py::test_avse4_full_train_step_vs_masked_oracle" > gpurun_out/gln_test.log 2>&1 || { tail -30 gpurun_out/gln_test.log; exit 1; }
tail -1 gpurun_out/gln_test.log
for i in 1 2; do timeout -k 10 120 python -u tools/gln_bench.py 2>&1 | grep '^{'; done
