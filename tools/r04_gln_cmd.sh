set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread "tests/test_gpu_kernels.py::test_dwconv_prelu_gln_fused_vs_fp64" "tests/test_gpu_models.py::test_avse4_tblock_golden_fwd_and_grads" > gpurun_out/gln_test.log 2>&1 || { tail -30 gpurun_out/gln_test.log; exit 1; }
tail -1 gpurun_out/gln_test.log
timeout -k 10 120 python -u tools/gln_bench.py > gpurun_out/gln_bench.txt 2>&1 || { tail gpurun_out/gln_bench.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/gln_bench.txt
