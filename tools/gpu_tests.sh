# Selected -m gpu tests on one MI355X (through gpurun): bash tools/gpu_tests.sh TAG "pytest -k expression"
mkdir -p gpurun_out; export HSA_ENABLE_IPC_MODE_LEGACY=0
tag=$1; expr=$2
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread -k "$expr" > gpurun_out/${tag}_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; grep -E "FAILED|ERROR|passed|failed|dconv split" gpurun_out/${tag}_tests.log | tail -30
exit $rc
