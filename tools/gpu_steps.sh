# Run GPU steps in order, each under its own time limit; stop at the first failure (no GPU step after a fault).
# usage (through gpurun): bash tools/gpu_steps.sh TAG 'pytest -k expr' [extra step commands...]
mkdir -p gpurun_out; export HSA_ENABLE_IPC_MODE_LEGACY=0
tag=$1; expr=$2; shift 2
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread -k "$expr" > gpurun_out/${tag}_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; grep -E "FAILED|ERROR|passed|failed|dconv split|wgrad16 vs|gemm_f32s err" gpurun_out/${tag}_tests.log | tail -40
[ $rc -eq 0 ] || exit $rc
i=0
for step in "$@"; do
  i=$((i+1))
  timeout -k 10 400 bash -c "$step" > gpurun_out/${tag}_step$i.log 2>&1; rc=$?
  echo "step $i rc=$rc: $step"; cut -c1-1200 gpurun_out/${tag}_step$i.log | tail -12
  [ $rc -eq 0 ] || exit $rc
done
