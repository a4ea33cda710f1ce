#!/bin/bash
# PMC of the scan kernels in the product's aligned layout: VALU / LDS issue share and HBM bytes (C3 fp32, C5 bf16)
set -u
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 AVSE_TIME_ALIGN_BYTES=128
export PMC_PASSES="SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_WAVES SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE;FETCH_SIZE;WRITE_SIZE"
bash tools/pmc_scan.sh gpurun_out/pmc_c3 --cfg 64,1024,3999 --no-conv --pad --iters 3 > /dev/null || exit 1
bash tools/pmc_scan.sh gpurun_out/pmc_c5 --cfg 32,1024,5999 --dtype bf16 --no-conv --pad --iters 3 > /dev/null || exit 1
grep -A4 "scan::" gpurun_out/pmc_c3/summary.txt | head -30
