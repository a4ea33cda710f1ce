#!/bin/bash
# scan forward: PMC (SQ group + FETCH/WRITE) of the 4-lane and 2-lane layouts at C3
set -u
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
for g in 4 2; do
  AVSE_SCAN_G=$g PMC_PASSES="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS;SQ_INSTS_SALU SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES SQ_BUSY_CYCLES SQ_INST_CYCLES_VMEM_RD SQ_WAIT_INST_VMEM" \
    bash tools/pmc_scan.sh gpurun_out/r03b_pmc_g$g --cfg 64,1024,3999 --pad --no-conv --iters 3 > gpurun_out/r03b_pmc_g$g.txt 2>&1 || { tail -20 gpurun_out/r03b_pmc_g$g.txt; exit 1; }
  grep -A4 "fwd" gpurun_out/r03b_pmc_g$g.txt | head -12
done
