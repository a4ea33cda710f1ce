mkdir -p gpurun_out; export HSA_ENABLE_IPC_MODE_LEGACY=0
bash tools/r04_gemm_abl.sh || exit 1
PHASES="cconv dwconv_gln_bwd dwconv_gln" bash tools/pmc_traffic.sh gpurun_out/r04i_pmc gpurun_out/r04i_traffic.json > gpurun_out/r04i_pmc.log 2>&1; echo "pmc rc=$?"; tail -4 gpurun_out/r04i_pmc.log
