set -o pipefail
mkdir -p gpurun_out
bash tools/r04_gemm_abl.sh && bash tools/pmc_gemm.sh gpurun_out/pmc_inproj --case "in_proj fwd" && bash tools/pmc_gemm.sh gpurun_out/pmc_dgrad --case "in_proj dgrad"
