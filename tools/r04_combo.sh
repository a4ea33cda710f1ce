set -o pipefail
bash tools/r04_gln_cmd.sh && bash tools/r04_gemm_pmc.sh
