# round 6 (ad): PMC HBM traffic (FETCH_SIZE / WRITE_SIZE passes) of the scan roofline kernels and the avse4 fused
# dwconv / gLN kernels on the final tree -> profiles/r06_traffic.json (bench.py's roofline `traffic`)
mkdir -p gpurun_out; export HSA_ENABLE_IPC_MODE_LEGACY=0
PHASES="scan scan_bwd scan_c5 scan_bwd_c5 cconv dwconv_gln dwconv_gln_bwd prelu_gln prelu_gln_bwd" bash tools/pmc_traffic.sh gpurun_out/r06ad_pmc gpurun_out/r06ad_traffic.json > gpurun_out/r06ad_pmc.log 2>&1; r=$?
echo "pmc rc=$r"; tail -40 gpurun_out/r06ad_pmc.log | cut -c1-200
exit $r
