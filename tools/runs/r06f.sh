# round 6: PMC passes over the dconv (d = 4) and sconv micro-benchmarks; the sconv timings
mkdir -p gpurun_out; export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u tools/sconv_bench.py --no-miopen > gpurun_out/r06f_sconv_bench.log 2>&1; r=$?
echo "sconv bench rc=$r"; cut -c1-400 gpurun_out/r06f_sconv_bench.log | tail -12
[ $r -eq 0 ] || exit $r
timeout -k 10 600 bash tools/pmc_cmd.sh gpurun_out/r06f_pmc_dconv tools/dconv_bench.py --no-miopen --dils 4 --iters 3 > gpurun_out/r06f_pmc_dconv.log 2>&1; r=$?
echo "pmc dconv rc=$r"; grep -A14 "dcf::fwd_kernel\|dcf::wgrad_kernel" gpurun_out/r06f_pmc_dconv/summary.txt | head -60
[ $r -eq 0 ] || exit $r
timeout -k 10 600 bash tools/pmc_cmd.sh gpurun_out/r06f_pmc_sconv tools/sconv_bench.py --no-miopen > gpurun_out/r06f_pmc_sconv.log 2>&1; r=$?
echo "pmc sconv rc=$r"; grep -A14 "scv::fwd_kernel\|scv::wgrad_kernel" gpurun_out/r06f_pmc_sconv/summary.txt | head -80
exit $r
