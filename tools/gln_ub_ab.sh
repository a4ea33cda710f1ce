# A/B of the gLN kernels' accesses in flight: tools/gln_bench.py against expso/gln_<v>.so builds (tools/build_exp.sh)
mkdir -p gpurun_out
for v in base ${GLN_VARIANTS:-u41 u44 r1 r4} base; do
  if [ $v = base ]; then lib=avse_challenge_amd/libavse_hip.so; else lib=expso/gln_$v.so; fi
  echo "$v $(AVSE_HIP_LIB=$lib timeout -k 10 120 python -u tools/gln_bench.py 2>&1 | grep '^{')" || exit 1
done
