mkdir -p gpurun_out
for v in base ub1 ub3 ub4 base; do
  if [ $v = base ]; then lib=avse_challenge_amd/libavse_hip.so; else lib=expso/gln_$v.so; fi
  echo "$v $(AVSE_HIP_LIB=$lib timeout -k 10 120 python -u tools/gln_bench.py 2>&1 | grep '^{' | python -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['dwconv_gln_bwd'], d['dwconv_gln_fwd'])")" || exit 1
done
