# round 6: kernel-time breakdown of the C3 / C4 / C5 steps (rocprofv3 window of the last eager warm-up step, MARK=roof)
mkdir -p gpurun_out; export HSA_ENABLE_IPC_MODE_LEGACY=0
for wl in avse4 mamba avmamba; do
  MARK=roof timeout -k 10 800 bash tools/profile_bench.sh gpurun_out/r06i_$wl 3 --workload $wl --warmup 1 --no-parity > gpurun_out/r06i_$wl.log 2>&1; r=$?
  echo "$wl rc=$r"; [ $r -eq 0 ] || exit $r
  head -16 gpurun_out/r06i_$wl/window_stats.csv | cut -c1-150
done
