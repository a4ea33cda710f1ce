# round-6 final validation of the last tree on one MI355X: every -m gpu test, smoke(), the default bench line (headline
# + secondaries with their parity legs), then the rocprofv3 windows of the headline (timed + roofline) and of C5 / C3
mkdir -p gpurun_out; export HSA_ENABLE_IPC_MODE_LEGACY=0
tag=${1:-r06f2}
bash tools/runs/r06final.sh $tag; rc=$?
echo "final rc=$rc"; [ $rc -eq 0 ] || exit $rc
bash tools/profile_bench.sh gpurun_out/${tag}_avse1 10; r=$?; echo "avse1 prof rc=$r"; [ $r -eq 0 ] || exit $r
MARK=roof bash tools/profile_bench.sh gpurun_out/${tag}_c5 3 --workload avmamba --warmup 2; r=$?; echo "c5 prof rc=$r"; exit $r
