# ResNet-18 (config 5) step: bench line and a rocprofv3 kernel-trace summary.
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python bench.py --arch resnet18 --steps 10 --warmup 3 > gpurun_out/s_bench.json 2> gpurun_out/s_bench.err
rc=$?; echo "bench rc=$rc"; cut -c1-300 gpurun_out/s_bench.json; [ $rc -eq 0 ] || exit $rc
rm -rf gpurun_out/s_prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/s_prof" -o run -- python3 bench.py --arch resnet18 --steps 5 --warmup 2 > gpurun_out/s_prof.log 2>&1
rc=$?; echo "prof rc=$rc"; [ $rc -eq 0 ] || exit $rc
f=$(find gpurun_out/s_prof -name '*kernel_stats.csv' | head -1); head -25 $f | cut -d, -f1-4 
