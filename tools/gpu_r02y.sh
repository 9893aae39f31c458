# VGG-16 224x224 batch 64 step: kernel trace summary (per-kernel totals and the last step's launches).
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
rm -rf gpurun_out/y_prof
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/y_prof" -o run -- python3 bench.py --arch vgg16 --steps 4 --warmup 2 --cpu-sample 0 > gpurun_out/y_prof.log 2>&1
rc=$?; echo "prof rc=$rc"; [ $rc -eq 0 ] || exit $rc
f=$(find gpurun_out/y_prof -name '*kernel_trace.csv' | head -1)
python3 tools/prof_summary.py $f 6 > gpurun_out/y_sum.txt; echo "sum rc=$?"
