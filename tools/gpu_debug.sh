set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python tools/debug_gradconv.py > gpurun_out/debug_gradconv.log 2>&1
rc=$?; echo "debug rc=$rc"; cat gpurun_out/debug_gradconv.log | grep -v amdgpu.ids
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/prof_r01a" -o run -- python3 bench.py --steps 10 --warmup 3 --cpu-sample 0 > gpurun_out/prof_r01a.log 2>&1
rc=$?; echo "rocprof rc=$rc"; tail -3 gpurun_out/prof_r01a.log
find gpurun_out/prof_r01a -name "*stats*" | head
exit $rc
