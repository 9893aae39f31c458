set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -x -q -p no:cacheprovider -k "taps or wgrad" --timeout 120 --timeout-method thread > gpurun_out/pytest_taps.log 2>&1
rc=$?; echo "pytest taps rc=$rc"; tail -5 gpurun_out/pytest_taps.log
[ $rc -eq 0 ] || exit $rc
VARIANTS="stamps st_abl1 st_abl2" SPLITS=4,8 bash tools/gpu_stamps.sh || exit 1
rm -rf gpurun_out/ts_taps
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/ts_taps" -o run -- python3 tools/wgrad_sweep.py --layer ${LAYER:-3} --splits 4,8,16 > gpurun_out/ts_taps.log 2>&1
rc=$?; echo "sweep rc=$rc"; [ $rc -eq 0 ] || exit $rc
python3 tools/sweep_summary.py $(find gpurun_out/ts_taps -name "*kernel_trace.csv" | head -1) | grep -v at::native
