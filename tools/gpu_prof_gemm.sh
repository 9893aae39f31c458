set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -rf gpurun_out/profg
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/profg" -o run -- python3 tools/gemm_bench.py --only ${ONLY:-4} --reps 5 > gpurun_out/profg.log 2>&1
rc=$?; echo "rc=$rc"; exit $rc
