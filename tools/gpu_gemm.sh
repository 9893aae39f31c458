# per-op GEMM timing; optional PMC passes PMC1..PMC3 (one rocprofv3 run each) on layers $ONLY
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python3 tools/gemm_bench.py --reps 20 > gpurun_out/gemm_bench.log 2>&1
rc=$?; echo "gemm_bench rc=$rc"; grep -v amdgpu.ids gpurun_out/gemm_bench.log
if [ $rc -ne 0 ]; then exit $rc; fi
for i in 1 2 3; do
  v="PMC$i"; P="${!v:-}"
  if [ -z "$P" ]; then continue; fi
  rm -rf gpurun_out/pmc$i
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $P --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/pmc$i" -o run -- python3 tools/gemm_bench.py --reps 3 --only ${ONLY:-3} > gpurun_out/pmc$i.log 2>&1
  rc=$?; echo "pmc$i rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 gpurun_out/pmc$i.log; exit $rc; fi
done
exit 0
