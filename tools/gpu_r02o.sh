# Kernel traces of the bench step with the fused P16 dy copy and with the separate conversion.
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
for sep in 0 1; do
  rm -rf gpurun_out/o_prof_$sep
  NITI_P16_SEPARATE=$sep timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/o_prof_$sep" -o run -- python3 bench.py --cpu-sample 0 --steps 10 --warmup 3 > gpurun_out/o_prof_$sep.log 2>&1
  rc=$?; echo "sep=$sep rc=$rc"; grep metric gpurun_out/o_prof_$sep.log | cut -c1-160; [ $rc -eq 0 ] || exit $rc
  f=$(find gpurun_out/o_prof_$sep -name '*kernel_trace.csv' | head -1)
  python3 tools/prof_summary.py $f 13 > gpurun_out/o_sum_$sep.txt; rc=$?; [ $rc -eq 0 ] || exit $rc
done
