set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for v in 0 1 3 4; do
  if [ $v = 0 ]; then unset NITI_HIP_LIB; else export NITI_HIP_LIB=$PWD/tools/ablate/$v/libniti_hip.so; fi
  echo "== ablate $v"
  timeout -k 10 200 python3 tools/gemm_bench.py --sweep --reps 10 > gpurun_out/ablate$v.log 2>&1 || exit 1
  grep sweep gpurun_out/ablate$v.log | grep -E "16384x256|16384x512"
  timeout -k 10 200 python3 tools/gemm_bench.py --only 3,5 --reps 10 > gpurun_out/ablateL$v.log 2>&1 || exit 1
  grep -E "^L" gpurun_out/ablateL$v.log
done
