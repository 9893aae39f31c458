set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for cfg in "0 0" "6464 1" "6464 2" "12864 1" "12864 2" "64128 1" "64128 2" "0 1"; do
  set -- $cfg
  if [ "$1" = 0 ]; then unset NITI_DIAG_TILE; else export NITI_DIAG_TILE=$1; fi
  if [ "$2" = 0 ]; then unset NITI_DIAG_SPLITS; else export NITI_DIAG_SPLITS=$2; fi
  timeout -k 10 120 python3 tools/gemm_bench.py --only ${ONLY:-4,5,6} --reps 20 > gpurun_out/tiles.log 2>&1 || exit 1
  echo "tile=$1 splits=$2 $(grep -E '^L' gpurun_out/tiles.log | awk '{print $1,$2,$(NF-4)}' | tr '\n' '|')"
done
