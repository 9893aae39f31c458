# rowconv variants (diagnostic builds under build/exp): per-layer times, forward and input gradient
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for e in base ${VARIANTS:-16}; do
  lib=build/exp/e$e/libniti_hip.so; [ $e = base ] && lib=mandheling-dsp-training_amd/niti_amd/_lib/libniti_hip.so
  for L in ${LAYERS:-2 3 4 5 6 7}; do
    for d in "" "--dgrad fused"; do
      echo "== RC_EXP=$e layer $L $d"
      NITI_HIP_LIB=$lib timeout -k 10 60 python -u tools/rowconv_bench.py --layer $L --modes 1,0 $d 2>&1 | grep -v amdgpu.ids || exit 1
    done
  done
done
