# rowconv ablation variants (tools/stages_build.sh -> tools/ablate/<name>): per-layer times and
# stamps, forward and input gradient, for the in-tree build and each variant
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for e in base ${VARIANTS:-e1 e2 e4 e8}; do
  lib=tools/ablate/$e/libniti_hip.so; [ $e = base ] && lib=mandheling-dsp-training_amd/niti_amd/_lib/libniti_hip.so
  for d in "" "--dgrad fused"; do
    echo "== $e $d"
    NITI_HIP_LIB=$lib timeout -k 10 90 python -u tools/rowconv_bench.py --stamps --modes ${MODES:-0} $d 2>&1 | grep -v amdgpu.ids || exit 1
  done
done
