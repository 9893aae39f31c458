# requant_quad grid cap A/B (NITI_RQ_BLOCKS): VGG-11 bench and VGG-16 bench, alternating.
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for rep in 1 2; do
  for cap in 2048 8192; do
    NITI_RQ_BLOCKS=$cap timeout -k 10 240 python bench.py --cpu-sample 0 > gpurun_out/z11_${cap}_$rep.json 2>/dev/null
    rc=$?; [ $rc -eq 0 ] || exit $rc
    NITI_RQ_BLOCKS=$cap timeout -k 10 300 python bench.py --arch vgg16 --steps 10 --warmup 3 > gpurun_out/z16_${cap}_$rep.json 2>/dev/null
    rc=$?; [ $rc -eq 0 ] || exit $rc
    python -c "import json; a=json.load(open('gpurun_out/z11_${cap}_$rep.json')); b=json.load(open('gpurun_out/z16_${cap}_$rep.json')); print('cap', $cap, a['value'], a['ms_per_step'], b['value'], b['ms_per_step'])"
  done
done
