#!/bin/bash
# Round-4: ResNet-18 roofline probe (speculative launch A of layer1.0.a) -- PMC FETCH / WRITE passes,
# traffic.json entry, then the bench line carrying it.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r04z}
for c in FETCH_SIZE WRITE_SIZE; do
  rm -rf gpurun_out/pmc_${TAG}_$c
  timeout -s KILL 240 rocprofv3 --kernel-trace --pmc $c --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/pmc_${TAG}_$c" -o run -- python3 bench.py --arch resnet18 --steps 2 --warmup 1 --no-autotune --cpu-sample 0 > gpurun_out/pmc_${TAG}_$c.log 2>&1
  rc=$?; echo "pmc $c rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
cp profiles/traffic.json gpurun_out/traffic.json
python3 tools/traffic.py gpurun_out/pmc_${TAG}_FETCH_SIZE gpurun_out/pmc_${TAG}_WRITE_SIZE gpurun_out/traffic.json resnet18_b128_L1_p0 0,0,0,3 > gpurun_out/traffic_${TAG}.txt 2>&1
rc=$?; cat gpurun_out/traffic_${TAG}.txt; [ $rc -eq 0 ] || exit $rc
rm -rf gpurun_out/pmc_${TAG}_FETCH_SIZE gpurun_out/pmc_${TAG}_WRITE_SIZE
cp gpurun_out/traffic.json profiles/traffic.json
timeout -k 10 300 python3 bench.py --arch resnet18 --steps 8 --warmup 2 > gpurun_out/resnet_$TAG.log 2>&1
rc=$?; echo "resnet rc=$rc $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/resnet_$TAG.log) $(grep -o '"traffic": [0-9a-z]*' gpurun_out/resnet_$TAG.log)"
