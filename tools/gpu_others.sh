# The other BASELINE networks on one GPU: VGG-16 224x224 batch 64 (config 4's per-GPU share of
# 512 on 8) with its probe's PMC traffic, LeNet batch 256, ResNet-18 224x224 batch 128 (config 5's
# per-GPU share of 1024 on 8) with its probe's PMC traffic; every line with roofline and cpu_baseline.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r03}
timeout -k 10 300 python3 bench.py --arch vgg16 --cpu-sample 0 --save-plans gpurun_out/plans_vgg16_$TAG.json > gpurun_out/vgg16_tune_$TAG.log 2>&1
rc=$?; echo "vgg16 tune rc=$rc"; [ $rc -eq 0 ] || exit $rc
P="--load-plans gpurun_out/plans_vgg16_$TAG.json"
rm -rf gpurun_out/pmcF_vgg16_$TAG gpurun_out/pmcW_vgg16_$TAG
timeout -s KILL 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/pmcF_vgg16_$TAG" -o run -- python3 bench.py --arch vgg16 --steps 2 --warmup 1 --cpu-sample 0 $P > gpurun_out/pmcF_vgg16_$TAG.log 2>&1
rc=$?; echo "pmcF rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -s KILL 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/pmcW_vgg16_$TAG" -o run -- python3 bench.py --arch vgg16 --steps 2 --warmup 1 --cpu-sample 0 $P > gpurun_out/pmcW_vgg16_$TAG.log 2>&1
rc=$?; echo "pmcW rc=$rc"; [ $rc -eq 0 ] || exit $rc
PLAN=$(python3 -c "import json; l=[x for x in open('gpurun_out/vgg16_tune_$TAG.log') if x.startswith('{')][-1]; p=json.loads(l)['roofline']['plan']; print(','.join(str(p[k]) for k in ('bm','bn','splits','strategy')))")
python3 tools/traffic.py gpurun_out/pmcF_vgg16_$TAG gpurun_out/pmcW_vgg16_$TAG profiles/traffic.json vgg16_b64_L3_p2 $PLAN > gpurun_out/traffic_vgg16_$TAG.txt 2>&1 || exit 1
cp profiles/traffic.json gpurun_out/traffic_$TAG.json
timeout -k 10 600 python3 bench.py --arch vgg16 --cpu-sample 1 $P > gpurun_out/vgg16_$TAG.log 2>&1
rc=$?; echo "vgg16 rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 bench.py --arch lenet --cpu-sample 0 --save-plans gpurun_out/plans_lenet_$TAG.json > gpurun_out/lenet_tune_$TAG.log 2>&1
rc=$?; echo "lenet tune rc=$rc"; [ $rc -eq 0 ] || exit $rc
PL="--load-plans gpurun_out/plans_lenet_$TAG.json"
rm -rf gpurun_out/pmcF_lenet_$TAG gpurun_out/pmcW_lenet_$TAG
timeout -s KILL 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/pmcF_lenet_$TAG" -o run -- python3 bench.py --arch lenet --steps 3 --warmup 1 --cpu-sample 0 $PL > gpurun_out/pmcF_lenet_$TAG.log 2>&1
rc=$?; echo "lenet pmcF rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -s KILL 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/pmcW_lenet_$TAG" -o run -- python3 bench.py --arch lenet --steps 3 --warmup 1 --cpu-sample 0 $PL > gpurun_out/pmcW_lenet_$TAG.log 2>&1
rc=$?; echo "lenet pmcW rc=$rc"; [ $rc -eq 0 ] || exit $rc
PLAN=$(python3 -c "import json; l=[x for x in open('gpurun_out/lenet_tune_$TAG.log') if x.startswith('{')][-1]; p=json.loads(l)['roofline']['plan']; print(','.join(str(p[k]) for k in ('bm','bn','splits','strategy')))")
python3 tools/traffic.py gpurun_out/pmcF_lenet_$TAG gpurun_out/pmcW_lenet_$TAG profiles/traffic.json lenet_b256_L1_p2 $PLAN > gpurun_out/traffic_lenet_$TAG.txt 2>&1 || exit 1
cp profiles/traffic.json gpurun_out/traffic_$TAG.json
timeout -k 10 300 python3 bench.py --arch lenet $PL > gpurun_out/lenet_$TAG.log 2>&1
rc=$?; echo "lenet rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 bench.py --arch resnet18 --cpu-sample 0 --save-plans gpurun_out/plans_resnet18_$TAG.json > gpurun_out/resnet18_tune_$TAG.log 2>&1
rc=$?; echo "resnet18 tune rc=$rc"; [ $rc -eq 0 ] || exit $rc
PR="--load-plans gpurun_out/plans_resnet18_$TAG.json"
rm -rf gpurun_out/pmcF_resnet18_$TAG gpurun_out/pmcW_resnet18_$TAG
timeout -s KILL 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/pmcF_resnet18_$TAG" -o run -- python3 bench.py --arch resnet18 --steps 2 --warmup 1 --cpu-sample 0 $PR > gpurun_out/pmcF_resnet18_$TAG.log 2>&1
rc=$?; echo "resnet18 pmcF rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -s KILL 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/pmcW_resnet18_$TAG" -o run -- python3 bench.py --arch resnet18 --steps 2 --warmup 1 --cpu-sample 0 $PR > gpurun_out/pmcW_resnet18_$TAG.log 2>&1
rc=$?; echo "resnet18 pmcW rc=$rc"; [ $rc -eq 0 ] || exit $rc
PLAN=$(python3 -c "import json; l=[x for x in open('gpurun_out/resnet18_tune_$TAG.log') if x.startswith('{')][-1]; p=json.loads(l)['roofline']['plan']; print(','.join(str(p[k]) for k in ('bm','bn','splits','strategy')))")
python3 tools/traffic.py gpurun_out/pmcF_resnet18_$TAG gpurun_out/pmcW_resnet18_$TAG profiles/traffic.json resnet18_b128_L1_p0 $PLAN > gpurun_out/traffic_resnet18_$TAG.txt 2>&1 || exit 1
cp profiles/traffic.json gpurun_out/traffic_$TAG.json
timeout -k 10 400 python3 bench.py --arch resnet18 --cpu-sample 1 $PR > gpurun_out/resnet18_$TAG.log 2>&1
rc=$?; echo "resnet18 rc=$rc"
exit $rc
