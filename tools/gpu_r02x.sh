# Bench lines of the other BASELINE networks on one GPU: LeNet (cfg 1), VGG-16 224 batch 64 (cfg 3's per-GPU share).
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 300 python bench.py --arch lenet --cpu-sample 0 > gpurun_out/x_lenet.json 2> gpurun_out/x_lenet.err
rc=$?; echo "lenet rc=$rc"; cut -c1-240 gpurun_out/x_lenet.json; [ $rc -eq 0 ] || { tail -5 gpurun_out/x_lenet.err; exit $rc; }
timeout -k 10 400 python bench.py --arch vgg16 --steps 10 --warmup 3 > gpurun_out/x_vgg16.json 2> gpurun_out/x_vgg16.err
rc=$?; echo "vgg16 rc=$rc"; cut -c1-240 gpurun_out/x_vgg16.json; [ $rc -eq 0 ] || { tail -5 gpurun_out/x_vgg16.err; exit $rc; }
