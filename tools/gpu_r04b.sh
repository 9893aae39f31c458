# Round-4 measurements: VGG-11 A/B (speculative epilogue, XCD tile order), a rocprofv3 kernel trace
# of the default bench, the VGG-16 / ResNet-18 lines, and the 224-px guard / float32-change samples.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r04b}
for rep in 1 2 3; do
  for v in "on:" "spec0:--rc-spec 0" "mapx:NITI_RC_MAP=x"; do
    name=${v%%:*}; opt=${v#*:}; envs=""; flags=""
    case "$opt" in *=*) envs=$opt;; *) flags=$opt;; esac
    env $envs timeout -k 10 300 python3 bench.py --cpu-sample 0 $flags > gpurun_out/bench_${TAG}_$name.log 2>&1
    rc=$?; [ $rc -eq 0 ] || { tail -5 gpurun_out/bench_${TAG}_$name.log; exit $rc; }
    echo "$name rep$rep $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/bench_${TAG}_$name.log)"
  done
done
rm -rf gpurun_out/tr_$TAG
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/tr_$TAG" -o run -- python3 bench.py --cpu-sample 0 --steps 10 --warmup 3 > gpurun_out/tr_$TAG.log 2>&1
rc=$?; echo "prof rc=$rc"; [ $rc -eq 0 ] || exit $rc
f=$(find gpurun_out/tr_$TAG -name "*kernel_trace.csv" | head -1)
python3 tools/prof_summary.py "$f" 13 > gpurun_out/tr_${TAG}_breakdown.txt
timeout -k 10 400 python3 bench.py --arch vgg16 --steps 4 --warmup 2 --cpu-sample 0 > gpurun_out/vgg16_$TAG.log 2>&1
rc=$?; echo "vgg16 rc=$rc $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/vgg16_$TAG.log)"; [ $rc -eq 0 ] || { tail -5 gpurun_out/vgg16_$TAG.log; exit $rc; }
timeout -k 10 400 python3 bench.py --arch resnet18 --steps 6 --warmup 2 --cpu-sample 0 > gpurun_out/resnet_$TAG.log 2>&1
rc=$?; echo "resnet rc=$rc $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/resnet_$TAG.log)"; [ $rc -eq 0 ] || { tail -5 gpurun_out/resnet_$TAG.log; exit $rc; }
timeout -k 10 500 python3 -u tools/guard_sample.py > gpurun_out/guard_$TAG.txt 2>&1
rc=$?; echo "guard rc=$rc"; tail -30 gpurun_out/guard_$TAG.txt
