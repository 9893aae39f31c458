#!/bin/bash
# Round-4: row-segment per-layer A/B at the current kernel (policy check), VGG-11 default and
# data-parallel-path (one GPU) steps, and a kernel trace of the data-parallel path.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r04i}
timeout -k 10 400 python3 -u tools/seg_bench.py > gpurun_out/seg_bench_$TAG.txt 2>&1
rc=$?; echo "seg rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/seg_bench_$TAG.txt; exit $rc; }
for v in "on:" "dp:--dp-path"; do
  name=${v%%:*}; opt=${v#*:}
  timeout -k 10 300 python3 bench.py --cpu-sample 0 $opt > gpurun_out/vgg11_${TAG}_$name.log 2>&1
  rc=$?; echo "vgg11 $name rc=$rc $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/vgg11_${TAG}_$name.log)"; [ $rc -eq 0 ] || { tail -5 gpurun_out/vgg11_${TAG}_$name.log; exit $rc; }
done
rm -rf gpurun_out/tr_${TAG}_dp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/tr_${TAG}_dp" -o run -- python3 bench.py --cpu-sample 0 --dp-path --steps 10 --warmup 3 > gpurun_out/tr_${TAG}_dp.log 2>&1
rc=$?; echo "prof rc=$rc"; [ $rc -eq 0 ] || exit $rc
f=$(find gpurun_out/tr_${TAG}_dp -name "*kernel_trace.csv" | head -1)
python3 tools/prof_summary.py "$f" 13 > gpurun_out/tr_${TAG}_dp_breakdown.txt
rm -rf gpurun_out/tr_${TAG}_dp
tail -14 gpurun_out/seg_bench_$TAG.txt
