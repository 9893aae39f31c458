# Host-tensor Execution tests + P16 diag variants (stamps; slab vs atomic split-K output).
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_exec_host.py tests/test_gpu_wgrad_p16.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t_r02f.log 2>&1
rc=$?; tail -3 gpurun_out/t_r02f.log; echo "tests rc=$rc"; [ $rc -eq 0 ] || { grep -E "Error|assert" gpurun_out/t_r02f.log | head -20; exit $rc; }
SPLITS=${SPLITS:-1,2,4} VARIANTS="${VARIANTS:-st at}" bash tools/wg_diag.sh
