set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 60 ./tools/probes/probe_tr8 > gpurun_out/probe_tr8.log 2>&1
rc=$?; echo "probe rc=$rc"; head -70 gpurun_out/probe_tr8.log
exit $rc
