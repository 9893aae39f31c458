# PMC counters of the register-fed conv (tools/rowconv_bench.py), one pass per counter group
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-rc}
LAYER=${LAYER:-3}
MODES=${MODES:-1}
i=0
for grp in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_BUSY_CYCLES" \
           "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INST_LEVEL_VMEM SQ_LDS_BANK_CONFLICT" \
           "TA_TA_BUSY TA_ADDR_STALLED_BY_TC_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i+1))
  rm -rf gpurun_out/pmc_${TAG}_$i
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $grp --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/pmc_${TAG}_$i" -o run -- python3 tools/rowconv_bench.py --layer $LAYER --modes $MODES --reps 5 > gpurun_out/pmc_${TAG}_$i.log 2>&1
  rc=$?; echo "pass $i rc=$rc"
  [ $rc -eq 0 ] || exit $rc
done
python3 tools/pmc_summary.py gpurun_out/pmc_${TAG}_* 2>&1 | tail -40
