# P16 weight gradient diag variants only (stamps), conv4 / conv6 at splits 1,2,4.
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
SPLITS=${SPLITS:-1,2,4} VARIANTS="${VARIANTS:-st at}" bash tools/wg_diag.sh
