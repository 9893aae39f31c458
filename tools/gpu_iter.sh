#!/bin/bash
# One development iteration on the GPU box: the selected GPU test files (TESTS), then the
# ImageNet-net benches and traces (NETS) with any extra environment given on the command line.
set -u
cd "$GRAFT_REPO_ROOT"
TAG=${TAG:-r05}
if [ -n "${TESTS:-}" ]; then TAG=$TAG TESTS="$TESTS" bash tools/gpu_suite.sh || exit $?; fi
if [ -n "${NETS:-}" ]; then TAG=$TAG NETS="$NETS" bash tools/gpu_nets.sh || exit $?; fi
