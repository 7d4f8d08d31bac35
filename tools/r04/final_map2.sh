#!/bin/bash
# Round-end (second) closing GPU call after the C5 conv2 weight-gradient change: the traced GPU
# suite for the per-test kernel map, then the C5 leg's kernel trace (its top-20 list).
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-/root/repo}
cd $ROOT
TAG=r04h TRACE=1 bash tools/gpu_tests_traced.sh || exit $?
TAG=r04h bash tools/r04/prof_c5.sh
