#!/bin/bash
# Round-4 closing GPU call: the traced GPU suite (per-test kernel map input), then the tile A/B.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-/root/repo}
cd $ROOT
TAG=r04f TRACE=1 bash tools/gpu_tests_traced.sh || exit $?
bash tools/r04/ab_tiles.sh
