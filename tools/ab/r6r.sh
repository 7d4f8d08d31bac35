#!/bin/bash
# conv_merge's forward and the LSTM's dh product on 128 x 64 tiles with K in two halves
# (VN_DENSE_SK2) against 64 x 64 x 64 tiles; 84² and 174² legs.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-/root/repo}
cd $ROOT
P="DenseRows, vn::DenseRows, vn::Epi(LstmDh|BiasAct|Slab)>|splitk_epilogue_kernel<vn::Epi(LstmDh|BiasAct)"
FLAG=VN_DENSE_SK2 PAT="$P" REPS=2 bash tools/ab/kflag_ab.sh || exit 1
