set -o pipefail
ROOT=$GRAFT_REPO_ROOT
export TMPDIR=/tmp
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $ROOT/gpurun_out/prof_tr -o run -- python3 $ROOT/bench.py --no-c5 --steps 20 --warmup 2 --no-cpu-baseline --no-pmc --no-train-ff --no-train-ref --train-steps 4 --train-warmup 1 > $ROOT/gpurun_out/prof_tr.log 2>&1
