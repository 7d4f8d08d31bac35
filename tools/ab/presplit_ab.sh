set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for V in on off; do
  if [ $V = off ]; then export VN_NO_PRESPLIT=1; fi
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/ab_ps_$V -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-pmc --no-train-ff --no-c5 --no-train-ref4 --train-steps 3 > $GRAFT_REPO_ROOT/gpurun_out/ab_ps_$V.log 2>&1) || exit $?
done
unset VN_NO_PRESPLIT
timeout -k 10 400 python tools/ab/dedup_drift.py 40 256 84 noaux control > gpurun_out/dedup_drift_84_control.txt 2>&1
tail -3 gpurun_out/dedup_drift_84_control.txt
