#!/bin/bash
# A/B of conv3's forward product tile (VN_C3_CFG, csrc/vn_policy.hip forward): rocprofv3
# kernel stats of the 84x84 LSTM and 174x174 LSTM + aux bench legs per form; prints each
# form's conv3 forward calls and average duration. The VN_C3_CFG switch (1: 128x32, 2: 64x64,
# 3: 128x64, 4: 128x64 with BK 64) was removed from the source after the measurement
# (profiles/r03/ab_conv3/summary.txt); re-add it to run this again.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-/root/repo}
export TMPDIR=/tmp
OUT=$ROOT/gpurun_out/ab_conv3
mkdir -p $OUT
for cfg in ${CFGS:-0 1 2 3 4}; do
  cd /tmp && VN_C3_CFG=$cfg timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/p$cfg -o run \
    -- python3 $ROOT/bench.py --no-c5 --steps 5 --warmup 1 --no-cpu-baseline --no-pmc --train-steps 2 --train-warmup 1 \
    --no-train-ff --no-train-ref4 > $OUT/cfg$cfg.log 2>&1 || exit 1
  S=$(find $OUT/p$cfg -name '*kernel_stats.csv' | head -1)
  echo "== cfg $cfg"
  python3 - "$S" <<'EOF'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    n = r["Name"]
    if "NhwcIm2col<32, 4, 4, 2," in n and "gemm_x6" in n or ("splitk_epilogue" in n and "BiasAct" in n):
        print("%8s calls %10.1f us  %s" % (r["Calls"], float(r["AverageNs"]) / 1e3, n[:120]))
EOF
  grep -o '"ms_per_update": [0-9.]*' $OUT/cfg$cfg.log | tr '\n' ' '; echo
done
