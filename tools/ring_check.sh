set -o pipefail
cd ${GRAFT_REPO_ROOT:-/root/repo}
R=$PWD
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_parity_dgrad_gpu.py -k conv2_ring -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/t_ring.log 2>&1; rc=$?; tail -5 gpurun_out/t_ring.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -m pytest tests/test_prod_oracle_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/t_prod.log 2>&1; rc=$?; tail -3 gpurun_out/t_prod.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/ab/conv2f_ab.py 4096 10 > gpurun_out/ab_ring.log 2>&1; rc=$?; tail -2 gpurun_out/ab_ring.log; [ $rc -eq 0 ] || exit $rc
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_ring -o run --output-format csv -- python3 $R/tools/ab/conv2f_ab.py 4096 5 > $R/gpurun_out/prof_ring.log 2>&1; rc=$?; [ $rc -eq 0 ] || exit $rc
grep -E "conv2_fwd|NhwcIm2col<32, 4, 4, 2, 42" $R/gpurun_out/prof_ring/run_kernel_stats.csv | cut -c1-200
