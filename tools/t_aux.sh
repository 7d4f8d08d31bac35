cd ${GRAFT_REPO_ROOT:-/root/repo}
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest tests/test_aux_gpu.py -k large_batch -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/t_aux_ring.log 2>&1
VN_CONV2F_GENERIC=1 timeout -k 10 200 python -u -m pytest tests/test_aux_gpu.py -k large_batch -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/t_aux_gen.log 2>&1
grep -E "passed|failed|AssertionError: " gpurun_out/t_aux_ring.log gpurun_out/t_aux_gen.log
exit 0
