timeout -k 10 300 python -u -m pytest tests/test_parity_dgrad_gpu.py -k "lean" -x -q --timeout 200 --timeout-method thread > gpurun_out/t_r6d.log 2>&1; rc=$?; tail -3 gpurun_out/t_r6d.log; [ $rc -eq 0 ] || exit $rc
FLAG=VN_CONV1WG_NOLEAN PAT="conv1_wgrad_x3_kernel" REPS=2 LEG_ARGS="--no-train-ff --no-train-ref4 --no-short --no-train-84" bash tools/ab/kflag_ab.sh
