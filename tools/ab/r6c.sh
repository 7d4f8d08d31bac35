timeout -k 10 500 python -u -m pytest tests/test_parity_dgrad_gpu.py -k "lean or prefetch or resident" -x -v --timeout 200 --timeout-method thread > gpurun_out/t_r6c.log 2>&1; rc=$?; tail -8 gpurun_out/t_r6c.log; [ $rc -eq 0 ] || exit $rc
FLAG=VN_CONV1WG_NOLEAN PAT="conv1_wgrad_x3" REPS=2 LEG_ARGS="--no-train-ff --no-train-ref4 --no-short --no-train-84" bash tools/ab/kflag_ab.sh && \
FLAG=VN_CONV2F_RING2_NOPF PAT="ring2" REPS=2 LEG_ARGS="--no-train-ff --no-train-ref4 --no-short --no-train-84" bash tools/ab/kflag_ab.sh
