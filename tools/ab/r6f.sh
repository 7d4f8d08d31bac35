timeout -k 10 300 python -u -m pytest tests/test_parity_dgrad_gpu.py -k "rotated or resident or lean" -x -q --timeout 200 --timeout-method thread > gpurun_out/t_r6f.log 2>&1; rc=$?; tail -3 gpurun_out/t_r6f.log; [ $rc -eq 0 ] || exit $rc
FLAG=VN_CONV2DG_NOROT PAT="conv2_dgrad" REPS=2 LEG_ARGS="--no-train-ff --no-train-ref4 --no-short" bash tools/ab/kflag_ab.sh
