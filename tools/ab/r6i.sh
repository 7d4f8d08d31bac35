timeout -k 10 300 python -u -m pytest tests/test_policy_gpu.py tests/test_replay_gpu.py tests/test_unreal_gpu.py tests/test_trainer_hooks_gpu.py tests/test_train_cli.py -x -q --timeout 200 --timeout-method thread > gpurun_out/t_r6i.log 2>&1; rc=$?; tail -3 gpurun_out/t_r6i.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/nan_stress.py > gpurun_out/nan_stress_r6i.log 2>&1; rc=$?; tail -2 gpurun_out/nan_stress_r6i.log; [ $rc -eq 0 ] || exit $rc
FLAG=VN_REPLAY_MERGED PAT="replay_push" REPS=2 LEG_ARGS="--no-train-ff --no-train-84 --no-train-174 --no-short" bash tools/ab/kflag_ab.sh
