timeout -k 10 400 python -u -m pytest tests/test_aux_gpu.py tests/test_prod_oracle_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/t_r6j.log 2>&1; rc=$?; tail -3 gpurun_out/t_r6j.log; [ $rc -eq 0 ] || exit $rc
TAG=l174r06j LEG_ARGS="--no-train-ff --no-train-84 --no-train-ref4 --no-short" UPDATES=2 PICK=2 bash tools/prof_leg.sh > /dev/null || exit 1
grep -E "aux_deconv2|aux_backward2|update 2" gpurun_out/breakdown_l174r06j.txt
TAG=c5r06j bash tools/prof_c5.sh > /dev/null || exit 1
grep -E "aux_deconv2|aux_backward2|update 2" gpurun_out/breakdown_c5r06j.txt
rm -f gpurun_out/prof_l174r06j/*kernel_trace.csv gpurun_out/prof_c5r06j/*kernel_trace.csv
