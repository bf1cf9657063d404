# (historical: the --prefetch / --overlap-dw-out switches were removed with the experiment)
# dW_out on the side stream beside the next batch's load + encoder (bench --prefetch / --overlap-dw-out)
set -e -o pipefail
O=gpurun_out/overlap; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_train_gpu.py tests/test_rows_dw_gpu.py tests/test_api_gpu.py tests/test_optim_ws_gpu.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for rep in 1 2; do
for a in "p0:--prefetch 0 --overlap-dw-out 0" "p1:--prefetch 1 --overlap-dw-out 1" "p1o0:--prefetch 1 --overlap-dw-out 0"; do
  n=${a%%:*}; x=${a#*:}
  timeout -k 10 300 python bench.py $x --steps 40 --cpu-baseline 0 --rmse 0 --fp32-steps 0 > $O/b_${n}_$rep.log 2>&1
  grep '^{' $O/b_${n}_$rep.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$n', d['ms_per_step'], d['value'], d['roofline']['kernel_mean_us'])"
done
done
