# A/B of the weight-gradient row lists built per epoch (ocf_epoch_row_lists) vs per step (ocf_row_lists):
#   bash tools/exp_epoch_lists.sh   (through gpurun; row-list GPU tests first, then 2 x 2 bench runs + a trace)
set -e -o pipefail
O=gpurun_out/epoch_lists; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_rows_dw_gpu.py tests/test_optim_ws_gpu.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for rep in 1 2; do
for a in "e0:--epoch-lists 0" "e1:--epoch-lists 1"; do
  n=${a%%:*}; x=${a#*:}
  timeout -k 10 300 python bench.py $x --steps 40 --cpu-baseline 0 --rmse 0 --fp32-steps 0 > $O/b_${n}_$rep.log 2>&1
  grep '^{' $O/b_${n}_$rep.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$n', d['ms_per_step'], d['value'], d['phases_ms'], d['row_lists'])"
done
done
cd /tmp; export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/ks -o ks -- python3 $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 3 --cpu-baseline 0 --rmse 0 --fp32-steps 0 > $GRAFT_REPO_ROOT/$O/ks.log 2>&1
echo done
