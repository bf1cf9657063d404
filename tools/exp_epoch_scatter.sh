# per-entry scatter outputs built per epoch (ocf_epoch_scatter, default) vs the per-step scatter: tests + 3 x 2 bench
set -e -o pipefail
O=gpurun_out/escat; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for rep in 1 2 3; do
  for f in 0 1; do
    OCF_EPOCH_SCATTER=$f timeout -k 10 300 python bench.py --steps 40 --cpu-baseline 0 --rmse 0 --fp32-steps 0 > $O/b_${f}_$rep.log 2>&1
    grep '^{' $O/b_${f}_$rep.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('epoch_scatter $f', d['ms_per_step'], d['phases_ms']['scatter'])"
  done
done
