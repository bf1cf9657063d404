# dW_out with and without the folded jobs (bench --fold-jobs), kernel trace per run -> gpurun_out/jobs/
set -e -o pipefail
O=gpurun_out/jobs; mkdir -p $O
cd /tmp; export TMPDIR=/tmp
for fj in 1 0; do
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/$O/fj$fj -o ks -- python3 $GRAFT_REPO_ROOT/bench.py --fold-jobs $fj --steps 20 --warmup 3 --cpu-baseline 0 --rmse 0 --fp32-steps 0 > $GRAFT_REPO_ROOT/$O/fj$fj.log 2>&1
  grep '^{' $GRAFT_REPO_ROOT/$O/fj$fj.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('fold $fj', d['ms_per_step'])"
done
