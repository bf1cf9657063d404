set -e -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/kt; mkdir -p $O
cd /tmp; export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/b -o b -- python3 $GRAFT_REPO_ROOT/bench.py --steps 8 --warmup 3 --cpu-baseline 0 --rmse 0 --fp32-steps 0 > $O/b.log 2>&1
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/b0 -o b -- python3 $GRAFT_REPO_ROOT/bench.py --steps 8 --warmup 3 --cpu-baseline 0 --rmse 0 --fp32-steps 0 --phase-timers 0 > $O/b0.log 2>&1
echo ok
