#!/bin/bash
set -e -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/prof_small2; mkdir -p $O
for c in ml1m:bfloat16 ml100k:float32; do
  n=${c%%:*}; d=${c#*:}
  timeout -k 10 300 rocprofv3 --kernel-trace -d $O/$n -o run -- python3 bench.py --cpu-baseline 0 --fp32-steps 0 --epoch 0 --rmse 0 --phase-timers 0 --config $n --dtype $d > $O/$n.json 2> $O/$n.err
done
