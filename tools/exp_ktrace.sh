#!/bin/bash
# rocprofv3 kernel traces of the small configs' bench steps (no phase timers) -> gpurun_out/ktrace/<cfg>/
set -e -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/ktrace; mkdir -p $O
cd /tmp; export TMPDIR=/tmp
for cfg in "ml1m:--config ml1m --dtype bfloat16" "ml100k:--config ml100k --dtype float32"; do
  n=${cfg%%:*}; a=${cfg#*:}
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/$n -o k -- python3 $R/bench.py --steps 20 \
    --warmup 5 --cpu-baseline 0 --rmse 0 --fp32-steps 0 --phase-timers 0 --epoch 0 $a > $O/$n.log 2>&1
  python3 $R/tools/kernel_gaps.py "$(find $O/$n -name '*kernel_trace.csv' | head -1)" 24 > $O/$n.txt
done
