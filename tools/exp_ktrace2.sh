#!/bin/bash
# ML-1M kernel trace with the folded jobs as separate kernels (--fold-jobs 0): are the dW launches bound by
# their jobs?  -> gpurun_out/ktrace2/
set -e -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/ktrace2; mkdir -p $O
cd /tmp; export TMPDIR=/tmp
for cfg in "ml1m_nofold:--config ml1m --dtype bfloat16 --fold-jobs 0" "ml100k_nofold:--config ml100k --dtype float32 --fold-jobs 0"; do
  n=${cfg%%:*}; a=${cfg#*:}
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/$n -o k -- python3 $R/bench.py --steps 20 \
    --warmup 5 --cpu-baseline 0 --rmse 0 --fp32-steps 0 --phase-timers 0 --epoch 0 $a > $O/$n.log 2>&1
  python3 $R/tools/kernel_gaps.py "$(find $O/$n -name '*kernel_trace.csv' | head -1)" 30 > $O/$n.txt
done
