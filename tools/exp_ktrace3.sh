#!/bin/bash
# kernel trace of the emulated 8-way feature-parallel rank step -> gpurun_out/ktrace3/
set -e -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/ktrace3; mkdir -p $O
cd /tmp; export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/fp8 -o k -- python3 $R/bench.py --emulate-shards 8 \
  --steps 20 --warmup 5 --cpu-baseline 0 --rmse 0 --fp32-steps 0 --phase-timers 0 --epoch 0 > $O/fp8.log 2>&1
python3 $R/tools/kernel_gaps.py "$(find $O/fp8 -name '*kernel_trace.csv' | head -1)" 40 > $O/fp8.txt
