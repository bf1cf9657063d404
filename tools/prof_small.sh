#!/bin/bash
# kernel-trace stats of the small BASELINE configs' bench steps (ML-1M bf16, ML-100K fp32) and the emulated
# 8-way feature rank step -> gpurun_out/prof_small/<tag>/
set -e -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/prof_small; mkdir -p $O
run() {
  tag=$1; shift
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/$tag -o run -- python3 bench.py --cpu-baseline 0 --fp32-steps 0 --epoch 0 --rmse 0 --phase-timers 0 "$@" > $O/$tag.json 2> $O/$tag.err
}
run ml1m --config ml1m --dtype bfloat16
run ml100k --config ml100k --dtype float32
run fp8 --emulate-shards 8
find $O -name "*kernel_stats.csv" | sort
