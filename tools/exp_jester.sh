#!/bin/bash
# Jester bench lines (f32 parity mode, bf16) + a kernel trace of the f32 one -> gpurun_out/jester/
set -e -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/jester; mkdir -p $O
timeout -k 10 300 python bench.py --config jester --dtype float32 > $O/f32.json 2> $O/err.log
timeout -k 10 300 python bench.py --config jester --dtype bfloat16 > $O/bf16.json 2>> $O/err.log
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/prof -o run -- python3 bench.py --config jester --dtype float32 --cpu-baseline 0 --phase-timers 0 > $O/prof.json 2>> $O/err.log
for f in $O/f32.json $O/bf16.json; do python -c "import json; d=json.loads(open('$f').read().strip().splitlines()[-1]); print('$f', d['ms_per_step'], d['value'], d['host_issue_ms_per_step'], d['phases_ms'], d.get('cpu_baseline',{}).get('value'))"; done
