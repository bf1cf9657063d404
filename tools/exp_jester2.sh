#!/bin/bash
set -e -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/jester2; mkdir -p $O
timeout -k 10 700 python -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_api_gpu.py tests/test_configs_gpu.py > $O/tests.log 2>&1
echo tests ok
timeout -k 10 300 python bench.py --config jester --dtype float32 > $O/f32.json 2> $O/err.log
timeout -k 10 300 python bench.py --config jester --dtype bfloat16 > $O/bf16.json 2>> $O/err.log
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/prof -o run -- python3 bench.py --config jester --dtype bfloat16 --cpu-baseline 0 --phase-timers 0 > $O/prof.json 2>> $O/err.log
for f in $O/f32.json $O/bf16.json; do python -c "import json; d=json.loads(open('$f').read().strip().splitlines()[-1]); print('$f', d['ms_per_step'], d['value'], d['host_issue_ms_per_step'], d['phases_ms'], d.get('cpu_baseline',{}).get('value'))"; done
