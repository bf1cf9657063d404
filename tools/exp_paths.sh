#!/bin/bash
# how many timed steps take the one-call path (bench.py timed_step_paths) and the host issue per step: the
# emulated 8-way rank step and the default single-GPU step
set -e -o pipefail
O=gpurun_out/paths; mkdir -p $O
timeout -k 10 200 python bench.py --emulate-shards 8 --cpu-baseline 0 --fp32-steps 0 --epoch 0 --rmse 0 > $O/fp8.log 2>&1
timeout -k 10 200 python bench.py --emulate-shards 4 --cpu-baseline 0 --fp32-steps 0 --epoch 0 --rmse 0 > $O/fp4.log 2>&1
timeout -k 10 200 python bench.py --cpu-baseline 0 --fp32-steps 0 --epoch 0 --rmse 0 > $O/ml20m.log 2>&1
for f in fp8 fp4 ml20m; do grep '^{' $O/$f.log | tail -1 > $O/$f.json; python -c "import json; d=json.load(open('$O/$f.json')); print('$f', d['ms_per_step'], d['host_issue_ms_per_step'], d.get('timed_step_paths'))"; done
