#!/bin/bash
# SURVEY.md 8(d) batch sweep on one MI355X (run through gpurun from the repo root):
#   bash tools/batch_sweep.sh [tag]
# ML-20M I-AutoRec step at B = 256 ... 4096 rows; one bench line per B -> gpurun_out/<tag>/sweep.jsonl
set -e -o pipefail
TAG=${1:-sweep}
O=gpurun_out/$TAG; mkdir -p $O
: > $O/sweep.jsonl
for B in 256 512 1024 2048 4096; do
  timeout -k 10 400 python bench.py --batch $B --steps 20 --warmup 4 --cpu-baseline 0 --rmse 0 --fp32-steps 0 > $O/b$B.log 2>&1
  grep '^{' $O/b$B.log | tail -1 >> $O/sweep.jsonl
  tail -1 $O/sweep.jsonl | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['config']['batch_per_gpu'], d['ms_per_step'], d['value'], d['step_roofline'])"
done
