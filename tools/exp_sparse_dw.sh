#!/bin/bash
# small configs: sparse (row-stream) vs dense-operand (MFMA role-split) weight-gradient launches
set -e -o pipefail
O=gpurun_out/sdw; mkdir -p $O
for c in "ml1m:--config ml1m --dtype bfloat16" "ml100k:--config ml100k --dtype float32" "ml1m_u:--config ml1m_u --dtype bfloat16"; do
  n=${c%%:*}; a=${c#*:}
  for s in 1 0; do
    timeout -k 10 300 python bench.py --fp32-steps 0 --cpu-baseline 0 --rmse 0 --epoch 0 $a --sparse-dw $s > $O/${n}_s$s.log 2>&1
    grep '^{' $O/${n}_s$s.log | tail -1 > $O/${n}_s$s.json
    python -c "import json; d=json.load(open('$O/${n}_s$s.json')); print('${n}_s$s', d['ms_per_step'], d.get('timed_step_paths'), d.get('phases_ms'))"
  done
done
