#!/bin/bash
# bench lines for the other BASELINE configs on one MI355X: ML-1M bf16 (configs[1]), Netflix width
# (configs[3] on one GPU), ML-100K fp32 (configs[0]) -> gpurun_out/<tag>/<config>.json
set -e -o pipefail
O=gpurun_out/${1:-cfg}; mkdir -p $O
timeout -k 10 300 python bench.py --config ml1m --dtype bfloat16 --fp32-steps 0 > $O/ml1m.log 2>&1
grep '^{' $O/ml1m.log | tail -1 > $O/ml1m.json
timeout -k 10 300 python bench.py --config ml100k --dtype float32 > $O/ml100k.log 2>&1
grep '^{' $O/ml100k.log | tail -1 > $O/ml100k.json
timeout -k 10 600 python bench.py --config netflix --steps 20 --fp32-steps 0 > $O/netflix.log 2>&1
grep '^{' $O/netflix.log | tail -1 > $O/netflix.json
for c in ml1m ml100k netflix; do
  python -c "import json; d=json.load(open('$O/$c.json')); print('$c', d['dtype'], d['ms_per_step'], d['value'], d['roofline'] and d['roofline']['frac'], d['step_roofline']['frac_of_binding_roof'], d.get('cpu_baseline', {}).get('value'))"
done
