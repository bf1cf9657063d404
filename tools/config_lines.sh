#!/bin/bash
# bench lines for the other BASELINE configs on one MI355X: ML-1M bf16 (configs[1], I- and U-AutoRec
# orientation), Netflix width (configs[3] on one GPU), ML-100K fp32 (configs[0]), Jester dense
# (configs[4], fp32 and bf16) -> gpurun_out/<tag>/<config>.json
set -e -o pipefail
O=gpurun_out/${1:-cfg}; mkdir -p $O
run() {   # name, timeout, bench args...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t python bench.py "$@" > $O/$n.log 2>&1
  grep '^{' $O/$n.log | tail -1 > $O/$n.json
  echo "$n done"
}
run ml1m 300 --config ml1m --dtype bfloat16 --fp32-steps 0
run ml1m_u 300 --config ml1m_u --dtype bfloat16 --fp32-steps 0
run ml100k 300 --config ml100k --dtype float32
run netflix 600 --config netflix --steps 20 --fp32-steps 0
run jester_f32 300 --config jester --dtype float32
run jester_bf16 300 --config jester --dtype bfloat16
for c in ml1m ml1m_u ml100k netflix jester_f32 jester_bf16; do
  python -c "import json; d=json.load(open('$O/$c.json')); r=d.get('roofline') or {}; sr=d.get('step_roofline') or {}; print('$c', d['dtype'], d['ms_per_step'], d['value'], r.get('frac'), sr.get('frac_of_binding_roof'), (d.get('cpu_baseline') or {}).get('value'))"
done
