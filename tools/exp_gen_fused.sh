#!/bin/bash
# the fused small-model step: Jester tests + trace + bench, the opt-in generator path's parity tests and its
# ML-100K / ML-1M lines against the row-gather path -> gpurun_out/gen_fused/
set -e -o pipefail
O=gpurun_out/gen_fused; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_mlp_step_gpu.py \
  tests/test_train_gpu.py -k "fused" > $O/tests.log 2>&1
timeout -k 10 120 python tools/mlp_trace.py --dtype bfloat16 > $O/trace_bfloat16.json 2> $O/trace.err
run() {   # name, bench args...
  local n=$1; shift
  timeout -k 10 300 python bench.py --fp32-steps 0 --cpu-baseline 0 --rmse 0 "$@" > $O/$n.log 2>&1
  grep '^{' $O/$n.log | tail -1 > $O/$n.json
}
run jester_bf16 --config jester --dtype bfloat16
run jester_f32 --config jester --dtype float32
run ml100k_fg --config ml100k --dtype float32 --fused-gen 1
run ml1m_fg --config ml1m --dtype bfloat16 --fused-gen 1
for f in $O/*.json; do python -c "import json; d=json.load(open('$f')); r=d.get('roofline') or {}; print('$f', d.get('ms_per_step'), d.get('host_issue_ms_per_step'), r.get('kernel'), r.get('kernel_mean_us'), r.get('frac'), d.get('phases_ms'))"; done
