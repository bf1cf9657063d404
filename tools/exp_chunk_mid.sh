#!/bin/bash
# the mid-size gather chunk rule: parity / bit-identity tests, then the small configs' bench lines
set -e -o pipefail
O=gpurun_out/${1:-chunk_mid}; mkdir -p $O
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_semantics_gpu.py \
  tests/test_configs_gpu.py tests/test_rows_dw_gpu.py tests/test_fast_step_gpu.py tests/test_api_gpu.py tests/test_train_gpu.py \
  tests/test_smoke_gpu.py > $O/tests.log 2>&1
tail -1 $O/tests.log
B="--cpu-baseline 0 --fp32-steps 0 --epoch 0"
for c in ml1m ml1m_u; do timeout -k 10 200 python bench.py --config $c --dtype bfloat16 $B > $O/$c.log 2>&1; grep '^{' $O/$c.log | tail -1 > $O/$c.json; done
timeout -k 10 200 python bench.py --config ml100k --dtype float32 $B > $O/ml100k.log 2>&1; grep '^{' $O/ml100k.log | tail -1 > $O/ml100k.json
for c in ml1m ml1m_u ml100k; do python -c "import json; d=json.load(open('$O/$c.json')); print('$c', d['ms_per_step'], d['phases_ms'], d.get('masked_rmse'))"; done
