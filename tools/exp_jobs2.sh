#!/bin/bash
# job-only workgroups in the row-stream kernel: bit-identity / parity tests, then bench lines
set -e -o pipefail
O=gpurun_out/jobs2; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_rows_dw_gpu.py \
  tests/test_semantics_gpu.py tests/test_optim_ws_gpu.py -k "not long_variant" > $O/tests.log 2>&1
echo tests ok
B="--cpu-baseline 0 --fp32-steps 0 --epoch 0 --rmse 0"
timeout -k 10 200 python bench.py $B --config ml1m --dtype bfloat16 > $O/ml1m.json 2>> $O/err.log
timeout -k 10 200 python bench.py $B --config ml100k --dtype float32 > $O/ml100k.json 2>> $O/err.log
timeout -k 10 200 python bench.py $B --emulate-shards 8 > $O/fp8.json 2>> $O/err.log
timeout -k 10 200 python bench.py $B > $O/ml20m.json 2>> $O/err.log
timeout -k 10 200 python bench.py $B > $O/ml20m_b.json 2>> $O/err.log
for f in $O/*.json; do python -c "import json; d=json.loads(open('$f').read().strip().splitlines()[-1]); print('$f', d['ms_per_step'], d['phases_ms'])"; done
