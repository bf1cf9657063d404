#!/bin/bash
# row-stream dW LONG variant: parity / bit-identity tests, then A/B bench lines (ML-20M default, emulated
# 8-way feature rank step, ML-1M bf16, ML-100K fp32) -> gpurun_out/long/
set -e -o pipefail
O=gpurun_out/long; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_rows_dw_gpu.py tests/test_semantics_gpu.py > $O/tests.log 2>&1
echo tests ok
for L in 0 1; do
  timeout -k 10 200 python bench.py --rows-long $L --cpu-baseline 0 --fp32-steps 0 --epoch 0 > $O/ml20m_L$L.json 2> $O/err.log
  timeout -k 10 200 python bench.py --rows-long $L --emulate-shards 8 --cpu-baseline 0 --fp32-steps 0 --rmse 0 > $O/fp8_L$L.json 2>> $O/err.log
  timeout -k 10 200 python bench.py --rows-long $L --config ml1m --dtype bfloat16 --cpu-baseline 0 --fp32-steps 0 --epoch 0 > $O/ml1m_L$L.json 2>> $O/err.log
  timeout -k 10 200 python bench.py --rows-long $L --config ml100k --dtype float32 --cpu-baseline 0 --epoch 0 > $O/ml100k_L$L.json 2>> $O/err.log
  echo L=$L done
done
for f in $O/*.json; do python -c "import json,sys; d=json.loads(open('$f').read().strip().splitlines()[-1]); print('$f', d['ms_per_step'], d['phases_ms'])"; done
