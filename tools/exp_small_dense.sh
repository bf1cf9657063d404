#!/bin/bash
# small configs: the row-gather path (default) vs the dense layer-wise GEMM path (--gather 0), phase timers
# on -> gpurun_out/small_dense/<cfg>_g<0|1>.json; then the ML-1M U-orientation parity test
set -e -o pipefail
O=gpurun_out/small_dense; mkdir -p $O
for g in 1 0; do
  timeout -k 10 300 python bench.py --config ml1m --dtype bfloat16 --fp32-steps 0 --cpu-baseline 0 --rmse 0 --gather $g > $O/ml1m_g$g.log 2>&1
  grep '^{' $O/ml1m_g$g.log | tail -1 > $O/ml1m_g$g.json
  timeout -k 10 300 python bench.py --config ml100k --dtype float32 --fp32-steps 0 --cpu-baseline 0 --rmse 0 --gather $g > $O/ml100k_g$g.log 2>&1
  grep '^{' $O/ml100k_g$g.log | tail -1 > $O/ml100k_g$g.json
done
for f in $O/*.json; do python -c "import json; d=json.load(open('$f')); print('$f', d['ms_per_step'], d.get('phases_ms'))"; done
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_configs_gpu.py -k ml1m_u > $O/tests.log 2>&1
