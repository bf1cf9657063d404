#!/bin/bash
# row-stream dW kernel: 12 vs 32 workgroups per tile on the small weights (ML-1M, ML-100K) and the emulated
# 8-way rank step -> gpurun_out/parts/
set -e -o pipefail
O=gpurun_out/parts; mkdir -p $O
B="--cpu-baseline 0 --fp32-steps 0 --epoch 0 --rmse 0"
for W in 0 100000; do
  timeout -k 10 200 python bench.py $B --rows-small-waves $W --config ml1m --dtype bfloat16 > $O/ml1m_W$W.json 2>> $O/err.log
  timeout -k 10 200 python bench.py $B --rows-small-waves $W --config ml100k --dtype float32 > $O/ml100k_W$W.json 2>> $O/err.log
  timeout -k 10 200 python bench.py $B --rows-small-waves $W --emulate-shards 8 > $O/fp8_W$W.json 2>> $O/err.log
  echo W=$W done
done
timeout -k 10 200 python bench.py $B > $O/ml20m.json 2>> $O/err.log
for f in $O/*.json; do python -c "import json; d=json.loads(open('$f').read().strip().splitlines()[-1]); print('$f', d['ms_per_step'], d['phases_ms'])"; done
