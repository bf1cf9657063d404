#!/bin/bash
# gather chunk sizes for the feature-parallel rank step (emulated 8- and 4-way) and ML-20M
set -e -o pipefail
O=gpurun_out/chunk_fp; mkdir -p $O
A="--cpu-baseline 0 --fp32-steps 0 --epoch 0 --rmse 0"
for rep in 1 2; do
  for c in 256 128 64; do
    for g in 8 4; do
      timeout -k 10 200 python tools/chunk_bench.py $c 64 96 -- --emulate-shards $g $A > $O/fp${g}_c${c}_$rep.log 2>&1
      python -c "import json; d=json.loads([l for l in open('$O/fp${g}_c${c}_$rep.log') if l.startswith('{')][-1]); print('fp$g c$c', d['ms_per_step'], d['phases_ms'].get('enc_gemm'), d['phases_ms'].get('dec_gemm_mse'))"
    done
  done
done
