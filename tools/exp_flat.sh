#!/bin/bash
# A/B of the pair launch's rank-range form (rows_flat = row workgroups per CU; 0 = tile parts), same box,
# interleaved; then the pair / fast-step bit-identity tests.
set -e
mkdir -p gpurun_out/flat
for r in 1 2; do
  for f in 0 6 4 8 12; do
    timeout -k 10 200 python bench.py --rows-flat $f --cpu-baseline 0 --fp32-steps 0 --epoch 0 --rmse 0 \
      > gpurun_out/flat/f${f}_$r.json 2> gpurun_out/flat/f${f}_$r.err
  done
done
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_fast_step_gpu.py \
  tests/test_pair_sync_gpu.py > gpurun_out/flat/tests.log 2>&1
