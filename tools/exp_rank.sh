#!/bin/bash
# the feature-parallel rank step as ocf_rank_step phases: GPU tests, the emulated G-way rank steps (rank 0
# alone, no-op collectives) and the 2-rank gloo rehearsal of bench.py's N>1 path
set -e
out=gpurun_out/rank
mkdir -p $out
timeout -k 10 500 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_feature_parallel_gpu.py tests/test_fast_step_gpu.py > $out/tests.log 2>&1
for G in 2 4 8; do
  timeout -k 10 200 python bench.py --emulate-shards $G --cpu-baseline 0 --fp32-steps 0 --epoch 0 --rmse 0 \
    > $out/fp$G.json 2> $out/fp$G.err
done
timeout -k 10 600 bash tools/rehearse_multi.sh $out/rehearse > $out/rehearse.log 2>&1
