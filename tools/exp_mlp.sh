#!/bin/bash
# the fused small-model step (ocf_mlp_step): parity tests, its phase trace (library grid and a sweep), then
# the Jester bench fused vs layer-wise
set -e
out=gpurun_out/mlp
mkdir -p $out
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread -m gpu tests/test_mlp_step_gpu.py \
  > $out/tests.log 2>&1
for dt in bfloat16 float32; do
  timeout -k 10 120 python tools/mlp_trace.py --dtype $dt > $out/trace_$dt.json 2> $out/trace_$dt.err
done
for w in 32 64 96 128; do
  timeout -k 10 120 python tools/mlp_trace.py --dtype bfloat16 --wgs $w > $out/trace_bfloat16_w$w.json 2> $out/trace_w$w.err
done
for dt in bfloat16 float32; do
  for f in 1 0; do
    timeout -k 10 200 python bench.py --config jester --dtype $dt --fused-mlp $f > $out/jester_${dt}_f$f.json 2> $out/jester_${dt}_f$f.err
  done
done
