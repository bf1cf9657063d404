#!/bin/bash
# ML-20M pair launch variants, same box, interleaved: tile form (default), LONG variant forced (entries as
# vectors), 32 parts per tile (rows_small_waves huge), both
set -e
mkdir -p gpurun_out/rv
for r in 1 2; do
  for v in "base:" "long:--rows-long 1" "p32:--rows-small-waves 1000000000" "long_p32:--rows-long 1 --rows-small-waves 1000000000"; do
    name=${v%%:*}; opts=${v#*:}
    timeout -k 10 200 python bench.py $opts --cpu-baseline 0 --fp32-steps 0 --epoch 0 --rmse 0 \
      > gpurun_out/rv/${name}_$r.json 2> gpurun_out/rv/${name}_$r.err
  done
done
