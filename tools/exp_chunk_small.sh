#!/bin/bash
# A/B of the small-batch gather chunk (data_reader.GATHER_CHUNK_SMALL: 64 vs 96 vs 128 entries) on the small
# BASELINE configs, interleaved -> gpurun_out/<tag>/
set -e -o pipefail
O=gpurun_out/${1:-chunk_small}; mkdir -p $O
run() {   # chunk, name, bench args...
  local c=$1 n=$2; shift 2
  timeout -k 10 200 python -c "
import sys, runpy
import omnidirectional_collaborative_filtering_amd.data_reader as d
d.GATHER_CHUNK_SMALL = $c
sys.argv = ['bench.py'] + sys.argv[1:]
runpy.run_path('bench.py', run_name='__main__')" "$@" > $O/${n}_C$c.json 2>> $O/err.log
  python -c "import json; d=json.loads(open('$O/${n}_C$c.json').read().strip().splitlines()[-1]); print('$n C=$c', d['ms_per_step'], d['phases_ms'])"
}
B="--cpu-baseline 0 --fp32-steps 0 --epoch 0 --rmse 0"
for rep in 1 2; do
  for c in 64 96 128; do
    run $c ml1m --config ml1m --dtype bfloat16 $B
    run $c ml1mu --config ml1m_u --dtype bfloat16 $B
    run $c ml100k --config ml100k --dtype float32 $B
  done
done
