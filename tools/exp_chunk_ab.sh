#!/bin/bash
# same-box A/B of the mid-size gather chunk (data_reader.GATHER_CHUNK_MID 64 = off, 96 = on) on ML-1M bf16
set -e -o pipefail
O=gpurun_out/${1:-chunk_ab}; mkdir -p $O
for rep in 1 2 3; do
  for c in 64 96; do
    timeout -k 10 200 python -c "
import sys, runpy
import omnidirectional_collaborative_filtering_amd.data_reader as d
d.GATHER_CHUNK_MID = $c
sys.argv = ['bench.py'] + sys.argv[1:]
runpy.run_path('bench.py', run_name='__main__')" --config ml1m --dtype bfloat16 --cpu-baseline 0 --fp32-steps 0 --epoch 0 --rmse 0 \
      > $O/ml1m_M${c}_$rep.json 2>> $O/err.log
    python -c "import json; d=json.loads(open('$O/ml1m_M${c}_$rep.json').read().strip().splitlines()[-1]); print('M=$c rep $rep', d['ms_per_step'], d['phases_ms'])"
  done
done
