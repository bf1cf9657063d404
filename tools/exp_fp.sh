#!/bin/bash
# feature-parallel rank steps emulated on one GPU (bench --emulate-shards G: rank 0 of a G-way job, its
# collective code path with no-op collectives); each rank's weight gradients by the row-stream kernel
set -e -o pipefail
O=gpurun_out/${1:-fp}
mkdir -p $O
for G in 2 4 8; do
  for sd in -1; do
    timeout -k 10 200 python bench.py --steps 30 --cpu-baseline 0 --rmse 0 --emulate-shards $G --sparse-dw $sd > $O/fp_${G}_$sd.log 2>&1
    python -c "import json; d=json.loads([l for l in open('$O/fp_${G}_$sd.log') if l.startswith('{')][-1]); print('G=$G sparse_dw=$sd', d['ms_per_step'], d['phases_ms'])"
  done
done
