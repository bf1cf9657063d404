# large-batch steps: default dW path vs the row-stream kernel forced (--sparse-dw 1) -> gpurun_out/bigb/
set -e -o pipefail
O=gpurun_out/bigb; mkdir -p $O
for B in 2048 4096; do
  for sd in -1 1; do
    timeout -k 10 300 python bench.py --batch $B --sparse-dw $sd --steps 10 --warmup 3 --cpu-baseline 0 --rmse 0 --fp32-steps 0 > $O/b${B}_$sd.log 2>&1
    grep '^{' $O/b${B}_$sd.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('B $B sparse_dw $sd', d['ms_per_step'], d['value'], d['phases_ms'])"
  done
done
