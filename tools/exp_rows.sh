#!/bin/bash
# A/B of the row-stream dW kernel (ocf_rows_dw.h) against the role-split MFMA kernel on the ML-20M step.
set -e -o pipefail
O=gpurun_out/${1:-rows}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_rows_dw_gpu.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
tail -2 $O/tests.log
for r in 0 1 0 1; do
  timeout -k 10 200 python bench.py --steps 40 --cpu-baseline 0 --rmse 0 --dw-rows $r > $O/bench_$r.log 2>&1
  python -c "import json,sys; d=json.loads([l for l in open('$O/bench_$r.log') if l.startswith('{')][-1]); print('dw_rows=$r', d['ms_per_step'], d['phases_ms'], d['roofline']['kernel_mean_us'])"
done
