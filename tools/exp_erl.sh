#!/bin/bash
# epoch row lists with 8 entries per lane in flight: list tests, then the default bench line and its kernel trace
set -e -o pipefail
O=gpurun_out/${1:-erl}; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_rows_dw_gpu.py tests/test_semantics_gpu.py tests/test_fast_step_gpu.py > $O/tests.log 2>&1
tail -1 $O/tests.log
timeout -k 10 300 python bench.py --cpu-baseline 0 > $O/bench.log 2>&1
grep '^{' $O/bench.log | tail -1 > $O/bench.json
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/ks -o ks -- python3 bench.py \
  --steps 20 --warmup 5 --cpu-baseline 0 --rmse 0 --fp32-steps 0 > $O/ks.log 2>&1
echo done
