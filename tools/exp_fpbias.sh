#!/bin/bash
# feature-parallel rank step with the hidden-bias update folded into dW_in + the batched bias_opt_partials
# kernel: parity tests, then emulated G = 2 / 4 / 8 rank steps and their kernel trace -> gpurun_out/<tag>/
set -e -o pipefail
O=gpurun_out/${1:-fpbias}; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_feature_parallel_gpu.py tests/test_dp_gpu.py tests/test_train_gpu.py > $O/tests.log 2>&1
tail -1 $O/tests.log
bash tools/exp_fp.sh ${1:-fpbias}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof8 -o run -- python3 bench.py \
  --cpu-baseline 0 --fp32-steps 0 --epoch 0 --rmse 0 --phase-timers 0 --emulate-shards 8 > $O/prof8.json 2> $O/prof8.err
echo prof done
