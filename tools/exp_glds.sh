#!/bin/bash
# LDS-DMA staging of the row-stream kernel's parameter / slot loads (OCF_RS_GLDS, libocf.so) vs register
# staging (libocf_reg.so): the row kernels' bit-identity tests, then the ML-20M / ML-1M benches A/B
set -e -o pipefail
O=gpurun_out/glds; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_rows_dw_gpu.py \
  tests/test_pair_sync_gpu.py tests/test_fast_step_gpu.py tests/test_optim_ws_gpu.py > $O/tests.log 2>&1
bash tools/exp_libs.sh glds_ml20m "--fp32-steps 0" base reg
bash tools/exp_libs.sh glds_ml1m "--config ml1m --dtype bfloat16 --fp32-steps 0" base reg
