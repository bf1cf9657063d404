#!/bin/bash
# MFMA utilisation evidence (rocprofv3 PMC, one pass per counter group, no other trace domains):
# the Netflix-width step with the encoder over column tiles on the matrix cores (--enc-tiles 1: ocf_encoder_tiles),
# the default ML-20M step, and the Jester step (one ocf_mlp_step launch); per-kernel
# SQ_VALU_MFMA_BUSY_CYCLES, SQ_BUSY_CYCLES, GRBM_GUI_ACTIVE plus a kernel trace for durations
# -> gpurun_out/<tag>/ (reduce with tools/mfma_reduce.py)
set -e -o pipefail
TAG=${1:-mfma}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp
export TMPDIR=/tmp
for cfg in "nf_tiles:--config netflix --enc-tiles 1" "b256:--batch 256" "jester:--config jester --dtype bfloat16"; do
  n=${cfg%%:*}; a=${cfg#*:}
  mkdir -p $O/$n
  timeout -s KILL 200 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv \
    -d $O/$n/pmc -o p -- python3 $R/bench.py --steps 6 --warmup 2 --cpu-baseline 0 --rmse 0 --fp32-steps 0 \
    --phase-timers 0 --configs 0 --epoch 0 $a > $O/$n/pmc.log 2>&1
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$n/ks -o ks -- \
    python3 $R/bench.py --steps 10 --warmup 2 --cpu-baseline 0 --rmse 0 --fp32-steps 0 --configs 0 --epoch 0 $a \
    > $O/$n/ks.log 2>&1
done
echo mfma_counters: done
