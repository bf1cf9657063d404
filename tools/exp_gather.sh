#!/bin/bash
# Row-gather A/B: bash tools/exp_gather.sh TAG "lib:chunk lib:chunk ..." [bench args]
# (lib "base" = libocf.so; chunk = OCF_GATHER_CHUNK entries per work unit)
set -e -o pipefail
O=gpurun_out/$1; VARS=$2; shift 2
mkdir -p $O
for rep in 1 2; do
  for v in $VARS; do
    lib=${v%%:*}; ch=${v#*:}
    if [ "$lib" = base ]; then unset OCF_LIB_PATH; else export OCF_LIB_PATH=$PWD/omnidirectional_collaborative_filtering_amd/libocf_$lib.so; fi
    OCF_GATHER_CHUNK=$ch timeout -k 10 200 python bench.py --steps 40 --cpu-baseline 0 --rmse 0 --fp32-steps 0 "$@" \
      > $O/bench_${lib}_${ch}_$rep.log 2>&1
    python -c "import json,sys; d=json.loads([l for l in open('$O/bench_${lib}_${ch}_$rep.log') if l.startswith('{')][-1]); print('$v', d['ms_per_step'], {k: round(x, 4) for k, x in d['phases_ms'].items()})"
  done
done
