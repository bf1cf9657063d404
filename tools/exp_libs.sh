#!/bin/bash
# bench.py A/B over variant builds: bash tools/exp_libs.sh TAG "bench args" lib1 lib2 ...  (lib "base" = libocf.so)
set -e -o pipefail
O=gpurun_out/$1; ARGS=$2; shift 2
mkdir -p $O
for rep in 1 2; do
  for lib in "$@"; do
    if [ "$lib" = base ]; then unset OCF_LIB_PATH; else export OCF_LIB_PATH=$PWD/omnidirectional_collaborative_filtering_amd/libocf_$lib.so; fi
    timeout -k 10 200 python bench.py --steps 40 --cpu-baseline 0 --rmse 0 $ARGS > $O/bench_${lib}_$rep.log 2>&1
    python -c "import json,sys; d=json.loads([l for l in open('$O/bench_${lib}_$rep.log') if l.startswith('{')][-1]); print('$lib', d['ms_per_step'], d['phases_ms'])"
  done
done
