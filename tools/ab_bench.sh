#!/bin/bash
# Interleaved A/B of bench.py variants on one GPU box (run through gpurun from the repo root):
#   bash tools/ab_bench.sh REPS "label1|[VAR=value ...] [--bench-arg value ...]" "label2|..." ...
# Each variant runs REPS times, interleaved; prints ms/step per run and the median.
set -e -o pipefail
REPS=$1; shift
O=gpurun_out/ab; mkdir -p $O
declare -A RES
for r in $(seq $REPS); do
  for v in "$@"; do
    lab=${v%%|*}; rest=${v#*|}
    envs=(); args=()
    for t in $rest; do if [[ ${#args[@]} -eq 0 && $t == *=* && $t != --* ]]; then envs+=("$t"); else args+=("$t"); fi; done
    env "${envs[@]}" timeout -k 10 300 python bench.py --cpu-baseline 0 --rmse 0 "${args[@]}" > $O/b.log 2>&1 || { tail -5 $O/b.log; exit 1; }
    ms=$(grep '^{' $O/b.log | python -c "import json,sys; print(json.loads(sys.stdin.read())['ms_per_step'])")
    RES[$lab]="${RES[$lab]} $ms"
    echo "$lab $ms"
  done
done
for v in "$@"; do lab=${v%%|*}; echo "$lab median $(echo ${RES[$lab]} | tr ' ' '\n' | sort -n | awk '{a[NR]=$1} END{print a[int((NR+1)/2)]}') :${RES[$lab]}"; done
