#!/bin/bash
# Rehearse bench.py's N>1 path (the driver's SCALE job) on ONE GPU: 2 ranks on device 0 over gloo
# (OCF_REHEARSAL=1, parallel.init_from_env), both layouts.  Correctness of the multi-rank code path only:
# the collectives are host-staged gloo, so the timings say nothing about RCCL over xGMI.
# usage (GPU box): bash tools/rehearse_multi.sh gpurun_out/<dir> [layouts] [extra bench args...]
#   e.g. bash tools/rehearse_multi.sh gpurun_out/rh_nf "feature dp" --config netflix --steps 4 --warmup 1
set -o pipefail
out=${1:-gpurun_out/rehearse}
layouts=${2:-"feature dp"}
shift 2 2>/dev/null
extra=("$@")
[ ${#extra[@]} -eq 0 ] && extra=(--steps 8 --warmup 2)
mkdir -p "$out"
export OCF_REHEARSAL=1
port=29531
for par in $layouts; do
    timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
        --master-port $port bench.py --gpus 2 --parallel $par "${extra[@]}" \
        > "$out/bench_$par.json" 2> "$out/bench_$par.err" || { echo "rehearsal $par failed: $?"; tail -5 "$out/bench_$par.err"; exit 1; }
    port=$((port + 1))
    cat "$out/bench_$par.json"
done
