#!/bin/bash
# Round evidence on one MI355X (run through gpurun from the repo root):
#   bash tools/profile_round.sh r01 [extra bench args...]
# 1) GPU test suite, 2) the default bench line, 3) rocprofv3 --kernel-trace --stats of the same
# bench, 4) two PMC passes (FETCH_SIZE, WRITE_SIZE; counters only, no other trace domains) reduced to
# per-phase HBM bytes by tools/pmc_traffic.py.  Outputs under gpurun_out/<tag>/; the summaries to
# commit are copied to profiles/<tag>_*.  Every GPU step has its own time limit; the first failure
# ends the script.
set -e -o pipefail
TAG=${1:?round tag, e.g. r01}
shift || true
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$O/tests.log" 2>&1
  tail -3 "$O/tests.log"
fi
timeout -k 10 400 python bench.py "$@" > "$O/bench.log" 2>&1
grep '^{' "$O/bench.log" | tail -1 > "$O/bench.json"
cat "$O/bench.json"
cd /tmp
export TMPDIR=/tmp
BARGS="--steps 20 --warmup 5 --cpu-baseline 0 --rmse 0 --fp32-steps 0"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/ks" -o ks -- \
  python3 "$R/bench.py" $BARGS "$@" > "$O/ks.log" 2>&1
BARGS_PMC="--steps 10 --warmup 2 --cpu-baseline 0 --rmse 0 --phase-timers 0 --fp32-steps 0"
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$O/pf" -o f -- \
  python3 "$R/bench.py" $BARGS_PMC "$@" > "$O/pf.log" 2>&1
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$O/pw" -o w -- \
  python3 "$R/bench.py" $BARGS_PMC "$@" > "$O/pw.log" 2>&1
cd "$R"
python tools/pmc_traffic.py "$(find "$O/pf" -name '*counter_collection.csv' | head -1)" \
  "$(find "$O/pw" -name '*counter_collection.csv' | head -1)" "$O/pmc_traffic.json"
cp "$(find "$O/ks" -name '*kernel_stats.csv' | head -1)" "$O/kernel_stats.csv"
echo "profile_round: done"
