set -e -o pipefail
mkdir -p gpurun_out/rs1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/rs1/tests.log 2>&1 || { tail -30 gpurun_out/rs1/tests.log; exit 1; }
tail -2 gpurun_out/rs1/tests.log
timeout -k 10 300 python bench.py --cpu-baseline 0 > gpurun_out/rs1/bench1.log 2>&1
grep '^{' gpurun_out/rs1/bench1.log
timeout -k 10 300 python bench.py --cpu-baseline 0 --rmse 0 --row-skip 0 > gpurun_out/rs1/bench0.log 2>&1
grep '^{' gpurun_out/rs1/bench0.log
