# PARTS 12 (in-tree) against 8 on the other workloads: Netflix width, B = 4,096, an 8-way feature-parallel rank
set -e -o pipefail
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_rows_dw_gpu.py > gpurun_out/parts_tests.log 2>&1 && tail -1 gpurun_out/parts_tests.log
for a in "nf:--config netflix --steps 15" "b4k:--batch 4096 --steps 10" "fp8:--emulate-shards 8 --steps 30"; do
  n=${a%%:*}; x=${a#*:}
  for lib in base p8; do
    if [ "$lib" = base ]; then unset OCF_LIB_PATH; else export OCF_LIB_PATH=$PWD/omnidirectional_collaborative_filtering_amd/libocf_$lib.so; fi
    timeout -k 10 300 python bench.py $x --cpu-baseline 0 --rmse 0 --fp32-steps 0 > gpurun_out/parts_${n}_$lib.log 2>&1
    grep '^{' gpurun_out/parts_${n}_$lib.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$n $lib', d['ms_per_step'])"
  done
done
