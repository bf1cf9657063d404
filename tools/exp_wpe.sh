# Row-stream dW kernel register budget (OCF_RS_WPE, ocf_rows_dw.h): in-tree build (75 VGPRs, 6 waves/SIMD)
# against 7 and 8 waves per SIMD (libocf_w7.so / libocf_w8.so), same box, interleaved ML-20M bench runs
set -e -o pipefail
O=gpurun_out/wpe; mkdir -p $O
for lib in w8 w7; do
  OCF_LIB_PATH=$PWD/omnidirectional_collaborative_filtering_amd/libocf_$lib.so timeout -k 10 200 \
    python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_rows_dw_gpu.py > $O/tests_$lib.log 2>&1
  tail -1 $O/tests_$lib.log
done
for rep in 1 2; do
  for lib in base w7 w8; do
    if [ "$lib" = base ]; then unset OCF_LIB_PATH; else export OCF_LIB_PATH=$PWD/omnidirectional_collaborative_filtering_amd/libocf_$lib.so; fi
    timeout -k 10 200 python bench.py --cpu-baseline 0 --rmse 0 --fp32-steps 0 --steps 60 > $O/b_${lib}_$rep.log 2>&1
    grep '^{' $O/b_${lib}_$rep.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$lib $rep', d['ms_per_step'], d['phases_ms'].get('dW_out'), d['phases_ms'].get('dW_in'))"
  done
done
