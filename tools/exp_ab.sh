# same-box A/B of the in-tree libocf.so against libocf_<variant>.so: bash tools/exp_ab.sh TAG variant [bench args]
set -e -o pipefail
O=gpurun_out/$1; V=$2; shift 2
mkdir -p $O
for rep in 1 2 3; do
  for lib in base $V; do
    if [ "$lib" = base ]; then unset OCF_LIB_PATH; else export OCF_LIB_PATH=$PWD/omnidirectional_collaborative_filtering_amd/libocf_$lib.so; fi
    timeout -k 10 200 python bench.py --steps 40 --cpu-baseline 0 --rmse 0 --fp32-steps 0 "$@" > $O/${lib}_$rep.log 2>&1
    grep '^{' $O/${lib}_$rep.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$lib', d['ms_per_step'], d['roofline']['kernel_mean_us'], d['phases_ms']['enc_gemm'], d['phases_ms']['dec_gemm_mse'], d['phases_ms']['dW_out'], d['phases_ms']['dW_in'])"
  done
done
