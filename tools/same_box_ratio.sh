# dW kernels against the optimizer stream alone on the same box: the stream probe, then the bench
set -e -o pipefail
O=gpurun_out/samebox; mkdir -p $O
timeout -k 10 120 tools/probes/opt_stream > $O/probe.jsonl
grep '"live": 1' $O/probe.jsonl | grep '"nt": 1' | grep '"shape": "row"'
grep '"copy"' $O/probe.jsonl
timeout -k 10 300 python bench.py --steps 40 --cpu-baseline 0 --rmse 0 --fp32-steps 0 > $O/bench.log 2>&1
grep '^{' $O/bench.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['roofline']['kernel_mean_us'], d['phases_ms'])"
