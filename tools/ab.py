"""Interleaved same-box A/B of bench.py variants (run on the GPU box from the repo root, through gpurun).

    python tools/ab.py --tag dual_large --reps 3 [--common "--steps 40"] \
        "pair|" "dual|--rows-dual-large 1 --reduce-in-decoder 1" "glds|OCF_LIB_PATH=/path/libocf_x.so"

A variant is "label|[VAR=value ...] [bench args ...]".  Every variant runs --reps times, interleaved (rep 1 of
every variant, then rep 2, ...), so box drift hits all of them alike.  One JSON line per run goes to
gpurun_out/ab/<tag>.jsonl (ms/step, the dominant kernel's event mean and frac, the warm-up phases); the
summary (medians) is printed and written to gpurun_out/ab/<tag>_summary.json.  A failing run ends the
script (no retries).  The bench's side legs (CPU baseline, test RMSE, fp32 mode, full epoch) are off unless
a variant turns them back on.  A variant's OCF_TUNING="key=value,..." is passed by bench.py to ocf_set_tuning
before any launch (e.g. "long1|OCF_TUNING=rows_long=1").
"""
import argparse
import json
import os
import shlex
import statistics
import subprocess
import sys

QUIET = ["--cpu-baseline", "0", "--rmse", "0", "--fp32-steps", "0", "--epoch", "0"]


def parse_variant(v):
    lab, _, rest = v.partition("|")
    env, args = {}, []
    for t in shlex.split(rest):
        if not args and "=" in t and not t.startswith("--"):
            k, _, val = t.partition("=")
            env[k] = val
        else:
            args.append(t)
    return lab, env, args


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tag", required=True)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--common", default="")
    ap.add_argument("--timeout", type=int, default=300)
    ap.add_argument("--script", default="bench.py", help="the program each variant runs (its last line: JSON)")
    ap.add_argument("variants", nargs="+")
    a = ap.parse_args()
    out = os.path.join("gpurun_out", "ab")
    os.makedirs(out, exist_ok=True)
    path = os.path.join(out, a.tag + ".jsonl")
    vs = [parse_variant(v) for v in a.variants]
    res = {lab: [] for lab, _, _ in vs}
    with open(path, "a") as f:
        for rep in range(a.reps):
            for lab, env, args in vs:
                cmd = ["timeout", "-k", "10", str(a.timeout), sys.executable, "-u", a.script] + \
                      (QUIET if a.script == "bench.py" else []) + shlex.split(a.common) + args
                e = dict(os.environ, **env)
                r = subprocess.run(cmd, env=e, capture_output=True, text=True)
                lines = [x for x in r.stdout.splitlines() if x.startswith("{")]
                if r.returncode != 0 or not lines:
                    sys.stdout.write(r.stdout[-2000:] + r.stderr[-3000:])
                    print("FAILED: %s rep %d rc %d" % (lab, rep, r.returncode), flush=True)
                    sys.exit(1)
                d = json.loads(lines[-1])
                roof = d.get("roofline") or {}
                rec = {"tag": a.tag, "label": lab, "rep": rep, "ms_per_step": d.get("ms_per_step"),
                       "kernel": roof.get("kernel"), "kernel_mean_us": roof.get("kernel_mean_us"),
                       "frac": roof.get("frac"), "phases_ms": d.get("phases_ms"), "args": args, "env": env,
                       "extra": {k: d[k] for k in ("configs", "masked_rmse", "value", "window_host_us") if k in d}}
                f.write(json.dumps(rec) + "\n")
                f.flush()
                res[lab].append(rec)
                print("%-14s rep %d  %.4f ms/step  %s %s us  frac %s" % (lab, rep, rec["ms_per_step"] or -1,
                                                                       rec["kernel"], rec["kernel_mean_us"],
                                                                       rec["frac"]), flush=True)
    summ = {}
    for lab, recs in res.items():
        ms = [r["ms_per_step"] for r in recs]
        ku = [r["kernel_mean_us"] for r in recs if r["kernel_mean_us"] is not None]
        summ[lab] = {"ms_median": statistics.median(ms), "ms": ms,
                     "kernel_us_median": statistics.median(ku) if ku else None, "kernel_us": ku}
        print("%-14s median %.4f ms/step  kernel %s us   %s" % (lab, summ[lab]["ms_median"],
                                                               summ[lab]["kernel_us_median"], ms))
    with open(os.path.join(out, a.tag + "_summary.json"), "w") as f:
        json.dump(summ, f, indent=1)


if __name__ == "__main__":
    main()
