"""Per-kernel MFMA utilisation from tools/mfma_counters.sh's PMC pass (diagnostic tool).

Usage: python tools/mfma_reduce.py gpurun_out/<tag> OUT.json

Per dispatch the counters are summed over their instances (XCDs / SEs); per kernel: mean kernel cycles =
GRBM_GUI_ACTIVE / 8 (the counter sums the 8 XCDs), MFMA utilisation = SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x
kernel cycles), MFMA instructions = busy cycles / 32 (v_mfma_*_32x32x16 and 32x32x2f32 occupy the unit 32
cycles per instruction per the microarch guide)."""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def reduce_dir(d):
    files = glob.glob(os.path.join(d, "pmc", "**", "*counter_collection.csv"), recursive=True)
    if not files:
        return None
    per = defaultdict(lambda: defaultdict(float))
    name = {}
    for r in csv.DictReader(open(files[0])):
        k = int(r["Dispatch_Id"])
        per[k][r["Counter_Name"]] += float(r["Counter_Value"])
        name[k] = r["Kernel_Name"]
    out = defaultdict(lambda: {"launches": 0, "kernel_cycles": 0.0, "mfma_busy_cycles": 0.0})
    for k, c in per.items():
        o = out[name[k][:120]]
        o["launches"] += 1
        o["kernel_cycles"] += c.get("GRBM_GUI_ACTIVE", 0.0) / 8
        o["mfma_busy_cycles"] += c.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0)
    res = {}
    for n, o in out.items():
        kc = o["kernel_cycles"] / o["launches"]
        mb = o["mfma_busy_cycles"] / o["launches"]
        res[n] = {"launches": o["launches"], "kernel_cycles": round(kc), "mfma_busy_cycles": round(mb),
                  "mfma_instructions": round(mb / 32), "mfma_util": round(mb / (1024 * kc), 4) if kc else 0.0}
    return res


def main():
    root, dst = sys.argv[1], sys.argv[2]
    res = {"note": __doc__.split("\n\n")[1].replace("\n", " "), "workloads": {}}
    for d in sorted(glob.glob(os.path.join(root, "*"))):
        r = reduce_dir(d)
        if r is not None:
            res["workloads"][os.path.basename(d)] = r
    with open(dst, "w") as f:
        json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
