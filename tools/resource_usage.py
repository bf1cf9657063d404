"""Summarise hipcc -Rpass-analysis=kernel-resource-usage output (make -C .../csrc asm)."""
import re
import sys

path = sys.argv[1] if len(sys.argv) > 1 else \
    "omnidirectional_collaborative_filtering_amd/csrc/build/asm/ocf_gemm.resource.txt"
rows, cur = [], None
for line in open(path):
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        cur = {"name": m.group(1)}
        rows.append(cur)
        continue
    for key, lab in (("VGPRs:", "v"), ("AGPRs:", "a"), ("ScratchSize", "scr"), ("Occupancy", "occ"),
                     ("LDS Size", "lds")):
        if cur is not None and key in line:
            cur[lab] = line.split(":")[-1].split("[")[0].strip()
for r in rows:
    n = r["name"]
    n = re.sub(r"_ZN3ocf11gemm_kernelI", "gemm<", n)[:60]
    print("%-60s v=%-4s a=%-4s scr=%-4s occ=%-2s lds=%s" % (n, r.get("v"), r.get("a"), r.get("scr"), r.get("occ"),
                                                          r.get("lds")))
