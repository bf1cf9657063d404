# Which calls issue PyTorch fill kernels in bench.py (torch.profiler, parent ops with Python stacks)
import sys, collections
sys.argv = ["bench.py", "--steps", "12", "--warmup", "3", "--cpu-baseline", "0", "--rmse", "0", "--fp32-steps", "0"]
sys.path.insert(0, ".")
import torch
from torch.profiler import ProfilerActivity, profile
import bench
with profile(activities=[ProfilerActivity.CPU], with_stack=True) as prof:
    bench.main()
c = collections.Counter()
for ev in prof.events():
    if ev.name in ("aten::fill_", "aten::zero_"):
        chain, p = [], ev.cpu_parent
        while p is not None and len(chain) < 4:
            chain.append(p.name)
            st = [str(s) for s in p.stack[:5]]
            if st:
                chain.append(st)
                break
            p = p.cpu_parent
        c[(ev.name, str(chain))] += 1
for (n, st), k in c.most_common(12):
    print(k, n, st)
