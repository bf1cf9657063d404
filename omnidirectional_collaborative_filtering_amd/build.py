"""Build libocf.so (gfx950) in-tree: ``python -m omnidirectional_collaborative_filtering_amd.build``."""
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))


def build(jobs=8, verbose=False):
    csrc = os.path.join(HERE, "csrc")
    cmd = ["make", "-C", csrc, "-j%d" % jobs]
    r = subprocess.run(cmd, capture_output=not verbose, text=True)
    if r.returncode != 0:
        sys.stderr.write((r.stdout or "") + (r.stderr or ""))
        raise RuntimeError("libocf build failed")
    return os.path.join(HERE, "libocf.so")


if __name__ == "__main__":
    print(build(verbose=True))
