"""bench.py with the row-gather chunk sizes overridden (diagnostic A/B tool):
    python tools/chunk_bench.py BIG SMALL MID -- <bench.py args>"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from omnidirectional_collaborative_filtering_amd import data_reader as DR  # noqa: E402

if __name__ == "__main__":
    i = sys.argv.index("--")
    big, small, mid = (int(x) for x in sys.argv[1:4])
    DR.GATHER_CHUNK, DR.GATHER_CHUNK_SMALL, DR.GATHER_CHUNK_MID = big, small, mid
    sys.argv = ["bench.py"] + sys.argv[i + 1:]
    import bench
    bench.main()
