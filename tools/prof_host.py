"""Host-side profile of the bench's fitting loop on the GPU box: cProfile of one timed step
(group 0's thread, i.e. the main thread), printed by cumulative and internal time."""
import cProfile
import os
import pstats
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

sys.argv = ["bench.py", "--no-cpu-baseline", "--steps", "1", "--warmup", "1"] + sys.argv[1:]
pr = cProfile.Profile()
pr.enable()
bench.main()
pr.disable()
st = pstats.Stats(pr)
st.sort_stats("tottime").print_stats(30)
st.sort_stats("cumtime").print_stats(30)
