"""cProfile of bench.py's rank process (the one-thread L-BFGS-B driver runs on its main thread):
python tools/prof_bench_host.py OUT.pstats -- <bench args>; prints the top cumulative entries."""
import cProfile
import os
import pstats
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
out = sys.argv[1]
sys.argv = ["bench.py"] + sys.argv[3:]
import bench  # noqa: E402

cProfile.run("bench.main()", out)
st = pstats.Stats(out)
st.sort_stats("tottime").print_stats(40)
