"""Host-side profile of the bench's fitting loop on the GPU box: cProfile of the fitting steps
(FitWorker.run_steps: model construction, rebinds, device calls, L-BFGS-B steps, predictions) in a
one-process bench run, printed by internal and cumulative time. Series generation and warm-up
are outside the profile.

usage: python tools/prof_host.py [bench args, e.g. --procs 1 --width 1024 --fits 768 --steps 4]"""
import cProfile
import os
import pstats
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

sys.argv = ["bench.py", "--no-cpu-baseline", "--no-secondary", "--steps", "4", "--warmup", "1"] + sys.argv[1:]
pr = cProfile.Profile()
real = bench.FitWorker.run_steps


def run_steps(self, k):
    pr.enable()
    try:
        return real(self, k)
    finally:
        pr.disable()


bench.FitWorker.run_steps = run_steps
bench.main()
st = pstats.Stats(pr)
st.sort_stats("tottime").print_stats(45)
st.sort_stats("cumtime").print_stats(45)
