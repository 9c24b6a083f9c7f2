"""GPU timeline summary of a rocprofv3 kernel trace (run_kernel_trace.csv[.gz]): the fraction
of the span in which at least one kernel runs, per-queue busy fractions and idle gaps between
a queue's kernels, and per-kernel-class time. usage: python tools/trace_util.py TRACE_CSV [t0_frac]"""
import sys

import numpy as np
import pandas as pd


def main():
    d = pd.read_csv(sys.argv[1]).sort_values("Start_Timestamp")
    skip = float(sys.argv[2]) if len(sys.argv) > 2 else 0.3   # skip warmup / setup
    # the fit stream only: from the first to the last banded-sweep kernel (engine setup's
    # copies and fills before and after it are not part of it), minus its first `skip` share
    bk = d[d.Kernel_Name.str.contains("band_")]
    t0, t1 = bk.Start_Timestamp.min(), bk.End_Timestamp.max()
    d = d[(d.Start_Timestamp >= t0 + skip * (t1 - t0)) & (d.End_Timestamp <= t1)]
    s, e = d.Start_Timestamp.to_numpy(), d.End_Timestamp.to_numpy()
    span = e.max() - s.min()
    # union of [s, e)
    busy, cur_s, cur_e = 0, s[0], e[0]
    for a, b in zip(s[1:], e[1:]):
        if a > cur_e:
            busy += cur_e - cur_s
            cur_s, cur_e = a, b
        else:
            cur_e = max(cur_e, b)
    busy += cur_e - cur_s
    print(f"span {span / 1e6:.1f} ms, any-kernel busy {busy / span:.3f}")
    for q, g in d.groupby("Queue_Id"):
        gs, ge = g.Start_Timestamp.to_numpy(), g.End_Timestamp.to_numpy()
        gaps = gs[1:] - ge[:-1]
        gaps = gaps[gaps > 0]
        print(f"queue {q}: kernels {len(g)}, busy {np.sum(ge - gs) / span:.3f}, "
              f"gaps > 0.2 ms: {np.sum(gaps > 2e5)}, mean gap {gaps.mean() / 1e6 if len(gaps) else 0:.3f} ms")
    d = d.assign(dur=(d.End_Timestamp - d.Start_Timestamp) / 1e6)
    top = d.groupby("Kernel_Name").dur.agg(["count", "sum", "mean"]).sort_values("sum", ascending=False).head(8)
    print(top.to_string())


if __name__ == "__main__":
    main()
