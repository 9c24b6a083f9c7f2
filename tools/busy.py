"""GPU occupancy of a rocprofv3 kernel trace (rocpd SQLite db): union of kernel intervals,
idle gaps and how the busy time splits into 1 / 2+ concurrent kernels, over the whole trace
or the last `--tail` seconds (the bench's timed region sits at the end of its run).

usage: python tools/busy.py gpurun_out/x/prof/run_results.db [--tail 6.0]
"""
import argparse
import sqlite3
from collections import defaultdict

ap = argparse.ArgumentParser()
ap.add_argument("db")
ap.add_argument("--tail", type=float, default=0.0, help="only the last TAIL seconds of the trace")
ap.add_argument("--skip-tail", type=float, default=0.0, help="drop the last SKIP seconds first")
args = ap.parse_args()

c = sqlite3.connect(args.db)
ev = c.execute("select start, end, name from kernels order by start").fetchall()
t_end = max(e for _, e, _ in ev) - args.skip_tail * 1e9
t_beg = t_end - args.tail * 1e9 if args.tail > 0 else min(s for s, _, _ in ev)
ev = [(max(s, t_beg), min(e, t_end), n) for s, e, n in ev if e > t_beg and s < t_end]

# sweep: +1 at start, -1 at end
pts = sorted([(s, 1, n) for s, _, n in ev] + [(e, -1, n) for _, e, n in ev], key=lambda p: (p[0], p[1]))
active = defaultdict(int)
depth = 0
last = t_beg
busy = excl = 0.0
excl_by = defaultdict(float)
gaps = []
for t, d, n in pts:
    dt = t - last
    if depth > 0:
        busy += dt
        if depth == 1:
            excl += dt
            (k,) = [k for k, v in active.items() if v > 0]
            excl_by[k] += dt
    elif dt > 0:
        gaps.append(dt)
    active[n] += d
    depth += d
    last = t
span = t_end - t_beg
print(f"window {span/1e9:.3f} s  busy {busy/span:.3f}  idle {1-busy/span:.3f}  "
      f"one-kernel {excl/span:.3f}  overlapped {(busy-excl)/span:.3f}")
gaps.sort(reverse=True)
print(f"idle gaps: {len(gaps)}  total {sum(gaps)/1e6:.1f} ms  largest {[round(g/1e3) for g in gaps[:8]]} us")
print("time with ONLY this kernel running (fraction of window):")
for k, v in sorted(excl_by.items(), key=lambda kv: -kv[1])[:12]:
    print(f"  {v/span:6.3f}  {k[:90]}")
