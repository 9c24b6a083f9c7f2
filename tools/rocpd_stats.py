"""Kernel statistics from a rocprofv3 rocpd database (run_results.db): per kernel name the total,
count and average duration, and optionally the dispatch sequence of one call window (start,
duration, gap to the previous kernel's end) — where a latency chain's time goes.

usage: python tools/rocpd_stats.py DB [--csv OUT] [--seq N] [--match SUBSTR]"""
import argparse
import collections
import csv
import sqlite3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--csv", default=None, help="write the per-kernel summary here")
    ap.add_argument("--seq", type=int, default=0, help="print N consecutive dispatches from the last --match one")
    ap.add_argument("--match", default="bcr_fwd_kernel", help="kernel name that starts a printed sequence")
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    rows = list(c.execute("select name, start, end, grid_x, grid_y, workgroup_x from kernels order by start"))
    agg = collections.defaultdict(list)
    for n, s, e, *_ in rows:
        agg[n].append(e - s)
    tot = sum(sum(v) for v in agg.values())
    out = []
    for n, v in sorted(agg.items(), key=lambda kv: -sum(kv[1])):
        out.append((n, len(v), sum(v) / 1e6, sum(v) / len(v) / 1e3, sum(v) / tot))
        print(f"{sum(v) / 1e6:10.3f} ms {len(v):7d} x {sum(v) / len(v) / 1e3:9.2f} us {100 * sum(v) / tot:5.1f}%  {n[:100]}")
    if a.csv:
        with open(a.csv, "w", newline="") as f:
            w = csv.writer(f)
            w.writerow(["kernel", "calls", "total_ms", "avg_us", "fraction"])
            w.writerows(out)
    if a.seq:
        idx = [i for i, r in enumerate(rows) if a.match in r[0]]
        if idx:
            # the last complete window: walk back from the end to a dispatch of `match` at level 0
            i0 = idx[-1]
            while i0 > 0 and a.match in rows[i0 - 1][0]:
                i0 -= 1
            i0 = max(0, i0)
            prev_end = rows[i0][1]
            t0 = rows[i0][1]
            for n, s, e, gx, gy, wx in rows[i0:i0 + a.seq]:
                print(f"{(s - t0) / 1e3:9.2f} us  dur {(e - s) / 1e3:8.2f}  gap {(s - prev_end) / 1e3:7.2f}  "
                      f"grid {gx // max(wx, 1)}x{gy}  {n[:70]}")
                prev_end = e


if __name__ == "__main__":
    main()
