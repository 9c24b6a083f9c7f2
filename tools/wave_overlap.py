"""Cross-process structure of a band16 wave trace (bench.py GPX_WAVE_TRACE=1 GPX_WAVE_TRACE_OUT=f.npz):
how many host processes have sweep wavefronts resident at the same time, and the resident
waves per process. If the GPU ran the processes' kernels concurrently, several processes would
be resident at once most of the time; if it time-slices between processes, mostly one.
usage: python tools/wave_overlap.py trace.npz"""
import sys

import numpy as np

d = np.load(sys.argv[1])
procs = sorted(d.files)
base = min(int(d[p][:, 0].min()) for p in procs if len(d[p]))
ev = []
for k, p in enumerate(procs):
    r = d[p].astype(np.int64)
    r = r[r[:, 2] < 32]
    a, b = r[:, 0] - base, r[:, 1] - base
    ev.append(np.stack([a, np.full_like(a, k), np.ones_like(a)], 1))
    ev.append(np.stack([b, np.full_like(b, k), -np.ones_like(b)], 1))
ev = np.concatenate(ev)
ev = ev[np.lexsort((ev[:, 2], ev[:, 0]))]
t, who, dlt = ev[:, 0], ev[:, 1], ev[:, 2]
P = len(procs)
nproc = np.zeros(len(ev), dtype=np.int32)
for k in range(P):
    nproc += (np.cumsum(np.where(who == k, dlt, 0)) > 0).astype(np.int32)
tot = np.cumsum(dlt)
dt = np.diff(t, append=t[-1]).astype(np.float64)
span = dt.sum()
print(f"processes {P}, records {sum(len(d[p]) for p in procs)}, span {span / 1e8:.3f} s")
for k in range(P + 1):
    sh = dt[nproc == k].sum() / span
    if sh > 0.001:
        m = (tot[nproc == k] * dt[nproc == k]).sum() / max(dt[nproc == k].sum(), 1)
        print(f"  {k} processes resident: {sh:.3f} of the span, mean resident waves then {m:.0f}")
print(f"mean resident waves {(tot * dt).sum() / span:.0f}; mean processes resident {(nproc * dt).sum() / span:.2f}")
