"""Per-call device timeline of each host process from a wave trace with stream-order markers
(bench.py GPX_WAVE_TRACE=1 GPX_WAVE_TRACE_OUT=f.npz; markers from gpx_api.hip trace_mark):
  38 submit reached the device   39 rebind gather done   40 band16 work starts
  43 a lane's K band built       41 lanes joined         42 reduce done   44 results downloaded
and the band16 waves (kind < 32) between them. Prints the median time of each segment per call
and the gap from one call's download to the next call's submit (the host's share).
usage: python tools/call_timeline.py trace.npz"""
import sys

import numpy as np

d = np.load(sys.argv[1])
HZ = 1e8
rows = []
for p in sorted(d.files):
    r = d[p].astype(np.int64)
    mk = r[r[:, 2] >= 32]
    mk = mk[np.argsort(mk[:, 0], kind="stable")]
    wv = r[r[:, 2] < 32]
    ws = np.sort(wv[:, 0])
    we = np.sort(wv[:, 1])
    t38 = mk[mk[:, 2] == 38][:, 0]
    for i in range(len(t38) - 1):
        a, b = t38[i], t38[i + 1]
        seg = mk[(mk[:, 0] >= a) & (mk[:, 0] < b)]
        get = lambda k: seg[seg[:, 2] == k][:, 0]
        t39, t40, t41, t42, t44, t43 = get(39), get(40), get(41), get(42), get(44), get(43)
        if not (len(t39) and len(t40) and len(t41) and len(t42) and len(t44)):
            continue
        i0, i1 = np.searchsorted(ws, t40[0]), np.searchsorted(ws, t41[0])
        first_wave = ws[i0] if i1 > i0 else t41[0]
        last_end = we[np.searchsorted(we, t41[0]) - 1] if i1 > i0 else t40[0]
        rows.append([t39[0] - a, t40[0] - t39[0], (t43.max() - t40[0]) if len(t43) else 0, first_wave - t40[0],
                     last_end - first_wave, t41[0] - last_end, t42[0] - t41[0], t44[0] - t42[0], b - t44[0], b - a])
rows = np.array(rows, dtype=np.float64) / HZ * 1e3
names = ["submit->gather done", "gather->band16 start", "K build (longest lane)", "band16 start->first wave",
         "first wave->last wave end", "last wave->lanes joined", "reduce", "download", "download->next submit (host)",
         "call to call"]
print(f"calls {len(rows)} over {len(d.files)} processes (ms: median / mean / p90)")
for k, nm in enumerate(names):
    c = rows[:, k]
    print(f"  {nm:32s} {np.median(c):8.3f} {c.mean():8.3f} {np.percentile(c, 90):8.3f}")
