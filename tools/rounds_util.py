"""Host/device split of the stepped driver's rounds (bench with GPX_TRACE_ROUNDS=1, which writes
rounds_trace.json: per round (group, call start, call end, steps end, finish end, n)).
usage: python tools/rounds_util.py rounds_trace.json"""
import json
import sys

import numpy as np


def main():
    tr = json.load(open(sys.argv[1]))
    ev = np.array([e for t in tr[len(tr) // 3:] for e in t])   # skip the warmup calls
    for g in np.unique(ev[:, 0]):
        e = ev[ev[:, 0] == g]
        e = e[np.argsort(e[:, 1])]
        span = e[-1, 4] - e[0, 1]
        call = np.sum(e[:, 2] - e[:, 1])
        steps = np.sum(e[:, 3] - e[:, 2])
        fin = np.sum(e[:, 4] - e[:, 3])
        gap = np.sum(e[1:, 1] - e[:-1, 4])     # bind + theta of the next round
        print(f"group {int(g)}: rounds {len(e)}, span {span * 1e3:.1f} ms, per round: call {call / len(e) * 1e3:.2f} ms, "
              f"steps {steps / len(e) * 1e3:.2f}, finish {fin / len(e) * 1e3:.2f}, bind+theta {gap / (len(e) - 1) * 1e3:.2f}, "
              f"fits/round {e[:, 5].mean():.0f}")


if __name__ == "__main__":
    main()
