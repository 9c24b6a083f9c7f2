"""C2 fit fixtures in distribution: the oracle's whole `Scipy().minimize(maxiter=100)` fit on many
seeds, so the device's fitted results AND its evaluation count per fit (fits/s ∝ 1/nfev) can be
compared with the oracle's over a population rather than on two seeds.

Protocol: GPR/model_trainer.py:15-20 (GPflow defaults σ² = ℓ = 1, σn² = 1e-5 fixed, L-BFGS-B
maxiter 100). Inputs: the C2 generator (oracle.synthetic_series, X = day offsets 0..N-1), seed s.

Run in the build container (nothing here reads /root/reference; ~15 min for N=2048 x 64 seeds,
~1 h for N=4096 x 32 seeds on 8 cores):

    python tests/golden/make_c2_dist_golden.py [--n 2048] [--seeds 64]

Writes tests/golden/c2_dist_n<N>.npz: seeds, loss [S], x [S, 2] (u*), theta [S, 2] (ℓ*, σ²*),
nfev [S], nit [S]. The series are regenerated from the seed by the tests (the generator is
restated in bench.py), so the fixture holds only the fit results.
"""
from __future__ import annotations

import argparse
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)
from oracle import gp_oracle as O  # noqa: E402

NOISE = 1e-5


def fit(n, seed):
    x, y = O.synthetic_series(n, seed)
    k = O.OSquaredExponential()
    m = O.OGPR(x, y, k, noise_variance=NOISE)
    m.noise.trainable = False
    r = O.scipy_minimize(m, 100)
    return r, np.array([p.value for p in k.params()])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=2048)
    ap.add_argument("--seeds", type=int, default=64)
    a = ap.parse_args()
    out_path = os.path.join(HERE, f"c2_dist_n{a.n}.npz")
    rows = []
    t0 = time.time()
    for s in range(a.seeds):
        r, th = fit(a.n, s)
        rows.append((s, r.fun, r.x, th, r.nfev, r.nit))
        print(f"N={a.n} seed {s}: loss {r.fun:.12g} theta {th} nfev {r.nfev} nit {r.nit} ({time.time() - t0:.0f} s)",
              flush=True)
        # written after every fit: a long run that is stopped keeps what it has
        np.savez_compressed(out_path, n=np.array([a.n]), noise=np.array([NOISE]),
                            seeds=np.array([q[0] for q in rows]), loss=np.array([q[1] for q in rows]),
                            x=np.array([q[2] for q in rows]), theta=np.array([q[3] for q in rows]),
                            nfev=np.array([q[4] for q in rows]), nit=np.array([q[5] for q in rows]))
    nf = np.array([q[4] for q in rows], dtype=np.float64)
    print(f"N={a.n}: {len(rows)} fits, nfev mean {nf.mean():.2f} (std {nf.std(ddof=1):.2f})")


if __name__ == "__main__":
    main()
