"""A large C2 fit population for the nfev-in-distribution check:
whole fits of the headline protocol (GPR/model_trainer.py:15-20: GPflow defaults, σn² = 1e-5
fixed, L-BFGS-B maxiter 100) on many C2 seeds, evaluated by oracle/band_oracle.py — the band
algorithm restated on numpy/LAPACK, pinned to the dense GPflow-form oracle at evaluation level
(tests/test_band_oracle.py, ≤ 1e-9) and ~300x faster at N = 4096, so hundreds of seeds fit in
minutes where the dense oracle needs ~80 s per fit.

Why a population: near C2's flat optimum L-BFGS-B's stop test reacts to 1e-9-level differences
of summation order, so WHICH fits take 40+ evaluations instead of ~15 changes between any two
correct implementations (dense oracle vs band oracle vs device, tests/golden/c2_dist_n4096.npz);
only the mean over many seeds is a stable quantity (fits/s ∝ 1/nfev).

    python tests/golden/make_c2_dist_band_golden.py [--n 4096] [--seeds 512] [--procs 8]

Writes tests/golden/c2_dist_band_n<N>.npz: seeds, loss, x (u*), theta (ℓ*, σ²*), nfev.
"""
from __future__ import annotations

import argparse
import multiprocessing as mp
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)

SEED0 = 5000  # (disjoint from the bench's seeds and from c2_dist_n4096.npz's)


def _fit(args):
    n, s = args
    import threadpoolctl
    from oracle import band_oracle as B
    from oracle import gp_oracle as O
    from oracle.gp_oracle import softplus
    with threadpoolctl.threadpool_limits(limits=1):
        x, y = O.synthetic_series(n, s)
        fun, u, nfev = B.fit(x, y, 1e-5, 100)
    return s, fun, u, np.array([float(softplus(u[0])), float(softplus(u[1]))]), nfev


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=4096)
    ap.add_argument("--seeds", type=int, default=512)
    ap.add_argument("--procs", type=int, default=8)
    a = ap.parse_args()
    t0 = time.time()
    with mp.get_context("spawn").Pool(a.procs) as pool:
        rows = pool.map(_fit, [(a.n, SEED0 + i) for i in range(a.seeds)], chunksize=4)
    out = os.path.join(HERE, f"c2_dist_band_n{a.n}.npz")
    np.savez_compressed(out, n=np.array([a.n]), noise=np.array([1e-5]), seeds=np.array([r[0] for r in rows]),
                        loss=np.array([r[1] for r in rows]), x=np.array([r[2] for r in rows]),
                        theta=np.array([r[3] for r in rows]), nfev=np.array([r[4] for r in rows]))
    nf = np.array([r[4] for r in rows], dtype=np.float64)
    print(f"N={a.n}: {len(rows)} fits in {time.time() - t0:.0f} s, nfev mean {nf.mean():.3f} "
          f"(std {nf.std(ddof=1):.2f}, standard error {nf.std(ddof=1) / np.sqrt(len(nf)):.3f}) -> {out}")


if __name__ == "__main__":
    main()
