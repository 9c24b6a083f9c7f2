"""Diagnostics of the banded path against the dense one on the same problem: logML / gradient,
then α (through the training-input mean) and diag(K⁻¹) (through the training-input variance)
block by block, to locate where a banded sweep departs."""
import os
import sys

import numpy as np

sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import portfoliooptgp_amd as gpx  # noqa: E402
from oracle import gp_oracle as O  # noqa: E402
from portfoliooptgp_amd.engine import Engine  # noqa: E402
from portfoliooptgp_amd.kernels import compile_spec  # noqa: E402

cases = [(8192, 40.0, 1e-2), (8192, 45.0, 1e-2)]
for n, ell, noise in cases:
    x, y = O.synthetic_series(n, seed=9)
    eng = Engine([x], [y], [compile_spec(gpx.kernels.SquaredExponential(), 1)])
    eng.ctx.set_profiling(True)
    th = np.ones((1, 16))
    th[0, :3] = [ell, 1.1, noise]
    out = {}
    for mode in ("1", "0"):
        os.environ["GPX_BAND"] = mode
        eng.reset_timing()
        l, g, _ = eng.lml_grad([0], th)
        mu, var, _ = eng._predict_train(np.zeros(1, dtype=np.int32), th, False)
        out[mode] = (l[0], g[0, :3].copy(), mu[0].cpu().numpy(), var[0].cpu().numpy(), eng.last_timing().band_p_sum)
    (l1, g1, m1, v1, p1), (l0, g0, m0, v0, _) = out["1"], out["0"]
    dm = np.abs(m1 - m0) / (1 + np.abs(m0).max())
    dv = np.abs(v1 - v0) / (np.abs(v0).max())
    bad_m = np.nonzero(dm > 1e-8)[0]
    bad_v = np.nonzero(dv > 1e-8)[0]
    print(n, ell, "p", p1, "dlml %.2e" % abs(l1 - l0), "dgrad %.2e" % (np.abs(g1 - g0).max() / (1 + np.abs(g0).max())),
          "mean err max %.2e first bad row %s" % (dm.max(), bad_m[:1]),
          "var err max %.2e first bad row %s last %s count %d" % (dv.max(), bad_v[:1], bad_v[-1:], len(bad_v)), flush=True)
