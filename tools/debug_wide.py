"""Debug aid for the wide-class reduction (bs = 128): logML / gradient / α / diag Z of the wide
chain against the dense path at several N, with the band check's redo disabled (GPX_BAND_TOL)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ["GPX_BAND_TOL"] = "1e300"
import portfoliooptgp_amd as gpx  # noqa: E402
from portfoliooptgp_amd import _native as N  # noqa: E402
from portfoliooptgp_amd.engine import Engine  # noqa: E402
from portfoliooptgp_amd.kernels import compile_spec  # noqa: E402
from oracle import gp_oracle as O  # noqa: E402

K = gpx.kernels
for n in [int(v) for v in (sys.argv[1] if len(sys.argv) > 1 else "512,640,1024,4096").split(",")]:
    ells = [2.5, 3.0]
    data = [O.synthetic_series(n, seed=70 + s) for s in range(len(ells))]
    eng = Engine([d[0] for d in data], [d[1] for d in data], [compile_spec(K.SquaredExponential(), 1)] * 2)
    eng.ctx.set_profiling(True)
    th = np.ones((2, N.GPX_THETA_STRIDE))
    for b, e in enumerate(ells):
        th[b, :3] = (e, 0.9, 1e-5)
    eng.reset_timing()
    lb, gb, ib = eng.lml_grad([0, 1], th)
    t = eng.last_timing()
    mb, vb, _ = eng._predict_train(np.arange(2, dtype=np.int32), th, False)
    os.environ["GPX_BAND"] = "0"
    ld, gd, idn = eng.lml_grad([0, 1], th)
    md, vd, _ = eng._predict_train(np.arange(2, dtype=np.int32), th, False)
    os.environ.pop("GPX_BAND")
    for b in range(2):
        print(f"n={n} ell={ells[b]} wide={t.bcr_wide_evals} info={ib[b]} lml {lb[b]:.10f} dense {ld[b]:.10f} "
              f"rel {abs(lb[b]-ld[b])/abs(ld[b]):.2e} grad {gb[b,:3]} dense {gd[b,:3]} "
              f"mean_err {np.abs(mb[b].cpu().numpy()-md[b].cpu().numpy()).max():.2e} "
              f"var_err {np.abs(vb[b].cpu().numpy()-vd[b].cpu().numpy()).max():.2e}", flush=True)
