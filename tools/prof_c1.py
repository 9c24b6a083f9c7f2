"""Host-side profile of the drop-in sweep (bench.secondary_c1_solo's sweep: the AAPL d/w/m series ×
the 8 shared kernels, one GPR at a time as GPR/model_trainer.py:14-20): cProfile of 3 sweeps after
a warm-up, by cumulative and internal time. usage: python tools/prof_c1.py (GPU box)"""
import cProfile
import os
import pstats
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
import portfoliooptgp_amd as gpx  # noqa: E402

K = gpx.kernels
series = bench._c1_series()


def sweep():
    ks = [K.SquaredExponential(), K.Matern12(), K.RationalQuadratic(), K.Exponential(),
          K.SquaredExponential() + K.Matern12(), K.Exponential() + K.Periodic(K.SquaredExponential()) + K.Linear(),
          K.Exponential() + K.Periodic(K.SquaredExponential()), K.SquaredExponential() * K.Matern12()]
    for tf, x, y in series:
        for k in ks:
            m = gpx.models.GPR(data=(x, y), kernel=k, device=0)
            m.likelihood.variance.assign(1e-5)
            gpx.set_trainable(m.likelihood.variance, False)
            try:
                gpx.optimizers.Scipy().minimize(m.training_loss, m.trainable_variables, options=dict(maxiter=100))
            except (gpx.NotPositiveDefiniteError, gpx.InvalidParameterError):
                continue
            mean, _ = m.predict_f(x)
            float(np.mean((y.reshape(-1) - mean.numpy().reshape(-1)) ** 2))


sweep()
torch.cuda.synchronize()
t0 = time.perf_counter()
sweep()
torch.cuda.synchronize()
print(f"one sweep unprofiled: {1e3 * (time.perf_counter() - t0):.1f} ms", flush=True)
pr = cProfile.Profile()
pr.enable()
for _ in range(3):
    sweep()
torch.cuda.synchronize()
pr.disable()
st = pstats.Stats(pr)
st.sort_stats("cumulative").print_stats(45)
st.sort_stats("tottime").print_stats(35)
