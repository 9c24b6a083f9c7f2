"""Per-operation host costs of the fitting loop on the GPU box (N=4096 slots, as the bench):
model construction, slot rebind, predict at the training inputs, and a minimal device call."""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
import portfoliooptgp_amd as gpx  # noqa: E402
from portfoliooptgp_amd.engine import Engine  # noqa: E402
from portfoliooptgp_amd.kernels import compile_spec  # noqa: E402


def timeit(label, fn, reps):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    print(f"{label}: {(time.perf_counter() - t0) / reps * 1e6:.1f} us", flush=True)


n = 4096
x, y = bench.synthetic_series(n, 0)
xd, yd = torch.as_tensor(x, device="cuda:0"), torch.as_tensor(y, device="cuda:0")


def make():
    m = gpx.models.GPR(data=(xd, yd), kernel=gpx.kernels.SquaredExponential(), device=0)
    m.likelihood.variance.assign(1e-5)
    gpx.set_trainable(m.likelihood.variance, False)
    return m


timeit("GPR construction", make, 200)
m = make()
timeit("compile_spec", lambda: compile_spec(m.kernel, 1), 200)
eng = Engine([xd] * 8, [yd] * 8, [compile_spec(m.kernel, 1)] * 8, device=0)
timeit("Engine.rebind (N=4096)", lambda: eng.rebind(3, xd, yd, compile_spec(m.kernel, 1)), 100)
th = np.ones((8, 16))
th[:, :3] = [1.2, 0.6, 1e-5]
eng.lml_grad(list(range(8)), th)
timeit("predict at X_train (8 slots, detection by torch.equal)",
       lambda: eng.predict(list(range(8)), th, [xd] * 8, False), 50)
timeit("_predict_train (8 slots)", lambda: eng._predict_train(np.arange(8, dtype=np.int32), th, False), 50)
xs, ys = torch.as_tensor(x[:64], device="cuda:0"), torch.as_tensor(y[:64], device="cuda:0")
e1 = Engine([xs], [ys], [compile_spec(m.kernel, 1)], device=0)
t1 = np.ones((1, 16))
t1[0, :3] = [1.2, 0.6, 1e-5]
timeit("lml_grad B=1 N=64 (fixed cost of a device call)", lambda: e1.lml_grad([0], t1), 200)
timeit("lml_grad B=8 N=4096 banded", lambda: eng.lml_grad(list(range(8)), th), 20)
