"""Fixed workload for rocprofv3: `reps` lml+grad evaluations of B problems at N (SE kernel)."""
import argparse, os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
from portfoliooptgp_amd import kernels as K
from portfoliooptgp_amd.engine import Engine
from portfoliooptgp_amd.kernels import compile_spec
from bench import synthetic_series

ap = argparse.ArgumentParser()
ap.add_argument("--n", type=int, default=4096)
ap.add_argument("--b", type=int, default=8)
ap.add_argument("--reps", type=int, default=3)
ap.add_argument("--predict", action="store_true")
ap.add_argument("--kernel", default="se", choices=["se", "m52", "expxexp"],
                help="se: config C2; m52 / expxexp: config C4 shapes (D=5: 4 z-scored random-walk "
                     "features + z-scored time)")
args = ap.parse_args()
if args.kernel == "se":
    data = [synthetic_series(args.n, s) for s in range(args.b)]
    spec = compile_spec(K.SquaredExponential(), 1)
    D = 1
else:
    D = 5
    data = []
    for s in range(args.b):
        rng = np.random.default_rng(100 + s)
        feats = np.cumsum(rng.standard_normal((args.n, 4)), axis=0)
        t = np.linspace(0.0, 1.0, args.n)[:, None]
        X = np.hstack([feats, t])
        X = (X - X.mean(0)) / X.std(0, ddof=1)
        data.append((X, synthetic_series(args.n, s)[1]))
    if args.kernel == "m52":
        spec = compile_spec(K.Matern52(), D)
    else:  # Multi-Input_GPR/main.py:118-135: Exponential(dims 0..D-2) x Exponential(dim D-1)
        spec = compile_spec(K.Exponential(active_dims=slice(0, D - 1)) * K.Exponential(active_dims=slice(D - 1, D)), D)
eng = Engine([d[0] for d in data], [d[1] for d in data], [spec] * args.b)
eng.ctx.set_profiling(True)
theta = np.ones((args.b, 16))
if args.kernel == "se":
    theta[:, 0] = 20.0; theta[:, 2] = 1e-5
elif args.kernel == "m52":
    theta[:, 0] = 2.0; theta[:, 2] = 1e-3
else:
    theta[:, 0] = 2.0; theta[:, 2] = 2.0; theta[:, 4] = 1e-3
act = list(range(args.b))
eng.lml_grad(act, theta)
torch.cuda.synchronize()
t = time.perf_counter()
for _ in range(args.reps):
    eng.lml_grad(act, theta)
dt = (time.perf_counter() - t) / args.reps
tm = eng.last_timing()
print(f"{args.kernel} N={args.n} B={args.b}: {dt*1e3:.2f} ms/eval  factor {tm.factor_ms:.2f} alpha {tm.alpha_ms:.2f} grad {tm.grad_ms:.2f} "
      f"alg {args.b*args.n**3/dt/1e12:.2f} TF/s")
if args.predict:
    X = [torch.as_tensor(d[0], device="cuda") for d in data]
    eng.predict(act, theta, X, False)
    torch.cuda.synchronize()
    t = time.perf_counter()
    eng.predict(act, theta, X, False)
    torch.cuda.synchronize()
    print(f"predict (cached factor) {1e3*(time.perf_counter()-t):.2f} ms")
