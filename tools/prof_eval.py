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
args = ap.parse_args()
data = [synthetic_series(args.n, s) for s in range(args.b)]
eng = Engine([d[0] for d in data], [d[1] for d in data], [compile_spec(K.SquaredExponential(), 1)] * args.b)
eng.ctx.set_profiling(True)
theta = np.ones((args.b, 16)); theta[:, 0] = 20.0; theta[:, 2] = 1e-5
act = list(range(args.b))
eng.lml_grad(act, theta)
torch.cuda.synchronize()
t = time.perf_counter()
for _ in range(args.reps):
    eng.lml_grad(act, theta)
dt = (time.perf_counter() - t) / args.reps
tm = eng.last_timing()
print(f"N={args.n} B={args.b}: {dt*1e3:.2f} ms/eval  factor {tm.factor_ms:.2f} alpha {tm.alpha_ms:.2f} grad {tm.grad_ms:.2f} "
      f"alg {args.b*args.n**3/dt/1e12:.2f} TF/s")
if args.predict:
    X = [torch.as_tensor(d[0], device="cuda") for d in data]
    eng.predict(act, theta, X, False)
    torch.cuda.synchronize()
    t = time.perf_counter()
    eng.predict(act, theta, X, False)
    torch.cuda.synchronize()
    print(f"predict (cached factor) {1e3*(time.perf_counter()-t):.2f} ms")
