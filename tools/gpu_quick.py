"""First GPU validation: lml / grad / predict of libgpx vs the oracle on small seeded inputs."""
import sys, time, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import portfoliooptgp_amd as gpx
from portfoliooptgp_amd import kernels as K
from oracle import gp_oracle as O

def pair(kind):
    return {
        "se": (K.SquaredExponential(), O.OSquaredExponential()),
        "m12": (K.Matern12(), O.OMatern12()),
        "m32": (K.Matern32(), O.OMatern32()),
        "m52": (K.Matern52(), O.OMatern52()),
        "exp": (K.Exponential(), O.OExponential()),
        "rq": (K.RationalQuadratic(), O.ORationalQuadratic()),
        "per": (K.Periodic(K.SquaredExponential()), O.OPeriodic(O.OSquaredExponential())),
        "lin": (K.Linear(), O.OLinear()),
        "se+m12": (K.SquaredExponential() + K.Matern12(), O.OSum([O.OSquaredExponential(), O.OMatern12()])),
        "exp+per+lin": (K.Exponential() + K.Periodic(K.SquaredExponential()) + K.Linear(),
                        O.OSum([O.OExponential(), O.OPeriodic(O.OSquaredExponential()), O.OLinear()])),
        "se*m12": (K.SquaredExponential() * K.Matern12(), O.OProduct([O.OSquaredExponential(), O.OMatern12()])),
    }[kind]

def set_params(gk, ok, rng):
    for gp, op in zip(gk.parameters, ok.params()):
        v = float(np.exp(rng.uniform(-0.5, 1.0)))
        gp.assign(v); op.value = v

worst = {}
rng = np.random.default_rng(0)
for n in [1, 2, 16, 64, 89, 128, 192, 256, 320, 512, 1024]:
    x = np.sort(rng.uniform(0, 30, n))[:, None]
    y = np.sin(x[:, 0]) + 0.3 * rng.standard_normal(n)
    y = ((y - y.mean()) / (y.std(ddof=1) if n > 1 else 1.0))[:, None]
    for kind in ["se", "m12", "m32", "m52", "exp", "rq", "per", "lin", "se+m12", "exp+per+lin", "se*m12"]:
        gk, ok = pair(kind)
        if n > 16: set_params(gk, ok, rng)
        noise = 1e-2 if kind in ("lin", "per", "exp+per+lin") else 1e-3
        m = gpx.models.GPR(data=(x, y), kernel=gk, noise_variance=noise)
        om = O.OGPR(x, y, ok, noise_variance=noise)
        loss_g, g_g = m.loss_and_grad_unconstrained()
        loss_o, g_o = om.loss_and_grad_u()
        scale = np.abs(g_o).max() + 1.0
        el = abs(loss_g - loss_o) / max(1.0, abs(loss_o))
        eg = np.abs(g_g - g_o).max() / scale
        mu, va = m.predict_f(x)
        mo, vo = om.predict_f(x)
        em = np.abs(mu.numpy() - mo).max() / (np.abs(mo).max() + 1e-12)
        ev = np.abs(va.numpy() - vo).max()
        key = kind
        w = worst.get(key, (0, 0, 0, 0))
        worst[key] = (max(w[0], el), max(w[1], eg), max(w[2], em), max(w[3], ev))
        if el > 1e-8 or eg > 1e-6 or em > 1e-6 or ev > 1e-6:
            print(f"MISMATCH n={n} {kind}: loss {loss_g} vs {loss_o} (rel {el:.2e}) grad rel {eg:.2e} mean {em:.2e} var {ev:.2e}")
            print("   g_gpu", g_g, " g_oracle", g_o)
for k, v in worst.items():
    print(f"{k:12s} loss {v[0]:.2e}  grad {v[1]:.2e}  mean {v[2]:.2e}  var {v[3]:.2e}")

# fit parity at N=89 SE
x = np.arange(89, dtype=np.float64)[:, None]
y = O.synthetic_series(89, seed=3)[1]
m = gpx.models.GPR(data=(x, y), kernel=K.SquaredExponential())
m.likelihood.variance.assign(1e-5); gpx.set_trainable(m.likelihood.variance, False)
t = time.time()
r = gpx.optimizers.Scipy().minimize(m.training_loss, m.trainable_variables, options=dict(maxiter=100))
print("gpu fit", r.fun, r.nfev, r.nit, time.time() - t)
om = O.OGPR(x, y, O.OSquaredExponential(), noise_variance=1e-5); om.noise.trainable = False
ro = O.scipy_minimize(om, 100)
print("oracle fit", ro.fun, ro.nfev, ro.nit, " dloss rel", abs(r.fun - ro.fun) / abs(ro.fun))

# timing at N=4096 (B=1 and B=8)
for B in [1, 8]:
    xs = [np.arange(4096, dtype=np.float64)[:, None]] * B
    ys = [O.synthetic_series(4096, seed=s)[1] for s in range(B)]
    from portfoliooptgp_amd.engine import Engine
    from portfoliooptgp_amd.kernels import compile_spec
    eng = Engine(xs, ys, [compile_spec(K.SquaredExponential(), 1)] * B)
    eng.ctx.set_profiling(True)
    theta = np.ones((B, 16)); theta[:, 2] = 1e-5
    theta[:, 0] = 20.0
    eng.lml_grad(list(range(B)), theta)
    import torch
    torch.cuda.synchronize()
    t = time.time()
    for _ in range(3):
        lml, g, info = eng.lml_grad(list(range(B)), theta)
    dt = (time.time() - t) / 3
    tm = eng.last_timing()
    print(f"N=4096 B={B}: {dt*1e3:.2f} ms/eval-batch  factor {tm.factor_ms:.2f} alpha {tm.alpha_ms:.2f} grad {tm.grad_ms:.2f} total {tm.total_ms:.2f} ms; "
          f"gemm TF/s {tm.gemm_flops/tm.total_ms/1e9:.2f}; alg TF/s {B*4096**3/tm.total_ms/1e9:.2f}; info {info}")
