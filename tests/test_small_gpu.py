"""The one-launch small-problem evaluations: small64_kernel for Np = 64 (N <= 64)
and small128_kernel for Np = 128 (N = 65..128, the reference's daily AAPL series at N = 89,
`GPR/model_trainer.py:14-20` fitting one GPR at a time). Oracle parity over kernel families and
ragged sizes at fixed θ, composition invariance (a problem's bits do not depend on the call), the
factor the predictions read, NOT_PD reporting, and agreement with the general launch chain
(GPX_SMALL64=0 / GPX_SMALL128=0, in a child process: the switch is read once per process).
The golden fixtures at N = 89 / 19 / 5 run through these kernels in tests/test_gpu_parity.py too."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

import portfoliooptgp_amd as gpx  # noqa: E402
from portfoliooptgp_amd import _native as N  # noqa: E402
from portfoliooptgp_amd.engine import Engine  # noqa: E402
from portfoliooptgp_amd.kernels import compile_spec  # noqa: E402
from oracle import gp_oracle as O  # noqa: E402
from tests.test_gpu_parity import check_grad, check_loss, check_mean, check_var, gpx_kernel, oracle_kernel  # noqa: E402

K = gpx.kernels
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _data(n, seed, d=1):
    rng = np.random.default_rng(seed)
    x = np.sort(rng.uniform(0, 30, (n, d)), axis=0)
    y = np.sin(x[:, :1]) + 0.1 * rng.standard_normal((n, 1))
    return x, y


@pytest.mark.parametrize("n", [65, 89, 100, 127, 128, 5, 19, 64])
@pytest.mark.parametrize("fam", ["se", "m32", "exp+per+lin", "se*m12", "rq"])
def test_small_against_oracle(n, fam):
    x, y = _data(n, 300 + n)
    m = gpx.models.GPR((x, y), kernel=gpx_kernel(fam), noise_variance=1e-2)
    om = O.OGPR(x, y, oracle_kernel(fam), noise_variance=1e-2)
    loss, g = m.loss_and_grad_unconstrained()
    lo, go = om.loss_and_grad_u()
    check_loss(loss, lo)
    check_grad(g, go)
    xs = np.linspace(-3, 33, 17)[:, None]
    mu, var = m.predict_f(xs)
    mo, vo = om.predict_f(xs)
    check_mean(mu.numpy(), mo)
    check_var(var.numpy(), vo, 1.0)


def test_small128_two_dimensional_product():
    x, y = _data(90, 7, d=2)
    k = K.Exponential(active_dims=slice(0, 1)) * K.Exponential(active_dims=slice(1, 2))
    m = gpx.models.GPR((x, y), kernel=k, noise_variance=1e-3)
    ok = O.OProduct([O.OExponential(active_dims=[0]), O.OExponential(active_dims=[1])])
    om = O.OGPR(x, y, ok, noise_variance=1e-3)
    loss, g = m.loss_and_grad_unconstrained()
    lo, go = om.loss_and_grad_u()
    check_loss(loss, lo)
    check_grad(g, go)


@pytest.mark.parametrize("sizes", [[128, 70, 100, 89, 65, 127], [64, 5, 19, 33, 64, 50]])
def test_small_composition_invariance(sizes):
    """Each problem alone in a batch of its own Np, and all six in one call: the same bits."""
    data = [_data(n, 40 + i) for i, n in enumerate(sizes)]
    spec = compile_spec(K.Matern52(), 1)
    theta = np.ones((len(sizes), N.GPX_THETA_STRIDE))
    theta[:, 0] = np.linspace(0.5, 3.0, len(sizes))
    theta[:, 1] = 1.3
    theta[:, 2] = 1e-2
    eb = Engine([d[0] for d in data], [d[1] for d in data], [spec] * len(sizes))
    assert eb.Nmax == max(sizes)
    lb, gb, ib = eb.lml_grad(list(range(len(sizes))), theta)
    assert not ib.any()
    for i, (x, y) in enumerate(data):
        # (a one-problem batch padded to the same Np: its own N would pick a smaller kernel)
        xp = np.vstack([x, np.zeros((max(sizes) - len(x), 1))])
        yp = np.vstack([y, np.zeros((max(sizes) - len(y), 1))])
        e1 = Engine([x, xp], [y, yp], [spec, spec])
        assert e1.Nmax == eb.Nmax
        l1, g1, _ = e1.lml_grad([0], np.repeat(theta[i:i + 1], 2, axis=0))
        assert l1[0] == lb[i]
        assert np.array_equal(g1[0, :3], gb[i, :3])


def test_small128_not_positive_definite():
    """K = σ²11ᵀ + σn²I with σ² = 1e12 rounds to rank one: pivot 2 fails, as on the chain."""
    x = np.zeros((90, 1))
    y = np.ones((90, 1))
    m = gpx.models.GPR(data=(x, y), kernel=K.SquaredExponential(variance=1e12), noise_variance=2e-6)
    with pytest.raises(N.NotPositiveDefiniteError) as e:
        m.training_loss()
    assert int(e.value.info) == 2
    good = gpx.models.GPR(data=(np.arange(90.0)[:, None], y), kernel=K.SquaredExponential())
    eng = Engine([x, good.data[0]], [y, y], [compile_spec(m.kernel, 1), compile_spec(good.kernel, 1)])
    lml, grad, info = eng.lml_grad([0, 1], np.stack([m.theta_row(), good.theta_row()]))
    assert info[0] == 2 and info[1] == 0 and np.isfinite(lml[1])


CHILD = r'''
import os, sys, json, numpy as np
sys.path.insert(0, os.environ["REPO"])
import portfoliooptgp_amd as gpx
from portfoliooptgp_amd.engine import Engine
from portfoliooptgp_amd.kernels import compile_spec
out = {}
for n in (89, 19):
    rng = np.random.default_rng(n)
    x = np.sort(rng.uniform(0, 30, (n, 1)), axis=0); y = np.cos(x) + 0.1 * rng.standard_normal((n, 1))
    eng = Engine([x], [y], [compile_spec(gpx.kernels.Matern32() + gpx.kernels.Linear(), 1)])
    th = np.ones((1, 16)); th[0, :4] = [1.7, 0.9, 0.3, 1e-2]
    l, g, info = eng.lml_grad([0], th)
    out[str(n)] = [float(l[0])] + [float(v) for v in g[0, :4]] + [int(info[0])]
print(json.dumps(out))
'''


def test_small_kernels_agree_with_the_launch_chain():
    def run(env):
        e = dict(os.environ, REPO=ROOT, **env)
        p = subprocess.run([sys.executable, "-c", CHILD], env=e, capture_output=True, text=True, timeout=240)
        assert p.returncode == 0, p.stderr[-3000:]
        return json.loads(p.stdout.strip().splitlines()[-1])
    a = run({})
    b = run({"GPX_SMALL64": "0", "GPX_SMALL128": "0"})
    for n in a:
        va, vb = np.array(a[n][:5]), np.array(b[n][:5])
        assert a[n][5] == b[n][5] == 0
        np.testing.assert_allclose(va, vb, rtol=1e-10, atol=1e-10 * np.abs(vb).max())
