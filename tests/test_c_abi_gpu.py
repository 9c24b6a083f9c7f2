"""The C ABI from a plain-C host (tests/c/gpx_c_smoke.c, built by `make` with gcc against
include/gpx.h and libgpx.so): a non-Python caller of the reference would bind exactly these
entry points. GPU test: its logML, gradient and predictions equal the CPU oracle's. CPU test:
the binary is built and resolves libgpx.so through its rpath."""
import json
import os
import subprocess

import numpy as np
import pytest

from oracle import gp_oracle as O

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(REPO, "tests", "c", "gpx_c_smoke")


def test_c_consumer_is_built_and_links():
    if not os.path.exists(BIN):
        pytest.skip("tests/c/gpx_c_smoke not built (run make)")
    out = subprocess.run(["ldd", BIN], capture_output=True, text=True, check=True).stdout
    line = [ln for ln in out.splitlines() if "libgpx.so" in ln][0]
    assert "not found" not in line and os.path.realpath(line.split("=>")[1].split("(")[0].strip()) == \
        os.path.realpath(os.path.join(REPO, "portfoliooptgp_amd", "libgpx.so"))


def _oracle(n, kern, noise):
    x = np.arange(n, dtype=np.float64)[:, None]
    y = np.sin(x / 7.0) + (0.3 * np.cos(x / 3.0) if isinstance(kern, O.OMatern52) else 0.0)
    m = O.OGPR(x, y, kern, noise_variance=noise)
    loss, gu = m.loss_and_grad_u()
    gth = -gu / np.array([p.dtheta_du() for p in m.trainable_params()])  # ∂logML/∂θ
    xs = np.array([-1.5, 0.0, 3.25, 10.0, 40.5, 88.0, 120.0])[:, None]
    mu, var = m.predict_f(xs)
    return -loss, gth, mu.ravel(), var.ravel(), m


@pytest.mark.gpu
def test_c_consumer_matches_oracle():
    assert os.path.exists(BIN), "build with make first"
    n = 89
    r = subprocess.run([BIN, str(n)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    out = json.loads(r.stdout.strip().splitlines()[-1])
    cases = [_oracle(n, O.OSquaredExponential(lengthscales=3.0, variance=1.5), 1e-2),
             _oracle(n // 2, O.OMatern52(lengthscales=5.0, variance=0.7), 1e-3)]
    for b, (lml, g, mu, var, m) in enumerate(cases):
        assert abs(out["lml"][b] - lml) <= 1e-9 * abs(lml)
        np.testing.assert_allclose(out["grad"][b], g, rtol=1e-7, atol=1e-9 * (1 + np.abs(g).max()))
        np.testing.assert_allclose(out["mean"][7 * b:7 * b + 7], mu, rtol=1e-7, atol=1e-10)
        np.testing.assert_allclose(out["var"][7 * b:7 * b + 7], var, rtol=1e-6, atol=1e-10)
    # predict_y at the first training input (add_noise=1) = predict_f there + σn²
    x0 = np.zeros((1, 1))
    _, v0 = cases[0][4].predict_f(x0)
    assert abs(out["ytrain_var0"] - (float(v0.ravel()[0]) + 1e-2)) <= 1e-8
    assert out["bad_arg_status"] == 2  # GPX_BAD_ARG, no exception across the ABI
    assert out["train_rows_match"] == 1  # gpx_batch_predict_train_rows: the same bits, packed by position
