"""SVGP model surface on the CPU (no device calls): GPflow variable order and transforms, and
the constrained → unconstrained gradient mapping against the oracle's."""
import numpy as np
import pytest

import portfoliooptgp_amd as gpx
from portfoliooptgp_amd.parameter import fill_triangular, fill_triangular_inverse
from oracle import gp_oracle as O
from oracle import svgp_oracle as S


def test_fill_triangular_product_matches_oracle():
    rng = np.random.default_rng(0)
    for n in (1, 3, 8):
        x = rng.standard_normal(n * (n + 1) // 2)
        np.testing.assert_array_equal(fill_triangular(x), S.fill_triangular(x))
        L = np.tril(rng.standard_normal((n, n)))
        np.testing.assert_array_equal(fill_triangular_inverse(L), S.fill_triangular_inverse(L))


def _model(M=5):
    Z = np.linspace(0, 10, M)[:, None]
    k = gpx.kernels.SquaredExponential(lengthscales=1.5, variance=0.7)
    m = gpx.models.SVGP(kernel=k, likelihood=gpx.likelihoods.Gaussian(variance=1e-4),
                        inducing_variable=Z, num_data=40)
    return m


def test_svgp_variables_follow_gpflow_order_and_shapes():
    m = _model()
    gpx.set_trainable(m.likelihood.variance, False)
    names = [v.name for v in m.trainable_variables]
    assert names == ["Z:0", "lengthscales:0", "variance:0", "q_mu:0", "q_sqrt:0"]
    shapes = [tuple(v.shape) for v in m.trainable_variables]
    assert shapes == [(5, 1), (), (), (5, 1), (1, 15)]
    # GPflow init: q_mu = 0, q_sqrt = I (FillTriangular-unconstrained)
    np.testing.assert_array_equal(m.q_sqrt.value[0], np.eye(5))
    np.testing.assert_array_equal(m.trainable_variables[4].numpy()[0], fill_triangular_inverse(np.eye(5)))
    m.trainable_variables[4].assign(np.arange(15.0)[None])
    np.testing.assert_array_equal(m.q_sqrt.value[0], fill_triangular(np.arange(15.0)))


def test_svgp_gradient_mapping_matches_oracle():
    rng = np.random.default_rng(3)
    X = rng.uniform(0, 10, (40, 1))
    Y = np.sin(X) + 0.1 * rng.standard_normal((40, 1))
    m = _model()
    gpx.set_trainable(m.likelihood.variance, False)
    R = np.tril(rng.standard_normal((5, 5)) * 0.2)
    R[np.diag_indices(5)] = rng.uniform(0.5, 1.0, 5)
    m.q_sqrt.assign(R[None])
    m.q_mu.assign(rng.standard_normal((5, 1)))
    om = S.OSVGP(O.OSquaredExponential(lengthscales=1.5, variance=0.7), m.inducing_variable.Z.value,
                 num_data=40, noise_variance=1e-4, q_mu=m.q_mu.value, q_sqrt=R)
    om.noise.trainable = False
    lo, go = om.loss_and_grad_u(X, Y)
    elbo, g = om.elbo_and_grads(X, Y)
    gth = np.zeros(16)
    gth[:2] = g["theta"]
    gth[2] = g["noise"]
    loss, gu = m.grads_to_unconstrained(m.trainable_variables, elbo, gth, g["Z"], g["q_mu"], g["q_sqrt"])
    assert loss == pytest.approx(lo, rel=1e-15)
    np.testing.assert_allclose(gu, go, rtol=1e-14, atol=1e-14)
    # and the packing the Scipy driver uses round-trips the unconstrained vector
    from portfoliooptgp_amd.optimizers import _pack, _unpack
    u = _pack(m.trainable_variables)
    np.testing.assert_allclose(u, om.get_u(), rtol=1e-15)
    _unpack(m.trainable_variables, u + 0.0)
    np.testing.assert_array_equal(_pack(m.trainable_variables), u)


def test_print_summary_lists_svgp_arrays(capsys):
    gpx.print_summary(_model())
    out = capsys.readouterr().out
    assert "SVGP.q_sqrt" in out and "FillTriangular" in out and "(1, 5, 5)" in out
