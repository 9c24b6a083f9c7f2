"""Pin the SVGP oracle (oracle/svgp_oracle.py) on the CPU: FillTriangular semantics,
closed-form known answers, the Titsias-bound identity against the exact-GPR oracle, and every
gradient against central finite differences of the ELBO itself."""
import math

import numpy as np
import pytest

from oracle import gp_oracle as O
from oracle import svgp_oracle as S
from tests.test_oracle import oracle_kernel


def test_fill_triangular_matches_tfp_docstring():
    # tfp.math.fill_triangular([1, 2, 3, 4, 5, 6]) == [[4, 0, 0], [6, 5, 0], [3, 2, 1]]
    L = S.fill_triangular(np.arange(1.0, 7.0))
    np.testing.assert_array_equal(L, [[4, 0, 0], [6, 5, 0], [3, 2, 1]])
    np.testing.assert_array_equal(S.fill_triangular_inverse(L), np.arange(1.0, 7.0))
    rng = np.random.default_rng(0)
    for n in (1, 2, 5, 9):
        x = rng.standard_normal(n * (n + 1) // 2)
        np.testing.assert_array_equal(S.fill_triangular_inverse(S.fill_triangular(x)), x)


def _problem(n=40, M=6, D=1, seed=0, fam="se"):
    rng = np.random.default_rng(seed)
    X = rng.uniform(0, 10, (n, D))
    Y = np.sin(X[:, :1]) + 0.1 * rng.standard_normal((n, 1))
    Z = rng.uniform(0, 10, (M, D))
    k = oracle_kernel(fam)
    m = S.OSVGP(k, Z, num_data=n, noise_variance=0.05)
    m.q_mu = rng.standard_normal(M) * 0.3
    R = np.tril(rng.standard_normal((M, M)) * 0.2)
    R[np.diag_indices(M)] = rng.uniform(0.4, 1.2, M)
    m.q_sqrt = R
    return m, X, Y


def test_prior_q_known_answer():
    """q = N(0, I) (GPflow's init): KL = 0, μ = 0, v = k_diag, so the ELBO is closed form."""
    rng = np.random.default_rng(1)
    X = rng.uniform(0, 5, (30, 1))
    Y = rng.standard_normal((30, 1))
    m = S.OSVGP(O.OSquaredExponential(variance=1.3, lengthscales=0.7), X[:5], num_data=30,
                noise_variance=0.2)
    want = np.sum(-0.5 * math.log(2 * math.pi * 0.2) - 0.5 * (Y[:, 0] ** 2 + 1.3) / 0.2)
    assert m.elbo(X, Y) == pytest.approx(want, rel=1e-12)


def test_optimal_q_with_z_equal_x_recovers_exact_log_marginal_likelihood():
    """Titsias: with the optimal whitened q(u) the ELBO is log N(y|0, Qnn+σ²I) − tr(Knn−Qnn)/(2σ²);
    with Z = X, Qnn = Knn up to the 1e-6 jitter, so ELBO → exact GPR logML."""
    rng = np.random.default_rng(2)
    X = np.sort(rng.uniform(0, 6, (25, 1)), axis=0)
    Y = np.sin(X) + 0.1 * rng.standard_normal((25, 1))
    k = O.OSquaredExponential(variance=0.9, lengthscales=1.1)
    s2 = 0.3
    m = S.OSVGP(k, X, num_data=25, noise_variance=s2)
    L = np.linalg.cholesky(k.K(X) + S.JITTER * np.eye(25))
    A = np.linalg.solve(L, k.K(X))
    Sq = np.linalg.inv(np.eye(25) + A @ A.T / s2)
    m.q_mu = Sq @ A @ Y[:, 0] / s2
    m.q_sqrt = np.linalg.cholesky(Sq)
    exact = O.OGPR(X, Y, k, noise_variance=s2).log_marginal_likelihood()
    assert m.elbo(X, Y) == pytest.approx(exact, abs=1e-4 * abs(exact))


@pytest.mark.parametrize("fam", ["se", "m12", "m52", "rq", "exp+per+lin", "se*m12"])
def test_gradients_match_finite_differences(fam):
    m, X, Y = _problem(fam=fam, seed=3)
    m.noise.trainable = True
    loss, g = m.loss_and_grad_u(X, Y)
    u0 = m.get_u()
    assert g.shape == u0.shape
    h = 1e-6
    fd = np.empty_like(u0)
    for i in range(u0.size):
        up, um = u0.copy(), u0.copy()
        up[i] += h
        um[i] -= h
        m.set_u(up)
        lp = m.training_loss(X, Y)
        m.set_u(um)
        lm = m.training_loss(X, Y)
        fd[i] = (lp - lm) / (2 * h)
    m.set_u(u0)
    assert m.training_loss(X, Y) == pytest.approx(loss, rel=1e-14)
    np.testing.assert_allclose(g, fd, rtol=2e-5, atol=2e-5 * (1 + np.abs(fd).max()))


def test_2d_inputs_and_minibatch_scale():
    m, X, Y = _problem(n=30, M=5, D=2, seed=4, fam="m32")
    m.num_data = 300  # minibatch scaling num_data / N
    loss, g = m.loss_and_grad_u(X, Y)
    u0 = m.get_u()
    h = 1e-6
    for i in (0, 3, 9, 11, 12, 20, u0.size - 1):
        up, um = u0.copy(), u0.copy()
        up[i] += h
        um[i] -= h
        m.set_u(up)
        lp = m.training_loss(X, Y)
        m.set_u(um)
        lm = m.training_loss(X, Y)
        assert (lp - lm) / (2 * h) == pytest.approx(g[i], rel=2e-5, abs=1e-5)
    m.set_u(u0)
