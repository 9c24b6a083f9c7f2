"""Host-side logic of the GPflow-shaped API (no GPU needed): parameter transforms, variable
ordering, kernel -> gpx_kernel_spec compilation, set_trainable, summaries, and that the
product path refuses to run without the HIP device (no CPU fallback)."""
import math

import numpy as np
import pytest
import torch

import portfoliooptgp_amd as gpx
from portfoliooptgp_amd import _native as N
from portfoliooptgp_amd.kernels import compile_spec
from portfoliooptgp_amd.parameter import Parameter, softplus, softplus_inverse


def test_parameter_softplus_semantics():
    p = Parameter(1.0)
    assert p.unconstrained == pytest.approx(0.5413248546129181, abs=1e-15)
    p.unconstrained_variable.assign(2.0)
    assert p.value == pytest.approx(math.log1p(math.exp(2.0)))
    p.assign(3.5)
    assert p.value == pytest.approx(3.5, rel=1e-14)
    n = Parameter(1.0, lower=1e-6)
    n.assign(1e-5)
    assert n.value == pytest.approx(1e-5, rel=1e-10)
    assert n.dtheta_du() == pytest.approx(1 / (1 + math.exp(-n.unconstrained)))
    for t in [1e-20, 1e-8, 0.3, 5.0, 40.0, 800.0]:
        assert softplus(softplus_inverse(t)) == pytest.approx(t, rel=1e-12)
    with pytest.raises(ValueError):
        Parameter(-1.0)


def test_reference_kernel_list_param_order():
    """GPflow flattening order for the 8 kernels of GPR/main.py:105-114."""
    K = gpx.kernels
    ks = [K.SquaredExponential(), K.Matern12(), K.RationalQuadratic(), K.Exponential(),
          K.SquaredExponential() + K.Matern12(),
          K.Exponential() + K.Periodic(K.SquaredExponential()) + K.Linear(),
          K.Exponential() + K.Periodic(K.SquaredExponential()),
          K.SquaredExponential() * K.Matern12()]
    names = [[n for n, _ in k._param_paths("")] for k in ks]
    assert names[0] == ["lengthscales", "variance"]
    assert names[2] == ["alpha", "lengthscales", "variance"]
    assert names[5] == ["kernels[0].lengthscales", "kernels[0].variance",
                        "kernels[1].base_kernel.lengthscales", "kernels[1].base_kernel.variance",
                        "kernels[1].period", "kernels[2].variance"]
    assert isinstance(ks[5], K.Sum) and len(ks[5].kernels) == 3  # flattened like GPflow
    specs = [compile_spec(k, 1) for k in ks]
    assert [s.n_params for s in specs] == [2, 2, 3, 2, 4, 6, 5, 4]
    assert specs[7].combine == N.GPX_PRODUCT and specs[5].combine == N.GPX_SUM
    assert [specs[5].terms[t].param_offset for t in range(3)] == [0, 2, 5]
    assert [specs[5].terms[t].kind for t in range(3)] == [N.GPX_EXPONENTIAL, N.GPX_PERIODIC_SE, N.GPX_LINEAR]


def test_active_dims_composite_spec():
    """Multi-Input_GPR/main.py:118-135: Exponential(dims 0..D-2) * Exponential(dim D-1)."""
    D = 5
    k = gpx.kernels.Exponential(active_dims=slice(0, D - 1)) * gpx.kernels.Exponential(active_dims=slice(D - 1, D))
    s = compile_spec(k, D)
    assert (s.terms[0].dim_start, s.terms[0].dim_count) == (0, 4)
    assert (s.terms[1].dim_start, s.terms[1].dim_count) == (4, 1)
    with pytest.raises(ValueError):
        compile_spec(gpx.kernels.SquaredExponential(active_dims=[3, 4, 5]), 5)
    with pytest.raises(NotImplementedError):
        compile_spec(gpx.kernels.SquaredExponential(active_dims=[0, 2]), 5)


def test_model_variables_and_set_trainable():
    x = np.arange(5.0)[:, None]
    y = np.sin(x)
    m = gpx.models.GPR(data=(x, y), kernel=gpx.kernels.RationalQuadratic())
    assert len(m.trainable_variables) == 4  # alpha, lengthscales, variance, likelihood.variance
    m.likelihood.variance.assign(1e-5)
    gpx.set_trainable(m.likelihood.variance, False)
    assert len(m.trainable_variables) == 3
    row = m.theta_row()
    assert row[3] == pytest.approx(1e-5)
    gpx.set_trainable(m.kernel, False)
    assert m.trainable_variables == ()
    m2 = gpx.models.GPR(data=(x, y), kernel=gpx.kernels.Matern52(), noise_variance=1e-3)
    assert m2.likelihood.variance.value == pytest.approx(1e-3)


def test_shared_kernel_objects_alias_like_gpflow():
    """the same kernel object in two models shares parameters."""
    k = gpx.kernels.SquaredExponential()
    x = np.arange(4.0)[:, None]
    a = gpx.models.GPR(data=(x, x), kernel=k)
    b = gpx.models.GPR(data=(x, x), kernel=k)
    a.trainable_variables[0].assign(1.7)
    assert b.kernel.lengthscales.unconstrained == 1.7


def test_print_summary(capsys):
    m = gpx.models.GPR(data=(np.zeros((3, 1)), np.zeros((3, 1))),
                       kernel=gpx.kernels.Exponential() + gpx.kernels.Periodic(gpx.kernels.SquaredExponential()))
    gpx.print_summary(m)
    out = capsys.readouterr().out
    assert "GPR.kernel.kernels[1].period" in out and "GPR.likelihood.variance" in out


@pytest.mark.skipif(torch.cuda.is_available(), reason="checks the no-GPU behaviour")
def test_no_cpu_fallback():
    m = gpx.models.GPR(data=(np.arange(3.0)[:, None], np.ones((3, 1))), kernel=gpx.kernels.SquaredExponential())
    with pytest.raises(N.GPXError, match="no CPU fallback"):
        m.training_loss()
    with pytest.raises(N.GPXError):
        gpx.optimizers.Scipy().minimize(m.training_loss, m.trainable_variables)


def test_empty_training_set_is_refused():
    """0 training rows: refused at construction (the device engine needs a point to factorise)."""
    with pytest.raises(ValueError, match="at least one training point"):
        gpx.models.GPR((np.zeros((0, 1)), np.zeros((0, 1))), kernel=gpx.kernels.SquaredExponential())


def test_scipy_rejects_foreign_closures():
    with pytest.raises(TypeError):
        gpx.optimizers.Scipy().minimize(lambda: 0.0, [Parameter(1.0).unconstrained_variable])


def test_predict_y_full_cov_not_implemented_like_gpflow():
    """GPflow 2.9 GPModel.predict_y raises NotImplementedError for full_cov/full_output_cov;
    predict_f(full_cov=True) is supported (GPU test_predict_full_cov)."""
    x = np.arange(5.0)[:, None]
    m = gpx.models.GPR((x, x), kernel=gpx.kernels.SquaredExponential())
    with pytest.raises(NotImplementedError):
        m.predict_y(x, full_cov=True)
    with pytest.raises(NotImplementedError):
        m.predict_y(x, full_output_cov=True)


def test_blend_optimizer_recovers_weights_and_respects_constraints():
    """GPR/optimizer.py semantics: SLSQP, bounds [0,1]², α+β ≤ 1, L1 penalty λ."""
    from portfoliooptgp_amd.trainer import BlendOptimizer
    rng = np.random.default_rng(0)
    fd, fw, fm = (rng.standard_normal((200, 1)) for _ in range(3))
    Y = 0.5 * fd + 0.3 * fw + 0.2 * fm
    w = BlendOptimizer(lambda_=1e-8).optimize_weights(Y, fd, fw, fm)
    np.testing.assert_allclose(w, [0.5, 0.3], atol=1e-4)
    w = BlendOptimizer(lambda_=0.01).optimize_weights(3 * fd + 3 * fw, fd, fw, fm)
    assert np.all(w >= -1e-9) and np.all(w <= 1 + 1e-9) and w.sum() <= 1 + 1e-9
    opt = BlendOptimizer(0.01)
    assert opt.loss_fn([0.2, 0.3], Y, fd, fw, fm) == pytest.approx(
        float(np.mean((Y - (0.2 * fd + 0.3 * fw + 0.5 * fm)) ** 2)) + 0.01 * 0.5)
