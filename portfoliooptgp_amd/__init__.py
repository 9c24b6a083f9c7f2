"""portfoliooptgp_amd — MI355X-native exact-GP regression engine.

Drop-in for the GP hot path of LUOJIUzxy/PortfolioOptGP (GPR/model_trainer.py,
GPR/predictor.py): the GPflow-2.9.1-shaped model API lives here in Python; every
log-marginal-likelihood, gradient and posterior is computed by hand-written HIP kernels for
gfx950 in ``libgpx.so`` behind the C ABI of ``include/gpx.h``.

    import portfoliooptgp_amd as gpx
    m = gpx.models.GPR(data=(X, Y), kernel=gpx.kernels.SquaredExponential())
    m.likelihood.variance.assign(1e-5); gpx.set_trainable(m.likelihood.variance, False)
    gpx.optimizers.Scipy().minimize(m.training_loss, m.trainable_variables, options=dict(maxiter=100))
    mean, var = m.predict_f(X)
"""
from . import _native, data, inducing_variables, kernels, likelihoods, models, optimizers, utilities
from ._native import GPXError, InvalidParameterError, NotPositiveDefiniteError
from .engine import set_default_band_route
from .parameter import Parameter
from .utilities import print_summary, set_trainable

__all__ = ["inducing_variables", "kernels", "likelihoods", "models", "optimizers", "utilities", "Parameter",
           "set_trainable", "print_summary", "GPXError", "InvalidParameterError",
           "NotPositiveDefiniteError", "set_default_band_route"]
__version__ = "0.1.0"
