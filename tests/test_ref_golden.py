"""Host-side rows either side of the hot path against golden vectors made by the REFERENCE'S OWN
modules (tests/golden/make_ref_golden.py imports /root/reference/GPR/optimizer.py): the α/β
timeframe blend (GPR/optimizer.py:5-28), the positional upsampling and the
blend arithmetic of Predictor.predict_combined (GPR/predictor.py:10-51). No GPU: the device
predictions these consume are pinned by tests/test_callers_gpu.py."""
import os

import numpy as np
import pytest
import torch

from portfoliooptgp_amd.trainer import BlendOptimizer, Predictor


@pytest.fixture(scope="module")
def blend(golden_dir):
    return np.load(os.path.join(golden_dir, "blend.npz"))


@pytest.mark.parametrize("case", ["synth0", "synth1", "synth2", "synth3"])
def test_blend_weights_match_reference_optimizer(blend, case):
    p = case + "|"
    ab = BlendOptimizer(float(blend[p + "lambda"][0])).optimize_weights(
        blend[p + "Y"], blend[p + "fd"], blend[p + "fw"], blend[p + "fm"])
    np.testing.assert_allclose(ab, blend[p + "alpha_beta"], rtol=0, atol=1e-9)


def test_aapl_flow_upsample_and_weights(blend):
    """GPR/main.py:47-56 on the oracle's AAPL d/w/m best models: weekly and monthly means
    upsampled to the daily grid exactly as the reference's pandas reindex + interpolate, then
    the α/β SLSQP with λ = 0.1, as the reference's Optimizer gave them."""
    pr = Predictor()
    xd, xw, xm = blend["aapl|d|x"], blend["aapl|w|x"], blend["aapl|m|x"]
    fw_up = pr.upsample_predictions(torch.as_tensor(xd), torch.as_tensor(xw), torch.as_tensor(blend["aapl|w|fm"]), "w")
    fm_up = pr.upsample_predictions(torch.as_tensor(xd), torch.as_tensor(xm), torch.as_tensor(blend["aapl|m|fm"]), "m")
    np.testing.assert_array_equal(fw_up.numpy(), blend["aapl|fw_up"])
    np.testing.assert_array_equal(fm_up.numpy(), blend["aapl|fm_up"])
    # 'd' passes the predictions through unchanged
    fd = torch.as_tensor(blend["aapl|d|fm"])
    assert pr.upsample_predictions(fd, fd, fd, "d") is fd
    assert blend["aapl|raises"][0] == 0
    ab = BlendOptimizer(float(blend["aapl|lambda"][0])).optimize_weights(blend["aapl|d|y"], blend["aapl|d|fm"],
                                                                         fw_up, fm_up)
    np.testing.assert_allclose(ab, blend["aapl|alpha_beta"], rtol=0, atol=1e-9)


class _FixedModel:
    """Duck-typed model whose predict_f / predict_y return fixed arrays (the oracle's)."""

    def __init__(self, f, v, y, yv):
        self.out = (torch.as_tensor(f), torch.as_tensor(v), torch.as_tensor(y), torch.as_tensor(yv))

    def predict_f(self, X, full_cov=False):
        return self.out[0], self.out[1]

    def predict_y(self, X):
        return self.out[2], self.out[3]


def test_predict_combined_blend_arithmetic(blend):
    """predict_combined's upsampling of all four outputs and the α/β combination, on the
    oracle's predictions at the extended inputs (golden: the same flow in the generator)."""
    models = [_FixedModel(*(blend[f"aapl|{t}|{k}"] for k in ("cm", "cv", "cym", "cyv"))) for t in "dwm"]
    a, b = blend["aapl|combined|alpha_beta"]
    xs = [torch.as_tensor(blend[f"aapl|{t}|xc"]) for t in "dwm"]
    out = Predictor().predict_combined(a, b, *models, *xs)
    for got, key in zip(out, ("cm", "cv", "cym", "cyv")):
        np.testing.assert_allclose(np.asarray(got), blend["aapl|combined|" + key], rtol=1e-15, atol=0,
                                   equal_nan=True)
