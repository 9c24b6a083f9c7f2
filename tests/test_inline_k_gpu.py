"""The band16 sweeps computing K's tiles from X inside the sweeps (GPX_B16_INLINE_K, DESIGN.md §3e:
bit 0 the forward sweep, bit 1 the backward; no K band through HBM when both) against the sweeps
that read the K band band16_build_kernel wrote: the same operations on the same inputs, so every
logML, gradient and training-input prediction must be identical bit for bit, for every band16
width (Q = 1..5, as separate launches and as the deferred wide launch) and a ragged series.

The library reads GPX_B16_INLINE_K once per process, so each setting runs in a child process
(one at a time: at most two processes use the GPU here)."""
import os
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r"""
import sys, numpy as np
sys.path.insert(0, {root!r})
from portfoliooptgp_amd import kernels as K, _native as N
from portfoliooptgp_amd.engine import Engine
from portfoliooptgp_amd.kernels import compile_spec
from oracle import gp_oracle as O
ells = [0.3, 0.7, 1.0, 1.18, 1.6, 1.9, 1.5, 1.18]
n = 4096
data = [O.synthetic_series(n, s) for s in range(len(ells))]
data[6] = (data[6][0][:3001], data[6][1][:3001])
spec = compile_spec(K.SquaredExponential(), 1)
out = {{}}
for defer in (-1, 3):
    eng = Engine([d[0] for d in data], [d[1] for d in data], [spec] * len(data), band_storage=True)
    th = np.ones((len(ells), N.GPX_THETA_STRIDE))
    th[:, 0] = ells
    th[:, 1] = 0.7
    th[:, 2] = 1e-5
    act = list(range(len(ells)))
    if defer >= 0:
        eng.set_deferred(defer)
        eng.lml_grad_submit(act, th)
        l, g, i = eng.lml_grad_complete()
        l3, g3, i3 = eng.deferred_wait()
        for b in act:
            if i[b] == N.INFO_DEFERRED:
                l[b], g[b], i[b] = l3[b], g3[b], i3[b]
    else:
        l, g, i = eng.lml_grad(act, th)
        m, v, _ = eng._predict_train(np.arange(len(ells), dtype=np.int32), th, False)
        out["mean"] = np.concatenate([x.cpu().numpy().ravel() for x in m])
        out["var"] = np.concatenate([x.cpu().numpy().ravel() for x in v])
        out["q"] = np.array(eng.band_class(act, th))
    out[f"lml{{defer}}"] = l
    out[f"grad{{defer}}"] = g[:, :3]
    out[f"info{{defer}}"] = i
np.savez({path!r}, **out)
"""


def _run(kin, path, wide=None, extra=None):
    env = dict(os.environ, GPX_B16_INLINE_K=str(kin), GPX_BCR_MAX="0")  # (the band16 sweeps, not gpx_bcr)
    for k in ("GPX_B16_INLINE_K_WIDE", "GPX_DEFER_STREAM"):
        env.pop(k, None)
    if wide is not None:
        env["GPX_B16_INLINE_K_WIDE"] = str(wide)
    env.update(extra or {})
    code = CHILD.format(root=ROOT, path=path)
    r = subprocess.run([sys.executable, "-c", code], env=env, cwd=ROOT, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    return np.load(path)


@pytest.mark.parametrize("kin,wide,extra", [(1, None, None), (2, None, None), (3, None, None), (3, 0, None),
                                            (3, None, {"GPX_DEFER_STREAM": "0"})])
def test_inline_k_bit_identical(tmp_path, kin, wide, extra):
    """(wide: GPX_B16_INLINE_K_WIDE, the setting of the deferred part's wide launch; extra: the
    deferred part on the call's own stream instead of a stream of its own)"""
    ref = _run(0, str(tmp_path / "k0.npz"))
    got = _run(kin, str(tmp_path / f"k{kin}.npz"), wide, extra)
    q = ref["q"]
    assert set(int(c) for c in q) >= {1, 2, 3, 4, 5}, q  # every band16 width present
    for key in ("lml-1", "grad-1", "info-1", "lml3", "grad3", "info3", "mean", "var"):
        assert np.array_equal(ref[key], got[key]), (kin, key, ref[key], got[key])
    assert not ref["info-1"].any() and not ref["info3"].any()
    # and the deferred evaluation equals the undeferred one
    assert np.array_equal(ref["lml-1"], ref["lml3"]) and np.array_equal(ref["grad-1"], ref["grad3"])
