"""Bit identity of two library builds on the dense paths (the in-tree libgpx.so and GPX_LIB_ALT):
logML and gradient of C4-shaped problems (N = 4096, D = 5, Matern52: the recursion and its
leaf128 launches; Exponential x Exponential and RQ + Linear: the general contraction) and of small problems (N = 89 / 19: the one-launch kernels), each build in its
own process. usage: GPX_LIB_ALT=... python tools/bits_dense_ab.py (GPU box)"""
import json
import os
import subprocess
import sys

CHILD = r'''
import os, sys, json, numpy as np
sys.path.insert(0, os.environ["REPO"])
import portfoliooptgp_amd as gpx
from portfoliooptgp_amd.engine import Engine
from portfoliooptgp_amd.kernels import compile_spec
out = {}
for n, D, B in ((4096, 5, 3), (89, 1, 4), (19, 1, 4)):
    data = []
    for s in range(B):
        rng = np.random.default_rng(100 + s)
        X = np.cumsum(rng.standard_normal((n, D)), axis=0)
        X = (X - X.mean(0)) / X.std(0, ddof=1)
        data.append((X, np.sin(X[:, :1]) + 0.1 * rng.standard_normal((n, 1))))
    eng = Engine([d[0] for d in data], [d[1] for d in data], [compile_spec(gpx.kernels.Matern52(), D)] * B)
    th = np.ones((B, 16)); th[:, 0] = np.linspace(1.5, 3.0, B); th[:, 1] = 0.8; th[:, 2] = 1e-3
    l, g, info = eng.lml_grad(list(range(B)), th)
    out[str(n)] = {"lml": [float(v).hex() for v in l], "g": [float(v).hex() for v in g[:, :3].ravel()], "info": info.tolist()}
# the general contraction (two-term specs): C4's Exponential(dims 0-3) x Exponential(dim 4), and a
# sum with a non-stationary term, at N = 4096, D = 5
K = gpx.kernels
for name, kern in (("expxexp", K.Exponential(active_dims=slice(0, 4)) * K.Exponential(active_dims=slice(4, 5))),
                   ("rq+lin", K.RationalQuadratic() + K.Linear())):
    data = []
    for s in range(2):
        rng = np.random.default_rng(200 + s)
        X = np.cumsum(rng.standard_normal((4096, 5)), axis=0)
        X = (X - X.mean(0)) / X.std(0, ddof=1)
        data.append((X, np.sin(X[:, :1]) + 0.1 * rng.standard_normal((4096, 1))))
    eng = Engine([d[0] for d in data], [d[1] for d in data], [compile_spec(kern, 5)] * 2)
    th = np.ones((2, 16)); th[:, 0] = [1.7, 2.4]; th[:, 4] = 1e-3
    l, g, info = eng.lml_grad([0, 1], th)
    out[name] = {"lml": [float(v).hex() for v in l], "g": [float(v).hex() for v in g[:, :5].ravel()], "info": info.tolist()}
print(json.dumps(out))
'''


def run(lib):
    env = dict(os.environ, REPO=os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    if lib:
        env["GPX_LIB"] = lib
    p = subprocess.run([sys.executable, "-c", CHILD], env=env, capture_output=True, text=True)
    if p.returncode != 0:
        sys.stderr.write(p.stderr[-4000:])
        raise SystemExit(f"child failed ({lib or 'in-tree'})")
    return json.loads(p.stdout.strip().splitlines()[-1])


a = run(None)
b = run(os.environ["GPX_LIB_ALT"])
for n in a:
    print(json.dumps({"n": n, "lml_identical": sum(x == y for x, y in zip(a[n]["lml"], b[n]["lml"])), "of": len(a[n]["lml"]),
                      "grad_identical": sum(x == y for x, y in zip(a[n]["g"], b[n]["g"])), "of_g": len(a[n]["g"]),
                      "info_equal": a[n]["info"] == b[n]["info"]}))
