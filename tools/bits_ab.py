"""Bit identity of two library builds on the band16 sweeps (the in-tree libgpx.so and
GPX_LIB_ALT): logML and gradient of 64 C2 problems at a spread of lengthscales (Q = 1..8), each
build in its own process, on the sweeps route (BITS_ROUTE=bcr: the block-cyclic-reduction route).
usage: python tools/bits_ab.py (GPU box)"""
import json
import os
import subprocess
import sys

CHILD = r'''
import os, sys, json, numpy as np
sys.path.insert(0, os.environ["REPO"])
import portfoliooptgp_amd as gpx
gpx.set_default_band_route(os.environ.get("BITS_ROUTE", "sweeps"))
from portfoliooptgp_amd.engine import Engine
from portfoliooptgp_amd.kernels import compile_spec
import bench
n = int(os.environ["BITS_N"])
ells = np.linspace(0.4, 3.2, 64)
data = [bench.synthetic_series(n, s) for s in range(64)]
eng = Engine([d[0] for d in data], [d[1] for d in data], [compile_spec(gpx.kernels.SquaredExponential(), 1)] * 64,
             band_storage=True)
th = np.ones((64, 16)); th[:, 0] = ells; th[:, 1] = 0.8; th[:, 2] = 1e-5
l, g, info = eng.lml_grad(list(range(64)), th)
print(json.dumps({"lml": [float(v).hex() for v in l], "g": [float(v).hex() for v in g[:, :3].ravel()],
                  "info": info.tolist()}))
'''


def run(lib, n):
    env = dict(os.environ, REPO=os.path.dirname(os.path.dirname(os.path.abspath(__file__))), BITS_N=str(n))
    if lib:
        env["GPX_LIB"] = lib
    p = subprocess.run([sys.executable, "-c", CHILD], env=env, capture_output=True, text=True)
    if p.returncode != 0:
        sys.stderr.write(p.stderr[-4000:])
        raise SystemExit(f"child failed ({lib or 'in-tree'}, n={n})")
    return json.loads(p.stdout.strip().splitlines()[-1])


for n in (4096, 4001):  # (a whole number of 16-row blocks, and a ragged last block)
    a = run(None, n)
    b = run(os.environ["GPX_LIB_ALT"], n)
    same_l = sum(x == y for x, y in zip(a["lml"], b["lml"]))
    same_g = sum(x == y for x, y in zip(a["g"], b["g"]))
    print(json.dumps({"n": n, "lml_identical": same_l, "of": len(a["lml"]), "grad_identical": same_g,
                      "of_g": len(a["g"]), "info_equal": a["info"] == b["info"]}))
