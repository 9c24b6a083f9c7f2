"""A/B of dense-path settings (environment variables) on config C4 shapes: bit identity of logML
and gradient of B problems at a fixed θ, and the evaluation time, each setting in its own process.
usage: python tools/dense_ab.py [--b 32] [--reps 5] "GPX_X=0" "GPX_X=1" ...   (GPU box; JSON lines)"""
import argparse
import json
import os
import subprocess
import sys

CHILD = r'''
import os, sys, json, time, numpy as np
sys.path.insert(0, os.environ["REPO"])
import torch
from portfoliooptgp_amd import kernels as K
from portfoliooptgp_amd.engine import Engine
from portfoliooptgp_amd.kernels import compile_spec
from bench import synthetic_series
B, reps, n = int(os.environ["AB_B"]), int(os.environ["AB_REPS"]), 4096
data = []
for s in range(B):
    rng = np.random.default_rng(100 + s)
    X = np.hstack([np.cumsum(rng.standard_normal((n, 4)), axis=0), np.linspace(0.0, 1.0, n)[:, None]])
    X = (X - X.mean(0)) / X.std(0, ddof=1)
    data.append((X, synthetic_series(n, s)[1]))
eng = Engine([d[0] for d in data], [d[1] for d in data], [compile_spec(K.Matern52(), 5)] * B)
th = np.ones((B, 16)); th[:, 0] = np.linspace(0.5, 3.0, B); th[:, 1] = 1.3; th[:, 2] = 1e-3
act = list(range(B))
l, g, info = eng.lml_grad(act, th)
torch.cuda.synchronize()
ts = []
for _ in range(reps):
    t = time.perf_counter()
    eng.lml_grad(act, th)
    torch.cuda.synchronize()
    ts.append(time.perf_counter() - t)
for b1 in (1, 4):
    eng.lml_grad(act[:b1], th)
torch.cuda.synchronize()
t1, small = {}, []
for b1 in (1, 4):
    t = time.perf_counter()
    for _ in range(reps):
        ls, gs_, _ = eng.lml_grad(act[:b1], th)
    torch.cuda.synchronize()
    t1[b1] = (time.perf_counter() - t) / reps * 1e3
    small += [float(v).hex() for v in ls[:b1]] + [float(v).hex() for v in gs_[:b1, :3].ravel()]
# (the small calls' bits against the same problems' in the B-problem call)
same_small = small == ([float(v).hex() for v in l[:1]] + [float(v).hex() for v in g[:1, :3].ravel()]
                       + [float(v).hex() for v in l[:4]] + [float(v).hex() for v in g[:4, :3].ravel()])
print(json.dumps({"small_calls_match_full": same_small, "small": small,
                  "lml": [float(v).hex() for v in l], "g": [float(v).hex() for v in g[:, :3].ravel()],
                  "info": info.tolist(), "ms_median": float(np.median(ts)) * 1e3, "ms_min": min(ts) * 1e3,
                  "ms_b1": t1[1], "ms_b4": t1[4]}))
'''


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--b", type=int, default=32)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("settings", nargs="+")
    args = ap.parse_args()
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    first = None
    for kv in args.settings:
        env = dict(os.environ, REPO=repo, AB_B=str(args.b), AB_REPS=str(args.reps))
        for item in kv.split():
            k, v = item.split("=", 1)
            env[k] = v
        out = subprocess.run([sys.executable, "-c", CHILD], env=env, capture_output=True, text=True, timeout=300)
        if out.returncode != 0:
            print(out.stderr[-3000:])
            sys.exit(1)
        d = json.loads(out.stdout.strip().splitlines()[-1])
        first = first or d
        same_s = first["small"] == d["small"]
        same_l = sum(x == y for x, y in zip(first["lml"], d["lml"]))
        same_g = sum(x == y for x, y in zip(first["g"], d["g"]))
        print(json.dumps({"setting": kv, "b": args.b, "ms_median": round(d["ms_median"], 2), "ms_min": round(d["ms_min"], 2),
                          "ms_b1": round(d["ms_b1"], 2), "ms_b4": round(d["ms_b4"], 2),
                          "lml_identical_to_first": f"{same_l}/{len(d['lml'])}",
                          "grad_identical_to_first": f"{same_g}/{len(d['g'])}", "info_equal": d["info"] == first["info"],
                          "b1_b4_bits_as_first": same_s, "b1_b4_bits_as_in_full_call": d["small_calls_match_full"]}),
              flush=True)


if __name__ == "__main__":
    main()
