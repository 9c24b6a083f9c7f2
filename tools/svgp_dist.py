"""Sharded SVGP rehearsal: every rank holds N/world rows, one all_reduce of the partial buffer
per evaluation (distributed.svgp_elbo_grad), checked against the unsharded evaluation on rank
0, then a short sharded fit. Launch (1 GPU box, ranks share the card over gloo):
  GPX_DEVICE=0 python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 \\
      --master-port 29533 tools/svgp_dist.py --backend gloo
On an 8-GPU node: --backend nccl (one GPU per rank, GPX_DEVICE unset)."""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=65536)
    ap.add_argument("--m", type=int, default=1024)
    ap.add_argument("--backend", default="nccl")
    ap.add_argument("--iters", type=int, default=5)
    a = ap.parse_args()
    rank, world = int(os.environ.get("RANK", 0)), int(os.environ.get("WORLD_SIZE", 1))
    local = int(os.environ.get("LOCAL_RANK", 0))
    os.environ.setdefault("GPX_DEVICE", str(local))
    import torch
    import torch.distributed as dist
    import portfoliooptgp_amd as gpx
    from portfoliooptgp_amd import distributed as D
    from portfoliooptgp_amd.engine import SVGPEngine
    from portfoliooptgp_amd.kernels import compile_spec

    dev = int(os.environ["GPX_DEVICE"])
    torch.cuda.set_device(dev)
    if world > 1:
        if a.backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device(f"cuda:{dev}"))
        else:
            dist.init_process_group("gloo")
    rng = np.random.default_rng(0)
    X = np.sort(rng.uniform(0, 360, (a.n, 1)), axis=0)
    Y = np.sin(X / 20.0) + 0.1 * rng.standard_normal((a.n, 1))
    Z = np.linspace(0, 360, a.m)[:, None]
    q = rng.standard_normal(a.m) * 0.3
    R = np.tril(rng.standard_normal((a.m, a.m)) * 1e-3)
    R[np.diag_indices(a.m)] = rng.uniform(0.05, 0.2, a.m)
    theta = np.ones(16)
    theta[:3] = [2.0, 1.0, 1e-4]
    k = gpx.kernels.SquaredExponential()
    sl = D.shard_rows(a.n, world, rank)
    eng = SVGPEngine(X[sl], Y[sl], compile_spec(k, 1), a.m, num_data=a.n, n_total=a.n, device=dev)
    out = D.svgp_elbo_grad(eng, theta, Z, q, R)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.iters):
        out = D.svgp_elbo_grad(eng, theta, Z, q, R)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / a.iters
    res = {"rank": rank, "world": world, "rows": sl.stop - sl.start, "elbo": out[0], "eval_ms": dt * 1e3}
    if rank == 0:
        full = SVGPEngine(X, Y, compile_spec(k, 1), a.m, num_data=a.n, device=dev).elbo_grad(theta, Z, q, R)
        res["elbo_unsharded"] = full[0]
        res["rel_elbo"] = abs(out[0] - full[0]) / abs(full[0])
        res["max_rel_grad"] = max(float(np.abs(x - y).max() / (1 + np.abs(y).max())) for x, y in zip(out[1:], full[1:]))
    print(json.dumps(res), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
