"""One rank of tests/test_distributed_gpu.py: fit_assets over a gloo group whose ranks share
cuda:0 (the multi-rank path with real device fits; the driver's 8-GPU run uses RCCL, one GPU per
rank). Writes this rank's view of the gathered results as JSON to argv[1]."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch.distributed as dist  # noqa: E402


def series():
    from oracle import gp_oracle as O
    out = [O.synthetic_series(2048 if i % 3 else 1024, seed=300 + i) for i in range(7)]
    hor = [x[-1:] + np.arange(1, 6, dtype=np.float64)[:, None] for x, _ in out]
    return out, hor


def main():
    dist.init_process_group("gloo")
    try:
        from portfoliooptgp_amd import distributed as D
        s, h = series()
        res = D.fit_assets(s, h)
        shard = D.shard_lpt([D.series_cost(x) for x, _ in s], dist.get_world_size())[dist.get_rank()]
        out = {"rank": dist.get_rank(), "shard": shard,
               "res": {str(i): {"loss": r["loss"], "nfev": r["nfev"], "theta": list(map(float, r["theta"])),
                                "mean": r["mean"][:, 0].tolist(), "var": r["var"][:, 0].tolist()}
                       for i, r in res.items()}}
        with open(sys.argv[1], "w") as f:
            json.dump(out, f)
    finally:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
