"""One rank of tests/test_distributed_gpu.py::test_nccl_world1_torchrun_device_gather, started by
`python -m torch.distributed.run --nproc-per-node 1`: the RCCL ("nccl") process group on cuda:0,
distributed.fit_assets with real device fits (its all_gather of the packed results runs on device
tensors over RCCL even at world 1), all_gather_results on a device tensor, and gather_table (the
strong-scaling bench's hand-off). Writes the gathered results as JSON to argv[1]."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def series():
    from oracle import gp_oracle as O
    out = [O.synthetic_series(2048, seed=500 + i) for i in range(3)]
    hor = [x[-1:] + np.arange(1, 4, dtype=np.float64)[:, None] for x, _ in out]
    return out, hor


def main():
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dist.init_process_group("nccl", device_id=torch.device(f"cuda:{local}"))
    try:
        from portfoliooptgp_amd import distributed as D
        assert dist.get_backend() == "nccl"
        s, h = series()
        res = D.fit_assets(s, h)
        dev_rows = torch.arange(12, dtype=torch.float64, device=f"cuda:{local}").reshape(3, 4)
        g = D.all_gather_results(dev_rows, 3)
        tab = D.gather_table(np.array([[2.0, 5.0], [0.0, 7.0], [1.0, 6.0]]))
        out = {"world": dist.get_world_size(), "backend": dist.get_backend(),
               "gathered_rows": g.tolist(), "table": tab.tolist(),
               "res": {str(i): {"loss": r["loss"], "nfev": r["nfev"], "theta": list(map(float, r["theta"])),
                                "mean": r["mean"][:, 0].tolist(), "var": r["var"][:, 0].tolist()}
                       for i, r in res.items()}}
        with open(sys.argv[1], "w") as f:
            json.dump(out, f)
    finally:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
