"""The multi-rank fit path with REAL device fits: two ranks (gloo, both on cuda:0) run
distributed.fit_assets over 7 C2/C3-shaped series (LPT shard by series_cost, each rank's shard
fitted through the continuous-batching driver, one all_gather of the packed results); every
rank ends with every asset's result, equal to the single-process fit of that asset (same N:
bit-identical arithmetic), in the Portfolio list format (portfolio_inputs)."""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_two_rank_gloo_fit_assets_with_device_fits(tmp_path):
    sys.path.insert(0, os.path.join(HERE, "helpers"))
    from dist_fit_worker import series
    from portfoliooptgp_amd import distributed as D
    port = _free_port()
    procs, outs = [], []
    for r in range(2):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE="2", LOCAL_RANK="0", MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port), GPX_DEVICE="0")
        out = tmp_path / f"rank{r}.json"
        outs.append(out)
        procs.append(subprocess.Popen([sys.executable, os.path.join(HERE, "helpers", "dist_fit_worker.py"), str(out)],
                                      env=env))
    for p in procs:
        assert p.wait(timeout=240) == 0
    views = [json.load(open(o)) for o in outs]
    assert sorted(views[0]["shard"] + views[1]["shard"]) == list(range(7))
    assert views[0]["res"] == views[1]["res"]                 # every rank holds every asset
    s, h = series()
    solo = D.fit_assets(s, h)                                  # this process alone (world 1)
    for i in range(7):
        g = views[0]["res"][str(i)]
        assert g["loss"] == solo[i]["loss"] and g["nfev"] == solo[i]["nfev"]
        np.testing.assert_array_equal(g["mean"], solo[i]["mean"][:, 0])
        np.testing.assert_array_equal(g["var"], solo[i]["var"][:, 0])
    # the Portfolio lists (Multi-Input_GPR/Portfolio/portfolio.py:111-124)
    rets, vols = D.portfolio_inputs({int(k): {"mean": np.asarray(v["mean"])[:, None], "var": np.asarray(v["var"])[:, None]}
                                     for k, v in views[1]["res"].items()}, order=list(range(7)))
    assert len(rets) == 7 and all(len(r) == 5 and np.asarray(r[0]).shape == (1,) for r in rets)


def test_nccl_world1_torchrun_device_gather(tmp_path):
    """The RCCL path of the result hand-off, run for real: one rank under
    `torch.distributed.run` with the "nccl" backend. distributed.fit_assets fits 3 series on the
    device and all_gathers the packed rows as DEVICE tensors (all_gather_results' nccl branch);
    the gathered results equal this process's own fits of the same series (no process group), and
    all_gather_results / gather_table return the rows unchanged at world 1."""
    sys.path.insert(0, os.path.join(HERE, "helpers"))
    from nccl_world1 import series
    from portfoliooptgp_amd import distributed as D
    out = tmp_path / "rank0.json"
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", GPX_DEVICE="0")
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT"):
        env.pop(k, None)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", "1",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(HERE, "helpers", "nccl_world1.py"), str(out)]
    p = subprocess.run(cmd, env=env, timeout=240)
    assert p.returncode == 0
    v = json.load(open(out))
    assert v["world"] == 1 and v["backend"] == "nccl"
    np.testing.assert_array_equal(np.asarray(v["gathered_rows"]), np.arange(12.0).reshape(3, 4))
    np.testing.assert_array_equal(np.asarray(v["table"]), [[0.0, 7.0], [1.0, 6.0], [2.0, 5.0]])
    s, h = series()
    solo = D.fit_assets(s, h)
    assert sorted(int(k) for k in v["res"]) == [0, 1, 2]
    for i in range(3):
        g = v["res"][str(i)]
        assert g["loss"] == solo[i]["loss"] and g["nfev"] == solo[i]["nfev"]
        np.testing.assert_array_equal(g["mean"], solo[i]["mean"][:, 0])
        np.testing.assert_array_equal(g["var"], solo[i]["var"][:, 0])
