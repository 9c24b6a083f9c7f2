"""Multi-process (world_size 2, gloo on CPU) coverage of the sharded fit + result gather.

The GPU fitter is swapped for a deterministic CPU stand-in (this container has no GPU); what
is tested is the distributed plumbing: LPT sharding, the single all_gather of packed results,
and the Portfolio input format."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from portfoliooptgp_amd import distributed as D


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _series(k):
    rng = np.random.default_rng(k)
    n = 20 + 7 * k
    x = np.arange(n, dtype=np.float64)[:, None]
    y = rng.standard_normal((n, 1))
    return x, y


def _stand_in_fit(series, horizons):
    out = []
    for (x, y), h in zip(series, horizons):
        out.append(dict(loss=float(np.sum(y * y)), nfev=len(x), theta=[float(len(x)), float(y.mean())],
                        mean=np.full(len(h), float(y.mean())), var=np.full(len(h), float(y.var()))))
    return out


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        series = [_series(k) for k in range(7)]
        horizons = [np.arange(len(s[0]), len(s[0]) + 5, dtype=np.float64)[:, None] for s in series]
        res = D.fit_assets(series, horizons, fit_fn=_stand_in_fit, n_theta=2)
        means, varis = D.portfolio_inputs(res, order=list(range(7)))
        q.put((rank, {i: (r["loss"], r["nfev"], r["theta"].tolist()) for i, r in res.items()},
               [[float(m[0]) for m in a] for a in means]))
    finally:
        dist.destroy_process_group()


def test_lpt_sharding_balances_cubic_costs():
    costs = [D.fit_cost(n) for n in (2048, 2048, 2048, 1024, 1024, 1024, 1024, 1024, 1024, 512)]
    shards = D.shard_lpt(costs, 2)
    loads = [sum(costs[i] for i in s) for s in shards]
    assert sorted(i for s in shards for i in s) == list(range(10))
    assert max(loads) / min(loads) < 1.15
    # one dominant fit goes alone
    sh = D.shard_lpt([D.fit_cost(n) for n in (4096, 2048, 2048, 1024)], 2)
    assert [0] in sh
    # 20 equal fits on 8 ranks -> 3/3/3/3/2/2/2/2
    sh = D.shard_lpt([1.0] * 20, 8)
    assert sorted(len(s) for s in sh) == [2, 2, 2, 2, 3, 3, 3, 3]


def test_pack_unpack_roundtrip():
    res = [dict(loss=1.5, nfev=12, theta=[2.0, 3.0], mean=np.arange(4.0), var=np.ones(4))]
    t = D.pack_results([5], res, horizon=4, n_theta=2)
    back = D.unpack_results(t, 4, 2)
    assert list(back) == [5] and back[5]["nfev"] == 12
    np.testing.assert_array_equal(back[5]["mean"][:, 0], np.arange(4.0))


def test_two_rank_gloo_gather_matches_single_process():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    outs = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    series = [_series(k) for k in range(7)]
    horizons = [np.zeros((5, 1))] * 7
    ref = _stand_in_fit(series, horizons)
    for rank, res, means in outs:
        assert sorted(res) == list(range(7))          # every rank holds every asset
        for i, r in enumerate(ref):
            loss, nfev, theta = res[i]
            assert loss == pytest.approx(r["loss"]) and nfev == r["nfev"]
            assert means[i][0] == pytest.approx(float(series[i][1].mean()))
    assert outs[0][1] == outs[1][1]


def _svgp_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from oracle import gp_oracle as O
        from tests.svgp_numpy_shard import NumpySVGPShard
        X, Y, Z, qm, R = _svgp_data()
        sl = D.shard_rows(len(X), world, rank)
        eng = NumpySVGPShard(O.OSquaredExponential(lengthscales=1.3, variance=0.8), X[sl], Y[sl],
                             len(Z), num_data=len(X), n_total=len(X))
        theta = np.ones(16)
        theta[:3] = [1.3, 0.8, 0.05]
        out = D.svgp_elbo_grad(eng, theta, Z, qm, R)
        q.put((rank, out[0], [np.asarray(a).tolist() for a in out[1:]]))
    finally:
        dist.destroy_process_group()


def _svgp_data():
    rng = np.random.default_rng(21)
    X = rng.uniform(0, 10, (103, 1))
    Y = np.sin(X) + 0.1 * rng.standard_normal((103, 1))
    Z = rng.uniform(0, 10, (7, 1))
    R = np.tril(rng.standard_normal((7, 7)) * 0.1)
    R[np.diag_indices(7)] = rng.uniform(0.4, 1.0, 7)
    return X, Y, Z, rng.standard_normal(7) * 0.3, R


def test_shard_rows_partition():
    for n, w in ((10, 3), (65536, 8), (5, 8)):
        sl = [D.shard_rows(n, w, r) for r in range(w)]
        assert sum(s.stop - s.start for s in sl) == n
        assert all(sl[i].stop == sl[i + 1].start for i in range(w - 1))


def test_two_rank_gloo_svgp_allreduce_matches_oracle():
    """C5's multi-GPU decomposition: each rank's partial sums over its rows, one all_reduce,
    the replicated finish — equal to the single-process oracle ELBO and gradients."""
    from oracle import gp_oracle as O
    from oracle import svgp_oracle as S
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_svgp_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    outs = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    X, Y, Z, qm, R = _svgp_data()
    om = S.OSVGP(O.OSquaredExponential(lengthscales=1.3, variance=0.8), Z, num_data=len(X),
                 noise_variance=0.05, q_mu=qm, q_sqrt=R)
    elbo, g = om.elbo_and_grads(X, Y)
    for rank, e, (gth, gZ, gq, gR) in outs:
        assert e == pytest.approx(elbo, rel=1e-10)
        np.testing.assert_allclose(gth[:2], g["theta"], rtol=1e-7, atol=1e-8)
        assert gth[2] == pytest.approx(g["noise"], rel=1e-7)
        np.testing.assert_allclose(np.asarray(gZ), g["Z"], rtol=1e-7, atol=1e-8)
        np.testing.assert_allclose(gq, g["q_mu"], rtol=1e-7, atol=1e-8)
        np.testing.assert_allclose(np.asarray(gR), g["q_sqrt"], rtol=1e-7, atol=1e-8)
    assert outs[0][1] == outs[1][1]


def test_fit_assets_checkpoint_resumes_at_asset_granularity(tmp_path):
    """A rerun with the same checkpoint prefix fits only the assets without a stored result;
    an asset whose inputs changed is refitted; results equal a fresh run's."""
    series = [_series(k) for k in range(5)]
    horizons = [np.arange(len(s[0]), len(s[0]) + 3, dtype=np.float64)[:, None] for s in series]
    calls = []

    def counting_fit(ss, hs):
        calls.append(len(ss))
        return _stand_in_fit(ss, hs)

    prefix = str(tmp_path / "sweep")
    fresh = D.fit_assets(series, horizons, fit_fn=_stand_in_fit)
    first = D.fit_assets(series, horizons, fit_fn=counting_fit, checkpoint=prefix)
    again = D.fit_assets(series, horizons, fit_fn=counting_fit, checkpoint=prefix)
    assert calls == [5]                       # the rerun fitted nothing
    x2, y2 = series[2]
    series[2] = (x2, y2 + 1.0)
    changed = D.fit_assets(series, horizons, fit_fn=counting_fit, checkpoint=prefix)
    assert calls == [5, 1]                    # only the changed asset
    for res in (first, again):
        for i in range(5):
            assert res[i]["loss"] == fresh[i]["loss"]
            np.testing.assert_array_equal(res[i]["mean"], fresh[i]["mean"])
    assert changed[2]["loss"] == pytest.approx(float(np.sum((y2 + 1.0) ** 2)))
    assert changed[0]["loss"] == fresh[0]["loss"]


def test_fit_assets_checkpoint_discarded_under_another_fit_configuration(tmp_path):
    """A checkpoint written by one fit protocol is not reused by another (different fit_fn,
    different bound arguments, or a different fit_config): everything is refitted."""
    import functools
    series = [_series(k) for k in range(3)]
    horizons = [np.arange(len(s[0]), len(s[0]) + 2, dtype=np.float64)[:, None] for s in series]
    calls = []

    def fit_a(ss, hs, scale=1.0):
        calls.append(("a", len(ss), scale))
        return _stand_in_fit(ss, hs)

    def fit_b(ss, hs):
        calls.append(("b", len(ss)))
        return _stand_in_fit(ss, hs)

    prefix = str(tmp_path / "cfg")
    D.fit_assets(series, horizons, fit_fn=fit_a, checkpoint=prefix, fit_config={"maxiter": 100})
    D.fit_assets(series, horizons, fit_fn=fit_a, checkpoint=prefix, fit_config={"maxiter": 100})
    assert calls == [("a", 3, 1.0)]          # same configuration: resumed, nothing refitted
    D.fit_assets(series, horizons, fit_fn=fit_a, checkpoint=prefix, fit_config={"maxiter": 50})
    assert calls[-1] == ("a", 3, 1.0) and len(calls) == 2   # other fit_config: refitted
    D.fit_assets(series, horizons, fit_fn=fit_b, checkpoint=prefix, fit_config={"maxiter": 50})
    assert calls[-1] == ("b", 3) and len(calls) == 3         # other fit function: refitted
    D.fit_assets(series, horizons, fit_fn=functools.partial(fit_a, scale=2.0), checkpoint=prefix,
                 fit_config={"maxiter": 50})
    assert calls[-1] == ("a", 3, 2.0) and len(calls) == 4    # other bound arguments: refitted
    assert D.config_fingerprint(fit_a, 1) != D.config_fingerprint(fit_b, 1)


def test_band_aware_fit_cost_and_shard():
    """LPT costs follow the path a fit takes: a C2-like day-offset series of N = 4096 starts on
    the 16-row band sweeps (Q = 3 16-blocks at GPflow's ℓ = 1: (N/16)·(Q+1) block-step work per
    evaluation), wider bands on the 64-row sweeps (N·w²), the same N on normalised inputs runs
    dense (N³); every cost in device seconds per evaluation, so the classes compare."""
    x_days = np.arange(4096.0)
    assert D.band_blocks_estimate(x_days) == 1
    assert D.band_blocks_estimate(x_days / 4096.0) is None        # dense
    assert D.band_blocks_estimate(np.arange(300.0)) is None       # < 8 blocks: dense
    assert D.band_blocks_estimate(np.arange(4096.0), lengthscale=1.72) == 2
    assert D.band16_estimate(x_days) == 3
    assert D.band16_estimate(x_days, lengthscale=1.6) == 4
    assert D.band16_estimate(x_days, lengthscale=1.72) == 5
    assert D.band16_estimate(x_days, lengthscale=2.2) is None     # wider than 5 16-blocks
    assert D.band16_estimate(x_days / 4096.0) is None
    assert D.series_cost(x_days) == D.fit_cost(4096, 1, 3)
    assert D.fit_cost(4096, 1, 4) / D.fit_cost(4096, 1, 3) == pytest.approx(5 / 4)
    assert D.fit_cost(2048, 1, 3) == pytest.approx(D.fit_cost(4096, 1, 3) / 2)
    assert D.series_cost(x_days / 4096.0) == D.fit_cost(4096) == pytest.approx(1 / 832.0)
    # one dense N=2048 fit outweighs eight banded N=4096 ones: it goes alone
    series = [np.arange(4096.0)] * 8 + [np.arange(2048.0) / 2048.0]
    sh = D.shard_lpt([D.series_cost(x) for x in series], 2)
    assert [8] in sh


def _skewed_mix():
    """Mixed N and band width: day offsets at N = 4096 / 2048 / 1024 with unit spacing (Q = 3)
    and at 0.7-day spacing (ℓ = 1 spans more points: Q = 4); C3-like."""
    xs = ([np.arange(4096.0)] * 3 + [np.arange(4096.0) * 0.7] * 2 + [np.arange(2048.0)] * 5
          + [np.arange(2048.0) * 0.7] * 3 + [np.arange(1024.0)] * 7)
    return [(x[:, None], np.zeros((len(x), 1))) for x in xs]


def _skew_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        series = _skewed_mix()
        horizons = [np.zeros((2, 1))] * len(series)
        mine = []

        def fit(ss, hs):   # stand-in fitter: records this rank's shard by series length/spacing
            out = []
            for x, _ in ss:
                mine.append(D.series_cost(x))
                out.append(dict(loss=float(len(x)), nfev=1, theta=[float(x[1, 0] - x[0, 0]), 1.0],
                                mean=np.zeros(2), var=np.ones(2)))
            return out
        res = D.fit_assets(series, horizons, fit_fn=fit, n_theta=2)
        q.put((rank, sum(mine), len(mine), sorted(res)))
    finally:
        dist.destroy_process_group()


def test_two_rank_gloo_skewed_mix_balances_band16_costs():
    """A skewed mix (N = 4096 / 2048 / 1024, bands of Q = 3 and Q = 4 16-blocks) sharded over 2
    gloo ranks by fit_assets' default band16-aware series_cost: every asset fitted once and
    gathered on both ranks, and the two ranks' device costs within 10 % (the round-3 64-row cost
    model, N·(64(p+1))², weighed both band widths alike)."""
    costs = [D.series_cost(x) for x, _ in _skewed_mix()]
    assert len(set(np.round(np.array(costs) / costs[-1], 6))) == 5   # five cost classes
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_skew_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    outs = sorted(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    loads = [o[1] for o in outs]
    assert sum(o[2] for o in outs) == len(costs)
    assert all(o[3] == list(range(len(costs))) for o in outs)
    assert max(loads) / min(loads) < 1.10, loads
    assert sum(loads) == pytest.approx(sum(costs))


def _portfolio_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        g = np.load(os.path.join(os.path.dirname(__file__), "golden", "portfolio.npz"))
        means, varis = g["means"], g["vars"]
        A, H = means.shape
        series = [(np.arange(10.0 + i)[:, None], np.zeros((10 + i, 1))) for i in range(A)]
        horizons = [np.zeros((H, 1))] * A

        def fit(ss, hs):   # stand-in fitter: the golden per-asset predictions as the fit results
            out = []
            for x, _ in ss:
                i = len(x) - 10
                out.append(dict(loss=0.0, nfev=1, theta=[1.0, 1.0], mean=means[i], var=varis[i]))
            return out
        res = D.fit_assets(series, horizons, fit_fn=fit, n_theta=2)
        rets, vols = D.portfolio_inputs(res, order=list(range(A)))
        out = {}
        for tag, log_ret in (("log", True), ("cml", False)):
            mus, sig, sd = zip(*[D.portfolio_day_moments(rets, vols, day, log_ret) for day in range(H)])
            out[tag] = (np.stack(mus).tolist(), np.stack(sig).tolist(), np.stack(sd).tolist())
        q.put((rank, out))
    finally:
        dist.destroy_process_group()


def test_portfolio_format_against_reference_optimizer_golden():
    """f3: per-asset predictions gathered over 2 gloo ranks, rebuilt into the lists
    Portfolio(...) indexes (Multi-Input_GPR/Portfolio/portfolio.py:111-124), give per day the
    same μ / Σ / σ the REFERENCE's Optimizer computes from those lists
    (Multi-Input_GPR/optimization/optimizer.py:20-56; tests/golden/portfolio.npz, made by
    tests/golden/make_ref_golden.py importing the reference module)."""
    g = np.load(os.path.join(os.path.dirname(__file__), "golden", "portfolio.npz"))
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_portfolio_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    outs = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, out in outs:
        for tag in ("log", "cml"):
            mu, sig, sd = (np.asarray(a) for a in out[tag])
            np.testing.assert_array_equal(mu, g[f"{tag}|mu"])
            np.testing.assert_array_equal(sig, g[f"{tag}|Sigma"])
            np.testing.assert_array_equal(sd, g[f"{tag}|std"])


def _fingerprint_worker(q):
    import portfoliooptgp_amd as gpx
    from portfoliooptgp_amd.kernels import compile_spec
    spec = compile_spec(gpx.kernels.Exponential(active_dims=slice(0, 4)) * gpx.kernels.Exponential(active_dims=slice(4, 5)), 5)
    q.put(D.config_fingerprint(_stand_in_fit, {"spec": spec, "maxiter": 100, "x": np.arange(3.0)}))


def test_config_fingerprint_is_stable_across_processes():
    """a compiled kernel spec (ctypes structure) in fit_config hashes by its bytes,
    so two processes with the same configuration agree (and a checkpoint is reused); a value
    whose repr is a memory address is refused instead of silently changing every run."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_fingerprint_worker, args=(q,)) for _ in range(2)]
    for p in procs:
        p.start()
    fps = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    assert fps[0] == fps[1]

    class Opaque:
        pass
    with pytest.raises(ValueError, match="stable representation"):
        D.config_fingerprint(_stand_in_fit, {"k": Opaque()})


def _strong_rows(ids, steps, total):
    """A deterministic stand-in for the bench's per-fit summary rows (global index first)."""
    ids = np.asarray(ids, dtype=np.float64)
    g = np.concatenate([ids + s * total for s in range(steps)])
    return np.stack([g, np.sin(g), g % 7.0, np.sqrt(g + 1.0)], axis=1)


def _strong_worker(rank, world, port, q, total, procs, steps):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        plan = D.strong_plan([1.0] * total, world, procs)
        local = np.concatenate([_strong_rows(ids, steps, total) for ids in plan[rank]])
        q.put((rank, D.gather_table(local).tolist()))
    finally:
        dist.destroy_process_group()


def test_strong_scaling_plan_and_table_world2_equals_world1():
    """bench.py --scaling strong: the fixed batch is split over the ranks and
    their host processes by strong_plan, and the all_gathered table (gather_table) is the same
    fits in the same order at world 2 as at world 1."""
    import bench
    total, procs, steps = 203, 3, 2
    for world in (1, 2, 8):
        plan = D.strong_plan([1.0] * total, world, procs)
        flat = sorted(i for pr in plan for p in pr for i in p)
        assert flat == list(range(total))
        sizes = [sum(len(p) for p in pr) for pr in plan]
        assert max(sizes) - min(sizes) <= 1
    one = D.gather_table(np.concatenate([_strong_rows(ids, steps, total)
                                         for ids in D.strong_plan([1.0] * total, 1, procs)[0]]))
    assert np.array_equal(one[:, 0], np.arange(total * steps))
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_strong_worker, args=(r, 2, port, q, total, procs, steps)) for r in range(2)]
    for p in ps:
        p.start()
    outs = [q.get(timeout=120) for _ in ps]
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    for _, tab in outs:
        np.testing.assert_array_equal(np.asarray(tab), one)
    # the bench's own plan: every fit of the batch exactly once over ranks x host processes
    args = bench.parse_args(["--scaling", "strong", "--total-fits", "1000", "--procs", "8"])
    ids = bench.strong_fit_ids(args, 2, 8)
    assert sorted(i for pr in ids for p in pr for i in p) == list(range(1000))
