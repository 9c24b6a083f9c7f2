"""Multi-GPU: independent per-asset fits sharded over ranks, results gathered once.

The reference fits its assets in a sequential Python loop (GPR/main.py:23 over tickers,
Multi-Input_GPR/main.py:535 over assets) and hands per-asset predicted means / variances to
the portfolio step (Multi-Input_GPR/main.py:555-574 -> Portfolio(assets, predicted_values,
predicted_variances), Multi-Input_GPR/Portfolio/portfolio.py:92-165). Here:

* one process per GPU (torch.distributed; backend "nccl" = RCCL over xGMI on MI355X,
  "gloo" for CPU tests);
* fits are assigned to ranks longest-processing-time first on their cost (device seconds per
  evaluation on the path the fit takes: (N/16)·(Q+1) on the 16-row band sweeps, N·w² on the 64-row
  band sweeps, N³ dense; no communication while fitting);
* every rank fits its shard through the continuous-batching driver and predicts its
  horizon;
* ONE all_gather of a packed fp64 tensor (θ*, loss*, nfev, mean[H], var[H] per asset) is the
  only data-path collective; rank 0 (or every rank) rebuilds the Portfolio input lists.
"""
from __future__ import annotations

import hashlib
import heapq
import os
from typing import Callable, Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch
import torch.distributed as dist


def shard_lpt(costs: Sequence[float], world: int) -> List[List[int]]:
    """Longest-processing-time-first assignment of items (by cost) to `world` bins."""
    heap = [(0.0, r) for r in range(world)]
    heapq.heapify(heap)
    out: List[List[int]] = [[] for _ in range(world)]
    for i in sorted(range(len(costs)), key=lambda k: (-costs[k], k)):
        load, r = heapq.heappop(heap)
        out[r].append(i)
        heapq.heappush(heap, (load + float(costs[i]), r))
    for r in out:
        r.sort()
    return out


def band_blocks_estimate(x, lengthscale: float = 1.0, cutoff: float = 38.63) -> Optional[int]:
    """Band width, in 64-row blocks, that a fit on inputs x starts on: the smallest p such that
    every pair of points more than p blocks apart is at least ``cutoff`` lengthscales apart
    (SquaredExponential: exp(−r²/2) underflows to exactly 0 in fp64 beyond r = 38.6; the device
    bounds it the same way from per-block boxes, gpx_api.hip band_width). At GPflow's default
    ℓ = 1 on the reference's unnormalised day offsets (GPR/data_handler.py:42-44) that is one
    block. None when the band does not apply (fewer than 8 blocks, as the device requires, or no
    block offset vanishes): the fit runs dense."""
    x = np.asarray(x, dtype=np.float64)
    x = x.reshape(len(x), -1)
    n = len(x)
    nb = (n + 63) // 64
    if nb < 8:
        return None
    lo = np.array([x[k * 64:(k + 1) * 64].min(0) for k in range(nb)])
    hi = np.array([x[k * 64:(k + 1) * 64].max(0) for k in range(nb)])
    for p in range(0, nb - 1):
        d = p + 1   # every offset >= d must vanish; the box gap only grows with d for sorted inputs
        ok = True
        for dd in range(d, nb):
            gap = np.maximum(0.0, np.maximum(lo[dd:] - hi[:nb - dd], lo[:nb - dd] - hi[dd:]))
            if np.sqrt((gap * gap).sum(1)).min() / lengthscale < cutoff:
                ok = False
                break
        if ok:
            return p
    return None


BAND16_MAX_Q = 5     # widest band of the 16-row sweeps (gpx_host.h kBand16MaxQ)
BAND16_MAX_D = 8     # input columns they stage per block (kBand16MaxD)


def band16_estimate(x, lengthscale: float = 1.0, cutoff: float = 38.63) -> Optional[int]:
    """Band width Q, in 16-row blocks, that the 16-row sweeps take for a fit on inputs x (the
    device's band_width16 bound from per-16-row boxes, gpx_api.hip): the smallest Q such that
    every pair of points more than Q blocks apart is at least ``cutoff`` lengthscales apart.
    None when that path does not take the series (the 64-row band is wider than 2 blocks, Q > 5,
    more than 8 input columns, or fewer than 8 64-blocks)."""
    x = np.asarray(x, dtype=np.float64)
    x = x.reshape(len(x), -1)
    p = band_blocks_estimate(x, lengthscale, cutoff)
    if p is None or p > 2 or x.shape[1] > BAND16_MAX_D:
        return None
    n = len(x)
    nb = (n + 15) // 16
    lo = np.array([x[k * 16:(k + 1) * 16].min(0) for k in range(nb)])
    hi = np.array([x[k * 16:(k + 1) * 16].max(0) for k in range(nb)])
    for q in range(0, min(BAND16_MAX_Q, nb - 1) + 1):
        ok = True
        for dd in range(q + 1, min(nb, q + 1 + 2 * BAND16_MAX_Q)):
            gap = np.maximum(0.0, np.maximum(lo[dd:] - hi[:nb - dd], lo[:nb - dd] - hi[dd:]))
            if np.sqrt((gap * gap).sum(1)).min() / lengthscale < cutoff:
                ok = False
                break
        if ok:
            return max(q, 1)
    return None


# Device seconds per evaluation at full-chip throughput, per unit of each path's work model
# (MI355X, round-3 measurements): band16 sweeps ~(N/16)·(Q+1) — a chain of N/16
# block steps whose cost grows ~linearly in Q+1 (290k / 228k / 183k C2 evaluations/s at Q = 3 /
# 4 / 5); the 64-row band sweeps N·w², w = 64(p+1) (60k evaluations/s at N = 4096, p = 1); the
# dense path N³ (832 evaluations/s at N = 4096)
_K16 = 1.0 / 290e3 / (256 * 4)
_K64 = 1.0 / 60e3 / (4096 * 128.0 ** 2)
_KDENSE = 1.0 / 832.0 / 4096.0 ** 3


def fit_cost(n: int, band_blocks: Optional[int] = None, band16_q: Optional[int] = None) -> float:
    """Relative device cost of one exact-GP fit (per evaluation; fits are assumed to take the
    same number of evaluations), in seconds at full-chip throughput: the 16-row band sweeps
    (band16_q: Q 16-blocks) ∝ (N/16)·(Q+1); the 64-row band sweeps (band of p
    64-blocks, §3c) ∝ N·w², w = 64(p+1); the dense path ∝ N³."""
    if band16_q is not None:
        return _K16 * (n / 16.0) * (band16_q + 1)
    if band_blocks is None:
        return _KDENSE * float(n) ** 3
    w = 64.0 * (band_blocks + 1)
    return _K64 * float(n) * w * w


def series_cost(x) -> float:
    """fit_cost of a series for the default fitter (SE at GPflow's default ℓ = 1), on the path
    the device routes it to at that ℓ."""
    return fit_cost(len(x), band_blocks_estimate(x), band16_estimate(x))


def pack_results(indices: Sequence[int], results: Sequence[dict], horizon: int, n_theta: int) -> torch.Tensor:
    """[k, 4 + n_theta + 2H] fp64 rows: index, loss, nfev, ok, θ..., mean[H], var[H]."""
    width = 4 + n_theta + 2 * horizon
    t = torch.full((len(indices), width), float("nan"), dtype=torch.float64)
    for row, (i, r) in enumerate(zip(indices, results)):
        t[row, 0] = i
        t[row, 1] = r["loss"]
        t[row, 2] = r["nfev"]
        t[row, 3] = 1.0
        th = np.asarray(r["theta"], dtype=np.float64)[:n_theta]
        t[row, 4:4 + len(th)] = torch.as_tensor(th)
        t[row, 4 + n_theta:4 + n_theta + horizon] = torch.as_tensor(np.asarray(r["mean"]).reshape(-1)[:horizon])
        t[row, 4 + n_theta + horizon:] = torch.as_tensor(np.asarray(r["var"]).reshape(-1)[:horizon])
    return t


def unpack_results(table: torch.Tensor, horizon: int, n_theta: int) -> Dict[int, dict]:
    out = {}
    for row in table.cpu().numpy():
        if not np.isfinite(row[0]) or row[3] != 1.0:
            continue
        out[int(row[0])] = dict(
            loss=float(row[1]), nfev=int(row[2]), theta=row[4:4 + n_theta].copy(),
            mean=row[4 + n_theta:4 + n_theta + horizon].reshape(-1, 1).copy(),
            var=row[4 + n_theta + horizon:].reshape(-1, 1).copy())
    return out


def all_gather_results(local: torch.Tensor, n_items: int, group=None) -> torch.Tensor:
    """One all_gather of the packed per-asset rows (padded to the largest shard)."""
    world = dist.get_world_size(group)
    backend = dist.get_backend(group)
    dev = torch.device("cuda", torch.cuda.current_device()) if backend == "nccl" else torch.device("cpu")
    k = torch.tensor([local.shape[0]], device=dev)
    ks = [torch.zeros_like(k) for _ in range(world)]
    dist.all_gather(ks, k, group=group)
    kmax = int(max(int(x.item()) for x in ks))
    pad = torch.full((kmax, local.shape[1]), float("nan"), dtype=torch.float64, device=dev)
    pad[: local.shape[0]] = local.to(dev)
    bufs = [torch.empty_like(pad) for _ in range(world)]
    dist.all_gather(bufs, pad, group=group)
    return torch.cat(bufs).cpu()


def strong_plan(costs: Sequence[float], world: int, procs: int = 1) -> List[List[List[int]]]:
    """A FIXED batch of fits (strong scaling: the same total work whatever the world size) split
    over `world` ranks by shard_lpt on their costs, then each rank's fits over its `procs` host
    processes in contiguous runs: plan[rank][proc] = the global fit indices that process fits.
    Deterministic, so every rank and helper process derives the same plan on its own."""
    plan = []
    for mine in shard_lpt(costs, world):
        k = len(mine)
        cut = [k * p // procs for p in range(procs + 1)]
        plan.append([mine[cut[p]:cut[p + 1]] for p in range(procs)])
    return plan


def gather_table(local, group=None) -> np.ndarray:
    """Rows keyed by a global index in column 0 (fp64), from every rank: one all_gather
    (all_gather_results: device tensors on the nccl backend, host tensors on gloo), padding rows
    dropped, sorted by the index — the same table whatever the world size."""
    t = torch.as_tensor(np.ascontiguousarray(local, dtype=np.float64))
    if dist.is_available() and dist.is_initialized() and dist.get_world_size(group) > 1:
        t = all_gather_results(t, len(t), group=group)
    a = t.cpu().numpy()
    a = a[np.isfinite(a[:, 0])]
    return a[np.argsort(a[:, 0], kind="stable")]


def portfolio_inputs(gathered: Dict[int, dict], order: Sequence[int]) -> Tuple[list, list]:
    """Per-asset lists of per-day [1]-arrays, the shape Portfolio(...) indexes as
    returns[i][day][0] (Multi-Input_GPR/Portfolio/portfolio.py:111-124)."""
    means = [[np.asarray(gathered[i]["mean"][d]) for d in range(len(gathered[i]["mean"]))] for i in order]
    varis = [[np.asarray(gathered[i]["var"][d]) for d in range(len(gathered[i]["var"]))] for i in order]
    return means, varis


def portfolio_day_moments(returns, variances, day: int, log_return: bool = True):
    """What the portfolio step computes from the gathered lists on ``day``: the indexing of
    Portfolio.evaluate_portfolio (Multi-Input_GPR/Portfolio/portfolio.py:111-124: returns[i][0][0]
    on day 0, returns[i][:(day+1)] afterwards, sqrt(variances[i][day][0]) for the std devs)
    followed by the reference Optimizer's set_predictions (day 0), set_cml_log_return
    (log returns) or set_predictions_cml (Multi-Input_GPR/optimization/optimizer.py:20-56).
    Returns (mu [A], Sigma [A, A] diagonal, std_devs [A]). Host code, the same numpy calls as
    the reference (pinned against its own outputs by tests/golden/portfolio.npz)."""
    A = len(returns)
    if day == 0:
        mu = np.array([returns[i][0][0] for i in range(A)])
        sigma = np.diag(np.array([variances[i][0][0] for i in range(A)]))
        std = [np.sqrt(variances[i][0][0]) for i in range(A)]
    else:
        rets = [returns[i][:(day + 1)] for i in range(A)]
        vols = [variances[i][:(day + 1)] for i in range(A)]
        std = [np.sqrt(variances[i][day][0]) for i in range(A)]
        if log_return:
            mu = np.array([np.sum(r) for r in rets])
        else:
            mu = np.array([np.prod([1 + r for r in rl]) - 1 for rl in rets])
        sigma = np.diag(np.array([np.sum(v) for v in vols]))
    return mu, sigma, np.asarray(std, dtype=np.float64)


def asset_fingerprint(x, y, horizon) -> str:
    """Content hash of one asset's fit inputs (training series and prediction inputs)."""
    h = hashlib.sha1()
    for a in (x, y, horizon):
        a = np.ascontiguousarray(np.asarray(a, dtype=np.float64))
        h.update(str(a.shape).encode())
        h.update(a.tobytes())
    return h.hexdigest()


def _canonical(obj) -> str:
    """A run-independent text form of a fit configuration value: containers element by
    element, numpy arrays and ctypes structures (a compiled gpx_kernel_spec) by their bytes,
    scalars and strings by repr. A value whose repr carries a memory address (' at 0x', the
    default object repr) has no stable form — hashing it would change the fingerprint on every
    run and silently discard every checkpoint — so it is refused."""
    import ctypes
    if isinstance(obj, dict):
        return "{" + ",".join(f"{_canonical(k)}:{_canonical(v)}" for k, v in
                              sorted(obj.items(), key=lambda kv: repr(kv[0]))) + "}"
    if isinstance(obj, (list, tuple)):
        return ("[" if isinstance(obj, list) else "(") + ",".join(_canonical(v) for v in obj) + ")"
    if isinstance(obj, np.ndarray):
        return f"ndarray{obj.dtype.str}{obj.shape}:{np.ascontiguousarray(obj).tobytes().hex()}"
    if isinstance(obj, (ctypes.Structure, ctypes.Array)):
        return f"{type(obj).__name__}:{bytes(obj).hex()}"
    r = repr(obj)
    if " at 0x" in r:
        raise ValueError(f"fit configuration value {r} has no stable representation (its repr holds a "
                         "memory address); pass plain values, arrays or a compiled kernel spec")
    return r


def config_fingerprint(fit_fn: Callable, fit_config=None) -> str:
    """Hash of what produced a checkpoint's results: the fit function's qualified name (with a
    functools.partial's bound arguments) and the caller's ``fit_config`` (kernel spec, maxiter,
    noise, ...), in the canonical form of ``_canonical`` (so the same configuration hashes the
    same in every process). A rerun whose configuration differs refits everything instead of
    reusing results of another fit protocol."""
    import functools
    parts = []
    f = fit_fn
    while isinstance(f, functools.partial):
        parts.append(_canonical((tuple(f.args), sorted(f.keywords.items()))))
        f = f.func
    parts.append(f"{getattr(f, '__module__', '?')}.{getattr(f, '__qualname__', repr(f))}")
    parts.append(_canonical(fit_config))
    return hashlib.sha1("\x1f".join(parts).encode()).hexdigest()


def _load_checkpoint(path: str, H: int, n_theta: int, config: str = "") -> Dict[str, dict]:
    """{fingerprint: result} of a previous run's rank file (absent, unreadable or written
    under another fit configuration: empty)."""
    if not os.path.exists(path):
        return {}
    try:
        with np.load(path, allow_pickle=False) as z:
            if int(z["H"]) != H or int(z["n_theta"]) != n_theta:
                return {}
            if "config" not in z.files or str(z["config"]) != config:
                return {}
            rows = unpack_results(torch.as_tensor(z["table"]), H, n_theta)
            fps = [str(f) for f in z["fingerprints"]]
            index = [int(i) for i in z["table"][:, 0]]
    except (OSError, KeyError, ValueError):
        return {}
    return {fp: rows[i] for fp, i in zip(fps, index) if i in rows}


def _save_checkpoint(path: str, table: torch.Tensor, fingerprints: Sequence[str], H: int, n_theta: int,
                     config: str = ""):
    tmp = path + ".tmp.npz"
    np.savez(tmp, table=table.numpy(), fingerprints=np.asarray(list(fingerprints), dtype="U40"),
             H=np.int64(H), n_theta=np.int64(n_theta), config=np.asarray(config, dtype="U40"))
    os.replace(tmp, path)


def fit_assets(series: Sequence[Tuple[np.ndarray, np.ndarray]], horizons: Sequence[np.ndarray],
               fit_fn: Optional[Callable] = None, n_theta: int = 2, group=None,
               checkpoint: Optional[str] = None, fit_config=None,
               cost_fn: Optional[Callable] = None) -> Dict[int, dict]:
    """Shard the assets over the ranks of `group`, fit the local shard with `fit_fn`
    (default: GPU exact GPR with a SquaredExponential kernel and σn² = 1e-5 fixed, the
    GPR/model_trainer.py:15-19 protocol, continuous-batched), predict each asset at its
    horizon inputs and all_gather the results. Returns {asset index: result} on every rank.

    ``checkpoint``: path prefix of per-rank result files (``<prefix>.rank<r>.npz``, θ*, loss*,
    nfev and the horizon predictions of each fitted asset, keyed by a content hash of its
    inputs). A rerun with the same prefix (say after a crash of another rank) fits only the
    assets whose results are missing, so a long multi-asset sweep resumes at asset
    granularity; changed inputs are refitted. The file also records a fingerprint of the fit
    configuration (``fit_fn``'s qualified name and bound arguments plus ``fit_config``, e.g. the
    kernel spec / maxiter / noise of a custom fitter); a file written under another
    configuration is discarded. The reference has no checkpointing.

    ``cost_fn(x)``: relative cost of fitting a series for the LPT shard (default ``series_cost``:
    O(N·w²) for the banded fits of the default SE fitter on day offsets, O(N³) for dense ones)."""
    world = dist.get_world_size(group) if dist.is_initialized() else 1
    rank = dist.get_rank(group) if dist.is_initialized() else 0
    cost_fn = cost_fn or series_cost
    shards = shard_lpt([cost_fn(x) for x, _ in series], world)
    mine = shards[rank]
    fit_fn = fit_fn or gpu_fit_shard
    H = max(len(h) for h in horizons)
    fps = {i: asset_fingerprint(series[i][0], series[i][1], horizons[i]) for i in mine} if checkpoint else {}
    path = f"{checkpoint}.rank{rank}.npz" if checkpoint else None
    cfg = config_fingerprint(fit_fn, fit_config) if checkpoint else ""
    done = _load_checkpoint(path, H, n_theta, cfg) if checkpoint else {}
    todo = [i for i in mine if fps.get(i) not in done]
    fitted = fit_fn([series[i] for i in todo], [horizons[i] for i in todo]) if todo else []
    by_index = dict(zip(todo, fitted))
    local = [by_index[i] if i in by_index else done[fps[i]] for i in mine]
    table = pack_results(mine, local, H, n_theta)
    if checkpoint:
        _save_checkpoint(path, table, [fps[i] for i in mine], H, n_theta, cfg)
    if dist.is_available() and dist.is_initialized():  # (world 1 too: a torchrun of one rank takes the same path)
        table = all_gather_results(table, len(series), group)
    return unpack_results(table, H, n_theta)


def gpu_fit_shard(series, horizons, width: int = 32, maxiter: int = 100):
    """Default per-rank fitter: exact GPR (SE kernel, σn² = 1e-5 fixed), L-BFGS-B through the
    continuous-batching driver, then predict_f at each asset's horizon inputs."""
    from . import kernels, models, optimizers
    from .utilities import set_trainable

    ms = []
    for x, y in series:
        m = models.GPR(data=(x, y), kernel=kernels.SquaredExponential())
        m.likelihood.variance.assign(1e-5)
        set_trainable(m.likelihood.variance, False)
        ms.append(m)
    res, preds = optimizers.Scipy().minimize_stream(ms, width=min(width, len(ms)), predict_inputs=list(horizons),
                                                    options=dict(maxiter=maxiter))
    out = []
    for m, r, (mean, var) in zip(ms, res, preds):
        mean, var = mean.cpu().numpy(), var.cpu().numpy()
        out.append(dict(loss=float(r.fun), nfev=int(r.nfev),
                        theta=[p.value for p in m.kernel.parameters],
                        mean=np.asarray(mean).reshape(-1), var=np.asarray(var).reshape(-1)))
    return out


# ----------------------------------------------------------------------------------------
# SVGP over N shards (BASELINE config C5 at 8 GPUs; SURVEY.md §8 e)
# ----------------------------------------------------------------------------------------
def shard_rows(n: int, world: int, rank: int) -> slice:
    """Contiguous, balanced row block of rank (sizes differ by at most one)."""
    base, extra = divmod(n, world)
    lo = rank * base + min(rank, extra)
    return slice(lo, lo + base + (1 if rank < extra else 0))


def svgp_elbo_grad(engine, theta, Z, q_mu, q_sqrt, group=None):
    """One sharded SVGP evaluation: this rank's partial sums (Kmn-side: G = Kmn Kmnᵀ, Kmn g_μ,
    θ/Z contractions, residual sums), ONE all_reduce of the packed partial buffer in place, then
    the replicated O(M³) tail. Every rank returns the same (ELBO, ∂θ, ∂Z, ∂q_mu, ∂q_sqrt)."""
    engine.eval_local(theta, Z, q_mu, q_sqrt)
    if dist.is_initialized() and dist.get_world_size(group) > 1:
        buf = engine.partials
        if buf.is_cuda and dist.get_backend(group) != "nccl":   # gloo: reduce a host copy
            host = buf.cpu()
            dist.all_reduce(host, op=dist.ReduceOp.SUM, group=group)
            buf.copy_(host)
        else:
            dist.all_reduce(buf, op=dist.ReduceOp.SUM, group=group)
    return engine.eval_finish()


def fit_svgp_sharded(model, X_local, Y_local, n_total: int, group=None, engine=None, **scipy_kwargs):
    """Fit ``model`` (models.SVGP) on data sharded by rows over the ranks of ``group``: every
    rank runs the same scipy L-BFGS-B on the all-reduced (hence identical) ELBO gradient, so
    the replicated variational parameters stay bit-identical across ranks. ``engine`` may be
    injected (tests); by default an SVGPEngine on this rank's rows with n_total set."""
    from .engine import SVGPEngine
    from .kernels import compile_spec
    from .optimizers import Scipy
    if engine is None:
        Xl = np.asarray(X_local, dtype=np.float64) if not isinstance(X_local, torch.Tensor) else X_local
        D = 1 if Xl.ndim == 1 else int(Xl.shape[1])
        engine = SVGPEngine(X_local, Y_local, compile_spec(model.kernel, D), model.M,
                            num_data=float(model.num_data if model.num_data is not None else n_total),
                            n_total=n_total, device=model.device)

    def loss_and_grad(variables=None):
        variables = model.trainable_variables if variables is None else variables
        out = svgp_elbo_grad(engine, *model._state(), group=group)
        return model.grads_to_unconstrained(variables, *out)

    def closure():
        return torch.tensor(loss_and_grad()[0], dtype=torch.float64)

    closure._gpx_loss_and_grad = loss_and_grad
    closure._gpx_model = model
    return Scipy().minimize(closure, model.trainable_variables, **scipy_kwargs)
