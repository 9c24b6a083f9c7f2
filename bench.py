#!/usr/bin/env python
"""Benchmark: GP fits/sec at N=4096, 1-D RBF (SquaredExponential), fp64, on MI355X.

BASELINE.json metric: "GP fits/sec (N=4096, 1-D RBF) at 1/2/4/8 MI355X; log-ML rel-err vs
GPflow". Workload = config C2: synthetic 1-D series, X = arange(N) day
offsets, Y = z-scored random-Fourier-feature draw from SE(ℓ=64) + N(0, 0.1²) noise.

One *fit* is exactly one inner iteration of GPR/model_trainer.py:14-25 for the SE kernel:
GPflow defaults (σ²=1, ℓ=1), σn²=1e-5 fixed, scipy L-BFGS-B (maxiter=100) on the
unconstrained variables to termination, then predict_f at the N training points.

One *step* = fitting `--fits` independent series per GPU (each driven by its own unmodified
scipy L-BFGS-B, from a fresh GPR model at GPflow defaults) through `--width` resident device
slots with continuous batching: the evaluations of all resident fits run as batched device
passes (`--groups` concurrent device batches), and a slot is refilled as soon as its fit
converges and has run its predict_f. The K timed steps are streamed back to back through the
slots (the next step's fits take slots as the previous step's finish; no drain between steps),
bracketed by one barrier + synchronize on each side. For N > 1 GPUs the step ends with an
RCCL all_gather of every fit's (θ*, loss*, nfev, last predicted mean/var) — the per-asset
hand-off to the portfolio step.
Inputs are resident in HBM before the timed region. Each rank fits its own series
(seed = rank * fits + f): weak scaling.

Launch: python bench.py [--gpus 1 --steps K --warmup W]; for N>1 the driver uses
python -m torch.distributed.run --nproc-per-node N bench.py --gpus N ...
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

N_POINTS = 4096
NOISE = 1e-5
MAXITER = 100
FP64_PEAK_TFLOPS = 78.6  # MI355X dense FP64 (matrix) datasheet peak, /opt/skills/guides/MI355X_MICROARCH.md


def synthetic_series(n: int, seed: int, lengthscale: float = 64.0, n_features: int = 2048,
                     noise_std: float = 0.1):
    """C2 generator (same recipe as oracle.gp_oracle.synthetic_series, restated here so the
    product bench does not import the oracle)."""
    rng = np.random.default_rng(seed)
    x = np.arange(n, dtype=np.float64)
    w = rng.standard_normal(n_features) / lengthscale
    b = rng.uniform(0.0, 2.0 * math.pi, n_features)
    coef = rng.standard_normal(n_features)
    f = np.sqrt(2.0 / n_features) * (np.cos(np.outer(x, w) + b) @ coef)
    y = f + noise_std * rng.standard_normal(n)
    y = (y - y.mean()) / y.std(ddof=1)
    return x.reshape(-1, 1), y.reshape(-1, 1)


def job_cpus():
    """CPUs this process may run on: the affinity mask, capped by a cgroup-v2 CPU quota when
    one is set (a container's mask can list every CPU of the host while its quota allots a
    share). Returns (cpus, affinity_count, quota_cpus_or_None)."""
    aff = len(os.sched_getaffinity(0))
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
        if q != "max":
            quota = max(1, math.ceil(int(q) / int(per)))
    except (OSError, ValueError):
        pass
    return (min(aff, quota) if quota else aff), aff, quota


def cpu_baseline(n: int, nfev_per_fit: float, evals: int = 3):
    """The oracle (numpy/scipy/OpenBLAS restatement of the GPflow CPU path) timed on this
    host on a bounded sample: `evals` loss+grad evaluations and one predict_f at N, scaled to
    fits/s with the GPU run's mean nfev per fit. BLAS runs on every CPU available to the job
    (job_cpus(); `cores`); a second, 1-thread sample (1 evaluation + 1 predict_f) gives the
    single-core figure SURVEY §8d asks for."""
    from oracle import gp_oracle as O
    import threadpoolctl

    x, y = synthetic_series(n, 0)
    m = O.OGPR(x, y, O.OSquaredExponential(), noise_variance=NOISE)
    m.noise.trainable = False
    cores, aff, quota = job_cpus()

    def timed(n_evals):
        m.kernel.lengthscales.value = 1.0
        m.loss_and_grad_u()  # warm-up (page in, thread pool up)
        t0 = time.perf_counter()
        for k in range(n_evals):
            m.kernel.lengthscales.value = 1.0 + 4.0 * k
            m.loss_and_grad_u()
        t_e = (time.perf_counter() - t0) / n_evals
        t0 = time.perf_counter()
        m.predict_f(x)
        return t_e, time.perf_counter() - t0

    with threadpoolctl.threadpool_limits(limits=cores, user_api="blas"):
        t_eval, t_pred = timed(evals)
    with threadpoolctl.threadpool_limits(limits=1, user_api="blas"):
        t_eval1, t_pred1 = timed(1)
    t_fit = nfev_per_fit * t_eval + t_pred
    t_fit1 = nfev_per_fit * t_eval1 + t_pred1
    cpu_model = None
    try:
        with open("/proc/cpuinfo") as f:
            cpu_model = next((l.split(":", 1)[1].strip() for l in f if l.startswith("model name")), None)
    except OSError:
        pass
    return {
        "value": 1.0 / t_fit,
        "unit": "fits/s",
        "cores": int(cores),
        "kind": "port",
        "sample": (f"oracle/gp_oracle.py (numpy {np.__version__} + OpenBLAS, fp64) on this host, "
                   f"BLAS on {cores} threads: {evals} loss+grad evals ({t_eval:.3f} s each) + 1 predict_f "
                   f"({t_pred:.3f} s) at N={n}; fit time = mean GPU nfev/fit ({nfev_per_fit:.1f}) x eval + "
                   "predict"),
        "eval_s": t_eval,
        "predict_s": t_pred,
        "value_1core": 1.0 / t_fit1,
        "eval_s_1core": t_eval1,
        "predict_s_1core": t_pred1,
        "cpu_model": cpu_model,
        "host_cpus_visible": aff,
        "cgroup_cpu_quota": quota,
    }


def band_traffic(kernel_key, problems_per_launch):
    """HBM bytes per launch of the banded roofline kernel from the committed PMC summary of
    THAT kernel (profiles/<round>_band*_traffic.json whose "kernel" names kernel_key, written by
    tools/pmc_summary.py from separate FETCH_SIZE / WRITE_SIZE passes): bytes per problem x
    the launch's problem count. None when absent."""
    import glob
    root = os.path.dirname(os.path.abspath(__file__))
    files = []
    for f in sorted(glob.glob(os.path.join(root, "profiles", "*_band*traffic.json"))):
        d = json.load(open(f))
        if any(kernel_key in k for k in d.get("kernel", [])):
            files.append((f, d))
    if not files:
        return None, None
    f, d = files[-1]
    return d["hbm_bytes_per_problem"] * problems_per_launch, os.path.relpath(f, root)


def band_problem_flops(n, p, fwd):
    """2·64³ block-product flops of one problem's fused sweep (gpx_api.hip band_fused_flops)."""
    U = 2.0 * 64 ** 3
    nb = (n + 63) // 64
    f = 0.0
    for k in range(nb):
        q = min(p, nb - 1 - k)
        f += (2.0 / 3.0 + q + q * (q + 1) / 2.0) * U if fwd else (1.0 + q + q * q + q) * U
    return f


def contract_traffic(n, flops_per_launch):
    """HBM bytes per contraction launch from the committed PMC summary of this bench command
    (profiles/<round>_contract_traffic.json, written by tools/pmc_summary.py from separate
    rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes): bytes per problem x the launch's average
    problem count (alg flops per launch / alg flops per problem). None when absent."""
    import glob
    files = sorted(glob.glob(os.path.join(os.path.dirname(os.path.abspath(__file__)), "profiles",
                                          "*_contract_traffic.json")))
    if not files:
        return None, None
    d = json.load(open(files[-1]))
    npad = (n + 63) // 64 * 64
    if d.get("Np") != npad:
        return None, None
    per_problem = sum(2.0 * (i + 1) * (npad - i) for i in range(npad))
    problems = flops_per_launch / per_problem
    return d["hbm_bytes_per_problem"] * problems, os.path.relpath(files[-1], os.path.dirname(os.path.abspath(__file__)))


def main():
    # HIP hardware queues for this process, set before the runtime starts (torch is imported
    # below): the 4 device batches each evaluate on their own stream (+ one forked stream for
    # the p = 2 class), and with the runtime's default 4 queues some of those streams share a
    # queue and serialise (3 batches: 2460–2630 fits/s at 4 queues, 2800 at 8)
    os.environ["GPU_MAX_HW_QUEUES"] = os.environ.get("GPX_HW_QUEUES", "8")
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    # 20 timed steps of 256 fits: enough fits to keep the 576 slots streaming (with 2 steps the
    # timed region is one wave of fits and its slowest fits' tail) and to average over the
    # batches' phase alignment (10-step runs spread by about ±8 %)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--fits", type=int, default=int(os.environ.get("GPX_BENCH_FITS", 256)),
                    help="independent series fitted per GPU per step")
    # band storage (25 MiB per slot) lets 1536 slots stay resident: every device call then
    # carries ~320 problems, so the chip's 512 two-per-CU places stay full while a batch is on
    # the host (dense layout, 384 MiB per slot: 576 slots, 3833–3955 fits/s; band storage
    # 3 x 1536: 4205, 4 x 1536: 4263–4415, 6 x 1536 on 16 queues: 4446 — tools/bench_sweep3.sh)
    ap.add_argument("--width", type=int, default=int(os.environ.get("GPX_BENCH_WIDTH", 1536)),
                    help="resident device slots (continuous-batching width)")
    ap.add_argument("--groups", type=int, default=int(os.environ.get("GPX_BENCH_GROUPS", 4)),
                    help="device batches kept in flight by the one host thread (host/device overlap)")
    ap.add_argument("--wide-slots", type=int, default=int(os.environ.get("GPX_BENCH_WIDE", 0)),
                    help="slots of an extra device batch that takes the evaluations whose band is wider "
                         "than one 64-block (0: none)")
    ap.add_argument("--storage", choices=("band", "dense"), default=os.environ.get("GPX_BENCH_STORAGE", "band"),
                    help="slot workspace: band storage (gpx_batch_create_banded, 25 MiB per slot) or the "
                         "dense N x N layout (384 MiB per slot)")
    ap.add_argument("--points", "--n", dest="n", type=int, default=N_POINTS,
                    help="points per series (use --points under torch.distributed.run, whose parser takes --n)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    os.environ.setdefault("GPX_DEVICE", str(local_rank))

    import torch
    import torch.distributed as dist
    import portfoliooptgp_amd as gpx
    from portfoliooptgp_amd.engine import Engine
    from portfoliooptgp_amd.kernels import compile_spec
    from portfoliooptgp_amd.models import predict_f_batch

    # GPX_BENCH_BACKEND=gloo + GPX_DEVICE=0: rehearsal of the multi-rank path with every rank
    # on one GPU (collectives on host tensors); the real run is RCCL, one GPU per rank
    backend = os.environ.get("GPX_BENCH_BACKEND", "nccl")
    gpu = int(os.environ["GPX_DEVICE"])
    torch.cuda.set_device(gpu)
    dev = torch.device(f"cuda:{gpu}")
    cdev = dev if backend == "nccl" else torch.device("cpu")
    if world > 1:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)

    F, W, n = args.fits, args.width, args.n
    seeds = [rank * F + f for f in range(F)]
    data = [synthetic_series(n, s) for s in seeds]
    Xd = [torch.as_tensor(x, device=dev) for x, _ in data]  # resident in HBM before timing
    Yd = [torch.as_tensor(y, device=dev) for _, y in data]
    def make_model(f):
        # GPflow defaults (σ²=1, ℓ=1), σn² = 1e-5 frozen — GPR/model_trainer.py:15-17
        m = gpx.models.GPR(data=(Xd[f], Yd[f]), kernel=gpx.kernels.SquaredExponential(), device=gpu)
        m.likelihood.variance.assign(NOISE)
        gpx.set_trainable(m.likelihood.variance, False)
        return m

    def make_models():
        return [make_model(f) for f in range(F)]

    # W resident device slots (continuous batching), sized for N-point problems, split into
    # `groups` independent device batches evaluated concurrently on their own streams
    G = max(1, args.groups)
    WS = max(0, min(args.wide_slots, W // 4)) if G > 1 else 0
    per = (W - WS) // G
    sizes = [per] * G + ([WS] if WS > 0 else [])
    proto = make_models()
    # slot shapes only: every slot is rebound to its fit's series when the fit starts
    engines = [Engine([Xd[(g * per + i) % F] for i in range(sz)], [Yd[(g * per + i) % F] for i in range(sz)],
                      [compile_spec(proto[(g * per + i) % F].kernel, 1) for i in range(sz)], device=gpu,
                      band_storage=args.storage == "band" and not (WS > 0 and g == G))
               for g, sz in enumerate(sizes)]
    NG = len(engines)
    engines[0].ctx.set_profiling(True)
    opt = gpx.optimizers.Scipy()

    traces = []
    stats = []

    def run_steps(k):
        """k steps (k × F fits, each from GPflow defaults) streamed back to back through the
        slots — the next step's fits fill slots as the previous step's finish, no drain in
        between — then every fit's summary row, all_gathered across ranks."""
        # every fit's model is built inside the timed region, on demand (as the reference's loop
        # builds each GPR right before fitting it), while the host thread waits for the device
        models = gpx.optimizers.ModelStream(k * F, lambda i: make_model(i % F), input_dim=1, max_points=n,
                                            device=gpu)
        res, preds = opt.minimize_stream(models, width=W, engine=engines, predict_train=True, groups=NG,
                                         options=dict(maxiter=MAXITER), wide_group=WS > 0)
        if getattr(opt, "last_trace", None):
            traces.append(opt.last_trace)
        if getattr(opt, "last_stats", None):
            stats.append(dict(opt.last_stats))
        # per fit [ℓ*, σ²*, loss*, nfev, mean and var of its last training-point prediction]:
        # the host columns as one table, the device ones as two gathers (one tensor per fit
        # and column cost ~0.3 s at 5120 fits)
        host = torch.tensor([[m.kernel.lengthscales.value, m.kernel.variance.value, float(r.fun), float(r.nfev)]
                             for m, r in zip(models, res)], dtype=torch.float64).to(dev)
        mu = torch.cat([p[0][-1:, 0] for p in preds])
        var = torch.cat([p[1][-1:, 0] for p in preds])
        summary = torch.cat([host, mu[:, None], var[:, None]], dim=1)
        if world > 1:
            summary = summary.to(cdev)
            gathered = [torch.empty_like(summary) for _ in range(world)]
            dist.all_gather(gathered, summary)
            summary = torch.cat(gathered)
        return res, summary

    if args.warmup > 0:
        run_steps(args.warmup)
    for e in engines:
        e.reset_timing()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    # trace markers (a ~1 us spin kernel) delimit the timed region in a rocprofv3 kernel trace,
    # so tools/trace_check.py can average the same contraction launches the bench timed
    torch.cuda._sleep(1000)
    res, summary = run_steps(args.steps)
    nfev = [r.nfev for r in res]
    torch.cuda._sleep(1000)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    tms = [e.last_timing() for e in engines]

    class _Tm:  # timing summed over the device batches
        pass
    tm = _Tm()
    for f in ("contract_ms_total", "contract_launches", "contract_alg_flops", "eval_ms_total", "evals",
              "band_ms_total", "band_calls", "band_evals", "band_p_sum", "band_fallbacks", "shadow_evals",
              "shadow_predicts"):
        setattr(tm, f, sum(getattr(t, f) for t in tms))
    # the roofline's fused-sweep launches: the narrow batches' (p <= 1 class), not the wide
    # batch's p = 2 sweeps
    for f in ("band_fwd_ms_total", "band_bwd_ms_total", "band_fused_launches", "band_fwd_flops", "band_bwd_flops"):
        setattr(tm, f, sum(getattr(t, f) for t in tms[:G]))
    if world > 1:
        t = torch.tensor([elapsed], device=cdev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        nf = torch.tensor([float(sum(nfev)), float(len(nfev)), float(tm.evals)], device=cdev,
                          dtype=torch.float64)
        dist.all_reduce(nf)
        nfev_mean = float(nf[0] / nf[1])
        evals_all = float(nf[2])  # device evaluations over all ranks
    else:
        nfev_mean = float(np.mean(nfev))
        evals_all = float(tm.evals)

    total_fits = F * args.steps * world
    value = total_fits / elapsed
    # isolated calibration (after the timed region, not part of `value`): one evaluation of a
    # full device batch with nothing else on the GPU, to separate the contraction kernel's own
    # rate from the sharing with the concurrent batch during the timed steps
    iso = None
    if G > 1:
        e0 = engines[0]
        if e0.band_storage:  # the dense path's own rate needs dense-layout slots (128 of them)
            e0 = Engine([Xd[i % F] for i in range(128)], [Yd[i % F] for i in range(128)],
                        [compile_spec(proto[0].kernel, 1)] * 128, device=gpu)
        th = np.ones((e0.B, 16))
        th[:, :3] = [40.0, 1.0, NOISE]
        e0.lml_grad(list(range(e0.B)), th)  # warm
        e0.reset_timing()
        e0.lml_grad(list(range(e0.B)), th)
        ti = e0.last_timing()
        iso = ti.contract_alg_flops / (ti.contract_ms_total * 1e-3) / 1e12 if ti.contract_ms_total else None
    contract_ms = tm.contract_ms_total / max(tm.contract_launches, 1.0)
    contract_flops = tm.contract_alg_flops / max(tm.contract_launches, 1.0)
    achieved = contract_flops / (contract_ms * 1e-3) / 1e12 if contract_ms > 0 else 0.0
    traffic, traffic_src = contract_traffic(n, contract_flops)
    eval_alg = (n ** 3 + 2 * 3 * n ** 2) * evals_all  # SURVEY §8d F_eval(N), P=2, all ranks (dense count)
    # the kernel with the most device time in the timed region: the fused banded sweep kernels
    # when the fits' evaluations take the banded path (C2: every evaluation), else the dense
    # fused K⁻¹ + gradient contraction
    band_kernels = {
        "band_fwd1_kernel (p<=1 class: banded Cholesky + z solve, one workgroup per problem)":
            (tm.band_fwd_ms_total, tm.band_fwd_flops, "band_fwd1_kernel", True),
        "band_bwd1_kernel<1> (p<=1 class: selected inversion + alpha solve + gradient contraction)":
            (tm.band_bwd_ms_total, tm.band_bwd_flops, "band_bwd1_kernel", False),
    }
    kname, (kms, kflops, kkey, kfwd) = max(band_kernels.items(), key=lambda kv: kv[1][0])
    if kms > tm.contract_ms_total:
        launches = tm.band_fused_launches
        b_ms = kms / max(launches, 1.0)
        b_flops = kflops / max(launches, 1.0)
        b_ach = b_flops / (b_ms * 1e-3) / 1e12 if b_ms > 0 else 0.0
        # problems per timed launch: its flops / one p-weighted problem's (mean p of the class)
        from_p = tm.band_p_sum / max(tm.band_evals, 1.0)
        # problems per timed launch (the p <= 1 class): its flops / one p = 1 problem's
        b_traffic, b_src = band_traffic(kkey, b_flops / band_problem_flops(n, 1, kfwd))
        f2 = min(max(from_p - 1.0, 0.0), 1.0)
        per_eval = ((1.0 - f2) * (band_problem_flops(n, 1, True) + band_problem_flops(n, 1, False))
                    + f2 * (band_problem_flops(n, 2, True) + band_problem_flops(n, 2, False)))
        chip_ach = tm.band_evals * per_eval / elapsed / 1e12
        roofline = {
            "kernel": kname, "bound": "mfma", "achieved": b_ach, "peak": FP64_PEAK_TFLOPS, "unit": "TFLOP/s",
            "frac": b_ach / FP64_PEAK_TFLOPS, "traffic": b_traffic, "traffic_source": b_src,
            "traffic_unit": "bytes/launch", "mean_p_blocks": from_p,
            "avg_launch_ms": b_ms, "launches": launches, "alg_flops_per_launch": b_flops,
            # the whole chip over the timed region: every banded evaluation's block products
            # (both sweeps; p = 1 and p = 2 classes mixed by the mean band width) / wall time.
            # Several device batches' launches overlap, so this is the MFMA rate the chip sustains
            "chip_achieved": chip_ach, "chip_frac": chip_ach / FP64_PEAK_TFLOPS,
            "note": ("banded path: each launch walks its problems' 64 block steps in sequence, one "
                     "workgroup (one CU) per problem; achieved = the 64^3 block products issued "
                     "(2*64^3 flops each, leaf 2/3 of one) / launch duration. The chain of "
                     "dependent block steps, not MFMA or HBM throughput, sets the duration "
                     "(DESIGN.md §3c); traffic: the kernel's profiles/<round>_band*_traffic.json"),
            "dense_contraction_isolated": iso, "dense_contraction_frac_isolated": iso / FP64_PEAK_TFLOPS if iso else None,
        }
    else:
        roofline = {
            "kernel": "gemm_kernel<128,T,N,EPI_CONTRACT1> (K^-1 = W^T W fused with the gradient contraction)",
            "bound": "mfma",
            "achieved": achieved,
            "peak": FP64_PEAK_TFLOPS,
            "unit": "TFLOP/s",
            "frac": achieved / FP64_PEAK_TFLOPS,
            "traffic": traffic,
            "traffic_unit": "bytes/launch",
            "traffic_source": traffic_src,
            "avg_launch_ms": contract_ms,
            "launches": tm.contract_launches,
            "alg_flops_per_launch": contract_flops,
            "note": (f"timed region runs {G} device batches concurrently on separate streams, so the "
                     "kernel's launches share the GPU with the other batch's kernels; "
                     "achieved_isolated = the same kernel alone (one full batch, after the timed region)"
                     if G > 1 else "one device batch"),
            "achieved_isolated": iso,
            "frac_isolated": iso / FP64_PEAK_TFLOPS if iso else None,
        }
    out = {
        "metric": "GP fits/sec (N=4096, 1-D RBF)",
        "value": value,
        "unit": "fits/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic (C2 generator, seeded per rank/series)",
        "config": {"workload": "C2: exact GPR fit, synthetic 1-D series, N=4096, SquaredExponential, "
                               "fp64, sigma_n^2=1e-5 fixed, L-BFGS-B maxiter=100 + predict_f(X_train)",
                   "N": n, "fits_per_gpu_per_step": F, "device_slots": W, "device_batches": NG, "slot_storage": args.storage,
                   "wide_batch_slots": WS,
                   "kernel": "SquaredExponential",
                   "parallelism": f"independent fits, {world} process(es) x 1 GPU, RCCL all_gather of results"},
        "nfev_mean": nfev_mean,
        "band_path": {"evals": tm.band_evals, "dense_evals": tm.evals - tm.band_evals,
                      "mean_p_blocks": tm.band_p_sum / max(tm.band_evals, 1.0),
                      "check_fallbacks": tm.band_fallbacks, "fallback_slot_evals": tm.shadow_evals,
                      "fallback_slot_predicts": tm.shadow_predicts,
                      "ms_per_call": tm.band_ms_total / max(tm.band_calls, 1.0),
                      "problems_per_call": tm.band_evals / max(tm.band_calls, 1.0)},
        "evals_per_s": evals_all / elapsed,
        # the dense algorithm's count F_eval(N) x evaluations / wall time: what the same job
        # would have to sustain on the dense path (the banded path does far fewer flops)
        "eval_dense_equiv_tflops": eval_alg / elapsed / 1e12,
        "roofline": roofline,
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(n, nfev_mean)
        out["cpu_baseline"]["gpu_over_cpu"] = value / out["cpu_baseline"]["value"]
    if stats and rank == 0:
        out["driver_stats_last_call"] = stats[-1]
    if traces and rank == 0:
        with open(os.environ.get("GPX_TRACE_OUT", "rounds_trace.json"), "w") as f:
            json.dump([[list(e) for e in tr] for tr in traces], f)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
