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
passes (`--groups` concurrent device batches per host process), and a slot is refilled as soon
as its fit converges and has run its predict_f. The K timed steps are streamed back to back
through the slots (no drain between steps), bracketed by one barrier + synchronize on each
side. For N > 1 GPUs the timed region ends with an RCCL all_gather of every fit's (θ*, loss*,
nfev, last predicted mean/var) — the per-asset hand-off to the portfolio step.

Host processes per GPU (``--procs``, default 8, each with one device batch of --width / procs
slots): a process's host work (model construction, L-BFGS-B steps, predictions) and its device
calls alternate, so several processes keep the GPU's queues full. The rank process starts
``procs - 1`` helper processes (multiprocessing "spawn", BEFORE any GPU call in the rank) that
share the GPU; each fits its own slice of the step's series through its own slots and device
batches. All of them finish their warmup and report ready; the rank starts its clock, signals
the helpers and fits its own slice; each helper synchronises its device work and then hands back
its per-fit summary rows and timing through a queue; the rank stops the clock when it has all of
them (and, for N > 1, after the all_gather and a barrier across ranks).

Inputs are resident in HBM before the timed region. Each rank fits its own series (seed =
rank * fits + f): weak scaling.

After the timed region (rank 0, one GPU only; never part of `value`): the CPU baseline, and two
secondary lines the driver times with the rest of the run — config C4 on the dense path
(Matern52, D = 5, N = 4096: fits/s and the fused K⁻¹ + gradient contraction's roofline) and
config C5 (SVGP, N = 65536, M = 1024: ms per ELBO + gradient evaluation).

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
WAVE_SLOTS = 2048        # band16 sweep places: 256 CUs x 4 SIMDs x 2 waves (one wavefront per problem)


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
    # context, not the baseline: the device's own band algorithm restated on the CPU
    # (oracle/band_oracle.py, numpy + LAPACK), whole fits (L-BFGS-B + predict) of C2 series run
    # one per process on every job core, so the GPU/CPU ratio can be split into algorithm and
    # hardware
    same_alg = None
    try:
        from oracle import band_oracle as BO
        seeds = list(range(1000, 1000 + 4 * cores))
        fps, nf_b, s_fit = BO.parallel_fits_per_s(n, seeds, cores, NOISE)
        same_alg = {"value": fps, "unit": "fits/s", "cores": int(cores), "kind": "port (band algorithm)",
                    "sample": (f"oracle/band_oracle.py: {len(seeds)} whole C2 fits at N={n} (block-tridiagonal "
                               "Cholesky + Takahashi selected inverse on the exact-zero band, scipy L-BFGS-B "
                               f"maxiter 100, predict_f at the training inputs), one per process on {cores} "
                               "processes, BLAS single-threaded"),
                    "nfev_mean": nf_b, "seconds_per_fit_1core": s_fit}
    except Exception as e:  # reported, never fatal
        same_alg = {"error": f"{type(e).__name__}: {e}"}
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
        "extrapolated": True,
        "sample": (f"EXTRAPOLATED from a timed sample: oracle/gp_oracle.py (numpy {np.__version__} + OpenBLAS, fp64) "
                   f"on this host, BLAS on {cores} threads: {evals} loss+grad evals ({t_eval:.3f} s each) + 1 "
                   f"predict_f ({t_pred:.3f} s) at N={n}; fit time = mean GPU nfev/fit ({nfev_per_fit:.1f}) x eval "
                   "+ predict (a whole fit is minutes on the CPU)"),
        "eval_s": t_eval,
        "predict_s": t_pred,
        "value_1core": 1.0 / t_fit1,
        "eval_s_1core": t_eval1,
        "predict_s_1core": t_pred1,
        "cpu_model": cpu_model,
        "host_cpus_visible": aff,
        "cgroup_cpu_quota": quota,
        "same_algorithm_context": same_alg,
    }


def band_traffic(kernel_key, problems_per_launch):
    """HBM bytes per launch of the banded roofline kernel from the committed PMC summary of
    THAT kernel (profiles/<round>_band*_traffic.json whose "kernel" names kernel_key, written by
    tools/pmc_summary.py from separate FETCH_SIZE / WRITE_SIZE passes): bytes per problem x
    the launch's problem count. None when absent. The summaries of the inline-K sweeps
    (GPX_B16_INLINE_K=3: no K band through HBM) are named *_kin3_*, and used only on that path."""
    import glob
    root = os.path.dirname(os.path.abspath(__file__))
    kin3 = (int(os.environ.get("GPX_B16_INLINE_K", "3") or 0) & 3) == 3  # (the library's default: 3)
    files = []
    for f in sorted(glob.glob(os.path.join(root, "profiles", "*_band*traffic.json"))):
        if ("_kin3_" in os.path.basename(f)) != kin3:
            continue
        d = json.load(open(f))
        if any(kernel_key in k for k in d.get("kernel", [])):
            files.append((f, d))
    if not files:
        return None, None
    f, d = files[-1]
    return d["hbm_bytes_per_problem"] * problems_per_launch, os.path.relpath(f, root)


def trace_check(kernel_key):
    """The committed rocprofv3 check of the roofline kernel's launch time in the headline layout
    (profiles/<round>_trace_multi.json, tools/trace_multi.py via tools/profile_round5.sh: 8
    concurrent traced instances): trace average vs the instances' HIP events and vs that round's
    default bench line. None when absent."""
    import glob
    root = os.path.dirname(os.path.abspath(__file__))
    files = sorted(glob.glob(os.path.join(root, "profiles", "*_trace_multi.json")))
    if not files:
        return None
    d = json.load(open(files[-1]))
    k = d.get("kernels", {}).get(kernel_key)
    if k is None:
        return None
    return {"source": os.path.relpath(files[-1], root), "trace_avg_launch_ms": k["trace_avg_launch_ms"],
            "rel_diff_trace_vs_instances_hip_events": k["rel_diff_trace_vs_instances"],
            "rel_diff_trace_vs_that_rounds_bench_line": k["rel_diff_trace_vs_reference_bench"]}


def fp64_profile(families):
    """The fp64 VALU work beside the MFMAs of each band16 kernel family, from the committed PMC pass
    (profiles/<round>_fp64_summary.csv, tools/mfma_summary.py via tools/profile_round6.sh: MFMA MOPS
    and the fp64 VALU instruction counts of one instance's launches): per family, the VALU/MFMA
    flop ratio and the VALU/MFMA datapath-cycle ratio, weighted over the family's Q instances by
    MFMA flops. On gfx950 the fp64 MFMA and fp64 VALU share one datapath (profiles/r06_ab.md), so
    these turn the live MFMA flops into the sweeps' whole fp64 load. None when absent."""
    import csv
    import glob
    root = os.path.dirname(os.path.abspath(__file__))
    files = sorted(glob.glob(os.path.join(root, "profiles", "*_fp64_summary.csv")))
    if not files:
        return None
    acc = {f: [0.0, 0.0, 0.0] for f in families}  # MFMA TFLOP, VALU TFLOP, VALU-cycles in MFMA-TFLOP units
    for r in csv.DictReader(open(files[-1])):
        fam = next((f for f in families if f + "<" in r["Kernel_Name"]), None)
        if fam is None or not r.get("fp64_datapath_busy_est"):
            continue
        m, v = float(r["Issued_fp64_TFLOP"]), float(r["VALU_fp64_TFLOP"])
        mb, dp = float(r["MFMA_busy_frac"]), float(r["fp64_datapath_busy_est"])
        acc[fam][0] += m
        acc[fam][1] += v
        acc[fam][2] += m * (dp - mb) / mb if mb > 0 else 0.0
    return {"source": os.path.relpath(files[-1], root),
            "families": {f: {"valu_over_mfma_flops": a[1] / a[0], "valu_over_mfma_datapath_cycles": a[2] / a[0]}
                         for f, a in acc.items() if a[0] > 0}}


def band_problem_flops(n, p, fwd):
    """2·64³ block-product flops of one problem's fused sweep (gpx_api.hip band_fused_flops)."""
    U = 2.0 * 64 ** 3
    nb = (n + 63) // 64
    f = 0.0
    for k in range(nb):
        q = min(p, nb - 1 - k)
        f += (2.0 / 3.0 + q + q * (q + 1) / 2.0) * U if fwd else (1.0 + q + q * q + q) * U
    return f


def fp64_datapath(sweeps, elapsed):
    """The chip's fp64 load in the timed region, MFMA and VALU together: each band16 family's live
    MFMA flops (ms_total x achieved) scaled by its committed VALU/MFMA ratios (fp64_profile) —
    fp64 flops/s and the estimated share of the fp64 datapath's cycles (MFMA 64 cycles per
    16x16x4 tile, a fp64 VALU instruction ~4) over the timed wall. None without the profile."""
    prof = fp64_profile(("band16_fwd_kernel", "band16_bwd_kernel", "band16_wide_kernel"))
    if not prof or not prof["families"]:
        return None
    fl = cyc = mf = 0.0
    for fam, r in prof["families"].items():
        k = sweeps.get(fam)
        if not k or not k["launches"]:
            continue
        m = k["achieved"] * 1e12 * k["ms_total"] * 1e-3  # the family's MFMA flops in the timed region
        mf += m
        fl += m * (1.0 + r["valu_over_mfma_flops"])
        cyc += m * (1.0 + r["valu_over_mfma_datapath_cycles"])
    return {"mfma_tflops": mf / elapsed / 1e12, "mfma_plus_valu_tflops": fl / elapsed / 1e12,
            "datapath_busy_est": cyc / elapsed / 1e12 / FP64_PEAK_TFLOPS, "peak": FP64_PEAK_TFLOPS,
            "ratios": prof["families"], "source": prof["source"],
            "note": "gfx950's fp64 MFMA and fp64 VALU share one datapath (profiles/r06_ab.md, "
                    "tools/micro/mfma_valu_overlap.hip); the band16 sweeps' exps and 16x16 leaf chains are fp64 "
                    "VALU work the MFMA-only frac leaves out; datapath_busy_est = (MFMA cycles + fp64 VALU "
                    "cycles) / (1024 SIMDs x clock x wall), by the committed per-family cycle ratios"}


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




# GpxTiming fields summed over a worker's device batches (all groups), and those summed over the
# narrow groups only (the roofline's fused p <= 1 sweeps)
SUM_FIELDS = ("contract_ms_total", "contract_launches", "contract_alg_flops", "eval_ms_total", "evals",
              "band_ms_total", "band_calls", "band_evals", "band_p_sum", "band_fallbacks", "shadow_evals",
              "shadow_predicts")
NARROW_FIELDS = ("band_fwd_ms_total", "band_bwd_ms_total", "band_fused_launches", "band_fused_p2_launches",
                 "band_fwd_flops", "band_bwd_flops",
                 "band16_fwd_ms_total", "band16_bwd_ms_total", "band16_launches", "band16_evals", "band16_q_sum",
                 "band16_fwd_flops", "band16_bwd_flops", "band16_wave_ms", "band16_wide_ms_total",
                 "band16_wide_launches", "band16_wide_flops", "band16_wide_evals")


def parse_args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    # a step is 6144 fits per GPU, so the driver's 20 steps (122,880 fits over 8192 slots, each
    # slot refilled ~15 times) are a steady-state region of several seconds rather than one
    # fill-and-drain wave (round 3: 256 fits per step, 20 steps = 5120 fits in 8192 slots, a
    # 0.46 s region whose figure moved ±10 % with the step count)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--fits", type=int, default=int(os.environ.get("GPX_BENCH_FITS", 6144)),
                    help="independent fits per GPU per step")
    ap.add_argument("--series", type=int, default=int(os.environ.get("GPX_BENCH_SERIES", 512)),
                    help="distinct synthetic series per GPU (fits cycle over them; generated on the host "
                         "before the timed region)")
    # band storage (25 MiB per slot) lets 8192 slots stay resident (205 GB of the 288): the
    # band16 sweeps run one wavefront per problem and each call is a chain of launches (build,
    # one sweep pair per band width, reduce), so the chip's 2048 two-per-SIMD sweep places stay
    # filled only with several calls' worth of problems in flight (round 3, profiles/r03_sweeps:
    # 4096 slots 7872 fits/s, 6144: 8572-8649, 8192: 8695-9925; 9216 thrashed HBM: 3646)
    ap.add_argument("--width", type=int, default=int(os.environ.get("GPX_BENCH_WIDTH", 8192)),
                    help="resident device slots per GPU (continuous-batching width), split over --procs")
    ap.add_argument("--groups", type=int, default=int(os.environ.get("GPX_BENCH_GROUPS", 1)),
                    help="device batches kept in flight by each host process")
    # a second device batch per process for the slow evaluation classes (Scipy.minimize_stream
    # wide_group, optimizers._wide_classes): the band16 sweeps wider than GPX_NARROW_Q 16-blocks
    # and the 64-row sweeps, so the narrow batch's calls never wait for them
    ap.add_argument("--defer-q", type=int, default=int(os.environ.get("GPX_DEFER_Q", 3)),
                    help="defer the band16 classes wider than this many 16-blocks and the 64-row sweeps (-1: off)")
    ap.add_argument("--wide-slots", type=int, default=int(os.environ.get("GPX_BENCH_WIDE", 0)),
                    help="slots per process of the slow-class device batch, taken from --width (0: one batch)")
    # 8 processes x 2 HIP hardware queues, one device batch of 1024 slots each: the GPU's queue
    # scheduler time-slices once the processes' queues exceed ~16; 8 host threads keep 8 calls in
    # flight (8 x 1 batch: 9925 fits/s, 8 x 2: 9074-9599, 10 x 2: 8228, 12 x 2: 7598, 4 x 2 at
    # 8192 slots: 8695; round 3, profiles/r03_sweeps)
    ap.add_argument("--procs", type=int, default=int(os.environ.get("GPX_BENCH_PROCS", 8)),
                    help="host processes per GPU (the rank + procs-1 spawned helpers)")
    # admission control (optimizers.DeviceAdmission): at most this many evaluation calls of the
    # GPU's host processes on the device at once, so calls complete one after another instead of
    # all together (0: off)
    ap.add_argument("--admission", type=int, default=int(os.environ.get("GPX_BENCH_ADMISSION", 0)),
                    help="device places shared by the GPU's host processes (0: no admission control)")
    ap.add_argument("--storage", choices=("band", "dense"), default=os.environ.get("GPX_BENCH_STORAGE", "band"),
                    help="slot workspace: band storage (gpx_batch_create_banded, 25 MiB per slot) or the "
                         "dense N x N layout (384 MiB per slot)")
    ap.add_argument("--points", "--n", dest="n", type=int, default=N_POINTS,
                    help="points per series (use --points under torch.distributed.run, whose parser takes --n)")
    # strong scaling: a FIXED batch of --total-fits fits per step over all
    # ranks (the reference's per-asset loop is fixed-size: Multi-Input_GPR/main.py:535-552), split by
    # distributed.shard_lpt; the timed region ends with the last rank's all_gather of the result
    # table. The default stays weak scaling (--fits per GPU, the headline metric).
    ap.add_argument("--scaling", choices=("weak", "strong"), default=os.environ.get("GPX_BENCH_SCALING", "weak"))
    ap.add_argument("--total-fits", type=int, default=int(os.environ.get("GPX_BENCH_TOTAL_FITS", 8 * 6144)),
                    help="strong scaling: fits per step over all ranks")
    ap.add_argument("--total-series", type=int, default=int(os.environ.get("GPX_BENCH_TOTAL_SERIES", 8 * 512)),
                    help="strong scaling: distinct series of the batch (fit i fits series i mod this)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-secondary", action="store_true", help="skip the C4 / C5 secondary lines")
    return ap.parse_args(argv)


def strong_fit_ids(args, world, procs):
    """distributed.strong_plan of the fixed batch: plan[rank][proc] = global fit indices. Every
    fit of the C2 batch has the same cost (the same N, the same day-offset inputs, GPflow's default
    start), so LPT deals them out evenly."""
    from portfoliooptgp_amd import distributed as D
    cost = D.series_cost(np.arange(args.n, dtype=np.float64)[:, None])
    return D.strong_plan([cost] * args.total_fits, world, procs)


def share(total, parts, i):
    """Item count of part i when `total` items are split as evenly as possible."""
    return total // parts + (1 if i < total % parts else 0)


def last_points(ts):
    """t[-1, 0] of every [n, 1] prediction tensor in ts (the horizon point of each fit's
    predict_f), by one gather per device buffer the predictions are views of (a call's finished
    fits share one) instead of an indexing op per fit."""
    import torch
    if not ts:
        return torch.empty(0, dtype=torch.float64)
    dev = ts[0].device
    out = torch.empty(len(ts), dtype=torch.float64, device=dev)
    groups = {}
    for i, t in enumerate(ts):
        b = t._base if t._base is not None else t
        g = groups.get(id(b))
        if g is None:
            g = groups[id(b)] = (b, [], [])
        g[1].append(i)
        g[2].append(t.storage_offset() - b.storage_offset() + (t.shape[0] - 1) * t.stride(0))
    for b, idx, offs in groups.values():
        flat = b.reshape(-1) if b.is_contiguous() else b.contiguous().reshape(-1)
        out[torch.as_tensor(idx, device=dev)] = flat[torch.as_tensor(offs, device=dev)]
    return out


class FitWorker:
    """One host process's part of a step on one GPU: its slice of the step's series (fits
    f0 .. f0 + F_w − 1 of the rank's F), its slots (width / procs) in `groups` device batches,
    fitted by one host thread through minimize_stream."""

    def __init__(self, args, w, P, rank, gpu, admission=None):
        import torch
        import portfoliooptgp_amd as gpx
        from portfoliooptgp_amd.engine import Engine
        from portfoliooptgp_amd.kernels import compile_spec
        self.torch, self.gpx = torch, gpx
        self.args, self.w, self.gpu = args, w, gpu
        self.admission = admission
        n = self.n = args.n
        dev = torch.device(f"cuda:{gpu}")
        self.fit_ids = None
        if args.scaling == "strong":
            # this process's share of the fixed batch (strong_plan: the same plan on every process);
            # global fit i fits series i mod total_series (seed = that series index)
            world = int(os.environ.get("WORLD_SIZE", "1"))
            self.fit_ids = strong_fit_ids(args, world, P)[rank][w]
            seeds = sorted({i % args.total_series for i in self.fit_ids})
            self.F, self.S = len(self.fit_ids), len(seeds)
            pos = {sd: k for k, sd in enumerate(seeds)}
            self.series_of = [pos[i % args.total_series] for i in self.fit_ids]
            data = [synthetic_series(n, sd) for sd in seeds]
        else:
            F = args.fits
            self.F = share(F, P, w)
            # distinct series of this process (fits cycle over them: fit f of a step is series
            # f mod S_w), seeds rank·S + s0 + s
            S = max(1, min(args.series, F))
            self.S = share(S, P, w)
            s0 = sum(share(S, P, i) for i in range(w))
            self.series_of = [f % self.S for f in range(self.F)]
            data = [synthetic_series(n, rank * S + s0 + s) for s in range(self.S)]
        self.Xd = [torch.as_tensor(x, device=dev) for x, _ in data]  # resident in HBM before timing
        self.Yd = [torch.as_tensor(y, device=dev) for _, y in data]
        # read-only series: their band-table boxes are computed at the first rebind and reused
        # (GPX_BOX_CACHE=0 turns that off: every rebind then downloads its boxes)
        from portfoliooptgp_amd.engine import mark_immutable
        mark_immutable(*self.Xd)
        W = share(args.width, P, w)
        G = max(1, min(args.groups, W))
        self.wide = args.wide_slots > 0
        if self.wide:  # [narrow batch(es) | the slow-class batch]
            Wn = W - args.wide_slots
            sizes = [share(Wn, G, g) for g in range(G)] + [args.wide_slots]
        else:
            sizes = [share(W, G, g) for g in range(G)]
        spec = compile_spec(gpx.kernels.SquaredExponential(), 1)
        # slot shapes only: every slot is rebound to its fit's series when the fit starts
        self.engines = [Engine([self.Xd[i % self.S] for i in range(sz)], [self.Yd[i % self.S] for i in range(sz)],
                               [spec] * sz, device=gpu, band_storage=args.storage == "band")
                        for sz in sizes]
        self.engines[0].ctx.set_profiling(True)
        # deferred completion of the slow width classes (Engine.set_deferred): a call completes
        # when its band16 problems of at most --defer-q 16-blocks are done; the wider ones (and
        # the 64-row sweeps) come back with a later call
        if args.defer_q >= 0:
            for e in self.engines:
                e.set_deferred(args.defer_q)
        # GPX_WAVE_TRACE=1: every band16 wavefront's residency (start, end) in the device clock,
        # merged over the GPU's host processes into an occupancy timeline (wave_trace_summary)
        self.wtrace = bool(int(os.environ.get("GPX_WAVE_TRACE", "0")))
        if self.wtrace:
            for e in self.engines:
                e.wave_trace(int(os.environ.get("GPX_WAVE_TRACE_CAP", 1 << 21)))
        self.opt = gpx.optimizers.Scipy()
        self.width, self.groups = W, G
        self.traces, self.driver_stats = [], []

    def make_model(self, f):
        # GPflow defaults (σ²=1, ℓ=1), σn² = 1e-5 frozen — GPR/model_trainer.py:15-17
        gpx = self.gpx
        sr = self.series_of[f]
        m = gpx.models.GPR(data=(self.Xd[sr], self.Yd[sr]), kernel=gpx.kernels.SquaredExponential(),
                           device=self.gpu)
        m.likelihood.variance.assign(NOISE)
        gpx.set_trainable(m.likelihood.variance, False)
        return m

    def run_steps(self, k):
        """k steps (k × F_w fits, each from GPflow defaults) streamed back to back through the
        slots; returns (nfev list, summary rows [k·F_w, 6] on the host: ℓ*, σ²*, loss*, nfev,
        mean and var of the last training-point prediction)."""
        torch, F = self.torch, self.F
        # every fit's model is built inside the timed region, on demand (as the reference's loop
        # builds each GPR right before fitting it), while the host thread waits for the device
        models = self.gpx.optimizers.ModelStream(k * F, lambda i: self.make_model(i % F), input_dim=1,
                                                 max_points=self.n, device=self.gpu)
        res, preds = self.opt.minimize_stream(models, width=self.width, engine=self.engines, predict_train=True,
                                              groups=len(self.engines), options=dict(maxiter=MAXITER),
                                              admission=self.admission, wide_group=self.wide)
        if getattr(self.opt, "last_trace", None):
            self.traces.append(self.opt.last_trace)
        if getattr(self.opt, "last_stats", None):
            self.driver_stats.append(dict(self.opt.last_stats))
        host = np.array([[m.kernel.lengthscales.value, m.kernel.variance.value, float(r.fun), float(r.nfev)]
                         for m, r in zip(models, res)], dtype=np.float64)
        mu = last_points([p[0] for p in preds]).cpu().numpy()
        var = last_points([p[1] for p in preds]).cpu().numpy()
        table = np.concatenate([host, mu[:, None], var[:, None]], axis=1)
        if self.fit_ids is not None:  # strong scaling: each row keyed by its global fit index
            ids = np.asarray(self.fit_ids, dtype=np.float64)
            gidx = np.concatenate([ids + st * self.args.total_fits for st in range(k)])
            table = np.concatenate([gidx[:, None], table], axis=1)
        return [r.nfev for r in res], table

    def reset_timing(self):
        for e in self.engines:
            e.reset_timing()
            if self.wtrace:
                e.wave_trace_read()  # (discarded: restarts the recording)
        self.driver_stats = []

    def wave_records(self):
        if not self.wtrace:
            return None
        return np.concatenate([e.wave_trace_read() for e in self.engines])

    def timing(self):
        tms = [e.last_timing() for e in self.engines]
        out = {f: float(sum(getattr(t, f) for t in tms)) for f in SUM_FIELDS}
        out.update({f: float(sum(getattr(t, f) for t in tms)) for f in NARROW_FIELDS})
        return out


def helper_main(w, P, argv, rank, gpu, start, q, admission=None):
    """A helper host process (spawned before the rank touched the GPU): warm up, report ready,
    wait for the rank's start signal, fit its slice of the K steps, synchronise, hand back its
    results (the message means its device work is done)."""
    os.environ["GPX_DEVICE"] = str(gpu)
    args = parse_args(argv)
    import torch
    torch.cuda.set_device(gpu)
    wk = FitWorker(args, w, P, rank, gpu, admission)
    if args.warmup > 0:
        wk.run_steps(args.warmup)
    wk.reset_timing()
    torch.cuda.synchronize()
    q.put(("ready", w))
    start.wait()
    t0 = time.perf_counter()
    nfev, summary = wk.run_steps(args.steps)
    torch.cuda.synchronize()
    busy = time.perf_counter() - t0
    q.put(("done", (w, nfev, summary, wk.timing(), wk.driver_stats[-1] if wk.driver_stats else None, busy,
                    wk.wave_records())))
    if os.environ.get("GPX_SUBMIT_STATS"):
        wk.engines.clear()  # destroyed now: the library prints the per-batch submit phases


def collect(q, helpers, kind, timeout):
    """The helpers' `kind` messages; raises if a helper dies or the wait exceeds `timeout`."""
    import queue as _q
    got, t_end = [], time.monotonic() + timeout
    while len(got) < len(helpers):
        try:
            k, v = q.get(timeout=1.0)
        except _q.Empty:
            # a helper that exits cleanly has flushed its message into the queue first
            failed = [h for h in helpers if not h.is_alive() and h.exitcode != 0]
            if failed:
                raise RuntimeError(f"bench helper process failed (exit code {failed[0].exitcode}) before '{kind}'")
            if time.monotonic() > t_end:
                raise TimeoutError(f"bench helpers: no '{kind}' after {timeout} s")
            continue
        assert k == kind, (k, kind)
        got.append(v)
    return got


def wave_trace_summary(recs, wall_s, clock_hz=1e8):
    """Occupancy timeline of the band16 sweeps from every host process's wavefront records
    (start, end, kind; the device's constant 100 MHz clock, shared by all processes): the mean
    number of resident sweep wavefronts over the span from the first start to the last end, the
    share of that span spent at each residency level, and the mean wave durations."""
    r = np.concatenate([x for x in recs if x is not None and len(x)])
    r = r[r[:, 2] < 32]  # (kinds >= 32: the library's stream-order markers, tools/call_timeline.py)
    if len(r) == 0:
        return {"records": 0}
    t0, t1, kind = r[:, 0].astype(np.int64), r[:, 1].astype(np.int64), r[:, 2].astype(np.int64)
    base = int(t0.min())
    a, b = t0 - base, t1 - base
    span = int(b.max())
    ev_t = np.concatenate([a, b])
    ev_d = np.concatenate([np.ones_like(a), -np.ones_like(b)])
    o = np.lexsort((ev_d, ev_t))  # ends before starts at equal times
    ev_t, ev_d = ev_t[o], ev_d[o]
    level = np.cumsum(ev_d)
    dt = np.diff(ev_t, append=ev_t[-1])
    edges = [0, 256, 512, 1024, 1536, 2048, 1 << 30]
    share = {f"{edges[i]}-{edges[i + 1] - 1 if edges[i + 1] < (1 << 30) else 'up'}":
             float(dt[(level >= edges[i]) & (level < edges[i + 1])].sum() / max(span, 1)) for i in range(len(edges) - 1)}
    fwd, bwd = kind < 16, kind >= 16
    dur = (b - a) / clock_hz * 1e3
    return {"records": int(len(r)), "span_s": span / clock_hz, "wall_s": wall_s,
            "mean_resident_waves": float(((b - a).sum()) / max(span, 1)),
            "occupancy_2048": float(((b - a).sum()) / max(span, 1) / WAVE_SLOTS),
            "share_of_span_by_resident_waves": share,
            "fwd_wave_ms_mean": float(dur[fwd].mean()) if fwd.any() else None,
            "bwd_wave_ms_mean": float(dur[bwd].mean()) if bwd.any() else None,
            "q_hist": {int(q): int((kind % 16 == q).sum() // 2) for q in np.unique(kind % 16)},
            # per width class: waves, mean forward / backward wave ms, share of all wave time
            "q_wave": {int(q): [int((kind == q).sum()), float(dur[kind == q].mean()) if (kind == q).any() else None,
                                float(dur[kind == 16 + q].mean()) if (kind == 16 + q).any() else None,
                                float(dur[kind % 16 == q].sum() / max(dur.sum(), 1e-30))]
                       for q in np.unique(kind % 16)},
            "note": "band16 wavefronts only (s_memrealtime at each wave's start and end); span = first "
                    "start to last end over all host processes of this GPU"}


def c4_kernel(gpx, kind):
    """C4's kernels: BASELINE.json configs[3]'s Matern52 on all five inputs, or the reference's
    own Multi-Input kernel, Exponential(dims 0..3) × Exponential(dim 4)
    (Multi-Input_GPR/main.py:118-135 create_composite_kernel, D = 5)."""
    K = gpx.kernels
    if kind == "m52":
        return K.Matern52()
    return K.Exponential(active_dims=slice(0, 4)) * K.Exponential(active_dims=slice(4, 5))


def secondary_c4(gpu, fits=32, kind="m52", groups=1):
    """Config C4 (BASELINE.json configs[3]) on the dense path: D = 5 (4 z-scored random-walk
    features + z-scored time), Matern52 (or `kind` "expxexp": the reference's Exponential ×
    Exponential product), N = 4096, fp64 (the reference's precision), σn² = 1e-3 fixed, scipy
    defaults + maxiter 100, predict_f at the training inputs; `fits` series in `groups` device
    batches (one: the 32-problem calls keep the GEMMs' tiles fuller than two concurrent batches of
    16 — 36.1 vs 33.7 fits/s on one box, 4 batches 30.8, tools/c4_layouts.py). Also the fused
    K⁻¹ + gradient contraction's rate over those launches."""
    import torch
    import portfoliooptgp_amd as gpx
    n = 4096
    data = []
    for s in range(fits):
        rng = np.random.default_rng(100 + s)
        X = np.hstack([np.cumsum(rng.standard_normal((n, 4)), axis=0), np.linspace(0.0, 1.0, n)[:, None]])
        X = (X - X.mean(0)) / X.std(0, ddof=1)
        data.append((torch.as_tensor(X, device=f"cuda:{gpu}"),
                     torch.as_tensor(synthetic_series(n, s)[1], device=f"cuda:{gpu}")))

    def models(k):
        out = []
        for x, y in data[:k]:
            m = gpx.models.GPR((x, y), kernel=c4_kernel(gpx, kind), device=gpu)
            m.likelihood.variance.assign(1e-3)
            gpx.set_trainable(m.likelihood.variance, False)
            out.append(m)
        return out
    from portfoliooptgp_amd.engine import Engine
    from portfoliooptgp_amd.kernels import compile_spec
    spec = compile_spec(c4_kernel(gpx, kind), 5)
    engines = [Engine([d[0] for d in data[g::groups]], [d[1] for d in data[g::groups]], [spec] * len(data[g::groups]),
                      device=gpu) for g in range(groups)]
    engines[0].ctx.set_profiling(True)
    opt = gpx.optimizers.Scipy()
    eng_arg = engines if groups > 1 else engines[0]
    opt.minimize_stream(models(groups), width=groups, engine=eng_arg, groups=groups, predict_train=True,
                        options=dict(maxiter=MAXITER))  # warm-up
    for e in engines:
        e.reset_timing()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    res, _ = opt.minimize_stream(models(fits), width=fits, engine=eng_arg, groups=groups, predict_train=True,
                                 options=dict(maxiter=MAXITER))
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    tms = [e.last_timing() for e in engines]
    c_ms = sum(t.contract_ms_total for t in tms)
    c_l = sum(t.contract_launches for t in tms)
    c_f = sum(t.contract_alg_flops for t in tms)
    evals = sum(t.evals for t in tms)
    ach = c_f / (c_ms * 1e-3) / 1e12 if c_ms > 0 else 0.0
    P = 2 if kind == "m52" else 4
    kname = "Matern52" if kind == "m52" else "Exponential(dims 0-3) x Exponential(dim 4)"
    epi = "EPI_CONTRACT1" if kind == "m52" else "EPI_CONTRACT2"
    return {"config": "C4", "workload": f"Multi-Input shape: D=5, {kname}, N=4096, fp64, sigma_n^2=1e-3 fixed, "
            f"{fits} fits, L-BFGS-B maxiter=100 + predict_f(X_train), dense path, {groups} device batch(es)",
            "fits_per_s": fits / dt, "fits": fits, "seconds": dt, "nfev_mean": float(np.mean([r.nfev for r in res])),
            "nfev_max": int(max(r.nfev for r in res)),
            "evals_per_s": evals / dt, "dense_evals": evals - sum(t.band_evals for t in tms),
            "eval_alg_tflops": evals * (n ** 3 + 2 * (P + 1) * n ** 2) / dt / 1e12,
            "contraction_roofline": {
                "kernel": f"gemm_kernel<128,T,N,{epi}> (K^-1 = W^T W fused with the gradient contraction)",
                "bound": "mfma", "achieved": ach, "peak": FP64_PEAK_TFLOPS, "unit": "TFLOP/s",
                "frac": ach / FP64_PEAK_TFLOPS, "avg_launch_ms": c_ms / max(c_l, 1.0), "launches": c_l,
                "alg_flops_per_launch": c_f / max(c_l, 1.0)}}


def secondary_c3(gpu, n=2048, series=20, share=3, reps=3):
    """Config C3 (BASELINE.json configs[2]): the per-asset batch, `series` synthetic series x
    N = 2048 (SE, GPflow defaults, σn² = 1e-5 fixed, maxiter 100, predict_f at the training
    inputs), fitted on one GPU; and `share` = ceil(20 / 8) series, the largest per-GPU share when
    the 20 are sharded over 8 GPUs (distributed.shard_lpt; the all_gather after it is a few
    KB). wall(20) / wall(3) bounds the 8-GPU strong-scaling speed-up of this batch: each GPU's
    fits run concurrently, so the batch takes about as long as its slowest fit's chain of
    evaluations either way. Median of `reps` runs each."""
    import torch
    import portfoliooptgp_amd as gpx
    from portfoliooptgp_amd.engine import Engine
    from portfoliooptgp_amd.kernels import compile_spec
    dev = f"cuda:{gpu}"
    data = [synthetic_series(n, s) for s in range(series)]
    data = [(torch.as_tensor(x, device=dev), torch.as_tensor(y, device=dev)) for x, y in data]
    spec = compile_spec(gpx.kernels.SquaredExponential(), 1)

    def model(i):
        m = gpx.models.GPR(data=data[i], kernel=gpx.kernels.SquaredExponential(), device=gpu)
        m.likelihood.variance.assign(NOISE)
        gpx.set_trainable(m.likelihood.variance, False)
        return m

    def run(k, route="bcr"):
        eng = Engine([d[0] for d in data[:k]], [d[1] for d in data[:k]], [spec] * k, device=gpu, band_storage=True,
                     band_route=route)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        res, _ = gpx.optimizers.Scipy().minimize_stream([model(i) for i in range(k)], width=k, engine=eng,
                                                        predict_train=True, options=dict(maxiter=MAXITER))
        torch.cuda.synchronize()
        return time.perf_counter() - t0, res

    run(share)  # warm-up
    w_all = sorted(run(series)[0] for _ in range(reps))[reps // 2]
    run(share, "sweeps")
    w_all_sweeps = sorted(run(series, "sweeps")[0] for _ in range(reps))[reps // 2]
    t_share, res_share = [], None
    for _ in range(reps):
        t, res_share = run(share)
        t_share.append(t)
    w_share = sorted(t_share)[reps // 2]
    return {"config": "C3", "workload": f"{series} synthetic series x N={n}, SE, fp64, sigma_n^2=1e-5 fixed, "
            "L-BFGS-B maxiter=100 + predict_f(X_train), band-storage slots, one GPU",
            "wall_s_all_series_1gpu": w_all, "fits_per_s_1gpu": series / w_all,
            "wall_s_per_gpu_share_at_8gpus": w_share, "share_series": share,
            "nfev_of_share": [int(r.nfev) for r in res_share],
            "ratio_wall_all_over_share": w_all / w_share,
            "band_route": "bcr",
            "wall_s_all_series_1gpu_sweeps_route": w_all_sweeps,
            "note": "the engine takes the latency route, block cyclic reduction (Engine(band_route='bcr'), "
                    "DESIGN.md §3f; the default route, the one-wavefront sweeps, is timed beside it); "
                    "wall(20) / wall(share) is an upper bound on the 8-GPU speed-up of this batch (the ranks' "
                    "shares run concurrently): each fit is a chain of ~20 dependent evaluations"}


def secondary_solo(gpu, n=N_POINTS, seeds=(0, 1, 2), reps=3):
    """The reference's own call pattern: ONE exact GPR fit at a time, as GPR/model_trainer.py:15-20
    runs it inside its kernel loop — models.GPR from GPflow's defaults, Scipy().minimize
    (maxiter=100), predict_f at the training inputs — on the C2 series (N = 4096, SE, sigma_n^2 =
    1e-5 fixed), on each banded route: the latency route (block cyclic reduction, DESIGN.md §3f;
    gpx.set_default_band_route("bcr")) and the default, the one-wavefront band16 sweeps. Median wall
    time of `reps` fits per seed (after a warm-up fit), and the device time of one evaluation's
    reduction chain (HIP events, profiling on, a separate pass)."""
    import torch
    import portfoliooptgp_amd as gpx
    from portfoliooptgp_amd import _native as N
    from portfoliooptgp_amd.engine import solo_engine

    def fit(x, y):
        m = gpx.models.GPR(data=(x, y), kernel=gpx.kernels.SquaredExponential(), device=gpu)
        m.likelihood.variance.assign(NOISE)
        gpx.set_trainable(m.likelihood.variance, False)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        r = gpx.optimizers.Scipy().minimize(m.training_loss, m.trainable_variables, options=dict(maxiter=MAXITER))
        m.predict_f(x)
        torch.cuda.synchronize()
        return time.perf_counter() - t0, int(r.nfev), float(r.fun), m

    out = {"config": "C2, one fit at a time", "workload": f"synthetic 1-D series, N={n}, SE, fp64, sigma_n^2=1e-5 "
           "fixed, models.GPR + Scipy().minimize(maxiter=100) + predict_f(X_train), one GPR per call (the "
           "reference's GPR/model_trainer.py:15-20 loop)", "seeds": list(seeds),
           "note": "band16_sweeps = the default route (the headline's; a fit's bits equal its bits in any batch); "
                   "bcr = gpx.set_default_band_route('bcr'), the latency route (DESIGN.md §3f)"}
    prev = os.environ.pop("GPX_BCR_MAX", None)
    prev_route = gpx.set_default_band_route("sweeps")
    try:
        for mode, route in (("bcr", "bcr"), ("band16_sweeps", "sweeps")):
            gpx.set_default_band_route(route)
            walls, nfevs, funs = [], [], []
            for s in seeds:
                x, y = synthetic_series(n, s)
                fit(x, y)  # warm-up: engine creation, first gather
                w = []
                for _ in range(reps):
                    t, nf, fun, _m = fit(x, y)
                    w.append(t)
                walls.append(sorted(w)[reps // 2])
                nfevs.append(nf)
                funs.append(fun)
            out[mode] = {"fit_ms_per_seed": [1e3 * v for v in walls], "fit_ms_median": 1e3 * sorted(walls)[len(walls) // 2],
                         "nfev": nfevs, "loss": funs}
        # one evaluation's device chain on the reduction path (profiling on: HIP events around it)
        gpx.set_default_band_route("bcr")
        x, y = synthetic_series(n, seeds[0])
        _, _, _, m = fit(x, y)
        ctx = N.Context.get(gpu)
        ctx.set_profiling(True)
        eng = solo_engine(m)
        m.loss_and_grad_unconstrained()
        eng.reset_timing()
        for _ in range(20):
            m.loss_and_grad_unconstrained()
        t = eng.last_timing()
        ctx.set_profiling(False)
        out["bcr_chain_ms_per_eval"] = t.bcr_ms_total / max(t.bcr_calls, 1.0)
        out["device_ms_per_eval"] = t.eval_ms_total / max(t.evals, 1.0)
    finally:
        gpx.set_default_band_route(prev_route)
        if prev is not None:
            os.environ["GPX_BCR_MAX"] = prev
    out["speedup_vs_band16_sweeps"] = out["band16_sweeps"]["fit_ms_median"] / out["bcr"]["fit_ms_median"]
    return out


def _c1_series():
    """The reference's own C1 data (BASELINE configs[0]): AAPL daily / weekly / monthly returns as
    GPR/data_handler.py:26-65 prepares them (N = 89 / 19 / 5, unnormalised day offsets), from the
    committed fixture tests/golden/kernel_cases.npz (generated from the reference's CSVs by
    tests/golden/make_golden.py)."""
    d = np.load(os.path.join(REPO, "tests", "golden", "kernel_cases.npz"))
    return [(tf, d[f"data|aapl_{tf}|x"], d[f"data|aapl_{tf}|y"]) for tf in ("d", "w", "m")]


def c1_cpu_baseline(reps=5):
    """The CPU leg of secondary_c1_solo (the oracle, never part of the GPU figures): the same
    sweep with oracle/gp_oracle.py's restatement of GPflow (numpy/scipy, fp64, one host thread of
    BLAS), and its per-evaluation time at each N."""
    import threadpoolctl
    from oracle import gp_oracle as O
    out = {"kind": "port", "cores": 1, "eval_us": {}}
    with threadpoolctl.threadpool_limits(limits=1, user_api="blas"):
        for tf, x, y in _c1_series():
            m = O.OGPR(x, y, O.OSquaredExponential(), noise_variance=1e-5)
            m.noise.trainable = False
            m.loss_and_grad_u()
            ts = []
            for _ in range(reps):
                t0 = time.perf_counter()
                for _ in range(50):
                    m.loss_and_grad_u()
                ts.append((time.perf_counter() - t0) / 50)
            out["eval_us"][str(len(x))] = sorted(ts)[reps // 2] * 1e6
        walls, nfev = [], 0
        for _ in range(3):
            ks = O.reference_kernel_list()  # (shared across d -> w -> m, as GPR/main.py:105-114)
            t0 = time.perf_counter()
            nfev = 0
            for tf, x, y in _c1_series():
                for k in ks:
                    m = O.OGPR(x, y, k, noise_variance=1e-5)
                    m.noise.trainable = False
                    try:
                        r = O.scipy_minimize(m, 100)
                        nfev += r.nfev
                        m.predict_f(x)
                    except np.linalg.LinAlgError:
                        pass
            walls.append(time.perf_counter() - t0)
        out["sweep_ms"] = 1e3 * sorted(walls)[1]
        out["sweep_nfev"] = nfev
    out["sample"] = ("oracle/gp_oracle.py on one host thread: the AAPL d/w/m 8-kernel sweep (median of 3) and 50 "
                     "SE evaluations per N (median of 5 x 50)")
    return out


def secondary_c1_solo(gpu, reps=5):
    """The drop-in pattern at the reference's real sizes: GPR/main.py's AAPL
    d -> w -> m sweep with the 8 shared kernel objects of GPR/main.py:105-114, each fit exactly as
    GPR/model_trainer.py:14-20 runs it — ONE GPR at a time (models.GPR, noise 1e-5 frozen,
    Scipy().minimize(maxiter=100), predict_f at the training inputs, the training MSE) — through the
    INTEGRATION.md §1 import swap. Reports the sweep's wall time, ms per evaluation inside the fits
    (scipy's own loop included), and µs per bare loss+gradient evaluation at N = 89 / 19 / 5, next
    to the CPU oracle's (c1_cpu_baseline)."""
    import torch
    import portfoliooptgp_amd as gpx
    K = gpx.kernels
    series = _c1_series()

    def kernels():
        return [K.SquaredExponential(), K.Matern12(), K.RationalQuadratic(), K.Exponential(),
                K.SquaredExponential() + K.Matern12(),
                K.Exponential() + K.Periodic(K.SquaredExponential()) + K.Linear(),
                K.Exponential() + K.Periodic(K.SquaredExponential()),
                K.SquaredExponential() * K.Matern12()]

    def sweep():
        ks = kernels()
        nfev, raised, best = 0, 0, {}
        for tf, x, y in series:
            best_mse = None
            for k in ks:
                m = gpx.models.GPR(data=(x, y), kernel=k, device=gpu)
                m.likelihood.variance.assign(1e-5)
                gpx.set_trainable(m.likelihood.variance, False)
                try:
                    r = gpx.optimizers.Scipy().minimize(m.training_loss, m.trainable_variables,
                                                        options=dict(maxiter=MAXITER))
                except (gpx.NotPositiveDefiniteError, gpx.InvalidParameterError):
                    raised += 1
                    continue
                nfev += int(r.nfev)
                mean, _ = m.predict_f(x)
                mse = float(np.mean((y.reshape(-1) - mean.numpy().reshape(-1)) ** 2))
                best_mse = mse if best_mse is None else min(best_mse, mse)
            best[tf] = best_mse
        return nfev, raised, best

    sweep()  # warm-up (engines for the three padded sizes, code objects)
    walls = []
    for _ in range(reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        nfev, raised, best = sweep()
        torch.cuda.synchronize()
        walls.append(time.perf_counter() - t0)
    wall = sorted(walls)[reps // 2]
    ev = {}
    for tf, x, y in series:
        m = gpx.models.GPR(data=(x, y), kernel=K.SquaredExponential(), device=gpu)
        m.likelihood.variance.assign(1e-5)
        gpx.set_trainable(m.likelihood.variance, False)
        m.loss_and_grad_unconstrained()
        ts = []
        for _ in range(reps):
            t0 = time.perf_counter()
            for _ in range(200):
                m.loss_and_grad_unconstrained()
            ts.append((time.perf_counter() - t0) / 200)
        ev[str(len(x))] = sorted(ts)[reps // 2] * 1e6
    out = {"config": "C1 (BASELINE configs[0]): the reference's plumbing at its real sizes",
           "workload": "AAPL d/w/m (N = 89 / 19 / 5), the 8 kernels of GPR/main.py:105-114 shared across timeframes, "
                       "one GPR at a time as GPR/model_trainer.py:14-20 (Scipy maxiter 100 + predict_f + MSE)",
           "sweep_ms": wall * 1e3, "sweep_fits": 24 - raised, "sweep_raised": raised, "sweep_nfev": nfev,
           "ms_per_fit_evaluation": wall * 1e3 / max(nfev, 1),
           "eval_us_gpu": ev, "best_train_mse": best,
           "note": "eval_us_gpu: one bare loss+gradient (m.loss_and_grad_unconstrained, SE) per call, median of "
                   f"{reps} x 200; ms_per_fit_evaluation: the sweep's wall / its evaluations (scipy's loop, "
                   "model construction and predict_f included). N <= 64 takes the one-launch small-problem "
                   "kernel (DESIGN.md §3h)"}
    try:
        out["cpu_baseline"] = c1_cpu_baseline()
        cb = out["cpu_baseline"]
        out["gpu_over_cpu_eval_time"] = {n: ev[n] / cb["eval_us"][n] for n in ev if n in cb["eval_us"]}
        out["sweep_speedup_vs_cpu"] = cb["sweep_ms"] / out["sweep_ms"]
    except Exception as e:  # reported, never fatal
        out["cpu_baseline"] = {"error": f"{type(e).__name__}: {e}"}
    return out


def secondary_c5(gpu, reps=20):
    """Config C5 (BASELINE.json configs[4]): SVGP ELBO + gradients at N = 65536, M = 1024, D = 1,
    SE, whitened full q_sqrt, fp64; ms per evaluation (one GPU)."""
    import torch
    import portfoliooptgp_amd as gpx
    from portfoliooptgp_amd.engine import SVGPEngine
    from portfoliooptgp_amd.kernels import compile_spec
    n, M = 65536, 1024
    rng = np.random.default_rng(0)
    X = np.sort(rng.uniform(0, 360, (n, 1)), axis=0)
    Y = np.sin(X / 20.0) + 0.1 * rng.standard_normal((n, 1))
    Z = np.linspace(0, 360, M)[:, None]
    eng = SVGPEngine(X, Y, compile_spec(gpx.kernels.SquaredExponential(), 1), M, num_data=n, device=gpu)
    theta = np.ones(16)
    theta[:3] = [2.0, 1.0, 1e-4]
    q = rng.standard_normal(M) * 0.3
    R = np.tril(rng.standard_normal((M, M)) * 1e-3)
    R[np.diag_indices(M)] = rng.uniform(0.05, 0.2, M)
    eng.elbo_grad(theta, Z, q, R)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        eng.elbo_grad(theta, Z, q, R)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / reps
    Mp = (M + 63) // 64 * 64
    flops = 3.0 * Mp * Mp * n + 14.0 * Mp ** 3   # SYRK G (M²N) + Y = 2c·P·Kmn (2M²N) + the O(M³) tail
    return {"config": "C5", "workload": f"SVGP N={n}, M={M}, SE, whitened full q_sqrt, fp64: one ELBO+gradient "
            f"evaluation (mean of {reps})", "ms_per_eval": dt * 1e3, "alg_tflops": flops / dt / 1e12,
            "frac_fp64_peak": flops / dt / 1e12 / FP64_PEAK_TFLOPS}


def main():
    # HIP hardware queues for this process (and the helpers, which inherit the environment), set
    # before the runtime starts: over all the GPU's processes the queues stay within what the
    # queue scheduler maps at once (8 processes x 2)
    os.environ["GPU_MAX_HW_QUEUES"] = os.environ.get("GPX_HW_QUEUES", "2")
    # driver phase times (host share of the timed region), cheap perf_counter reads
    os.environ.setdefault("GPX_DRIVER_STATS", "1")
    argv = sys.argv[1:]
    args = parse_args(argv)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    os.environ.setdefault("GPX_DEVICE", str(local_rank))
    gpu = int(os.environ["GPX_DEVICE"])
    P = max(1, args.procs)

    # helper processes first, before anything here touches the GPU (a process that has
    # initialised HIP must not fork/exec)
    helpers, start, q, admission = [], None, None, None
    if P > 1:
        import multiprocessing as mp
        ctx = mp.get_context("spawn")
        start = ctx.Event()
        q = ctx.Queue()
        # (optimizers.DeviceAdmission's semaphore, made here without importing the package: nothing
        # may touch the GPU before the helpers are spawned)
        admission = ctx.BoundedSemaphore(args.admission) if args.admission > 0 else None
        helpers = [ctx.Process(target=helper_main, args=(w, P, argv, rank, gpu, start, q, admission), daemon=True)
                   for w in range(1, P)]
        for h in helpers:
            h.start()

    import torch
    import torch.distributed as dist

    # GPX_BENCH_BACKEND=gloo + GPX_DEVICE=0: rehearsal of the multi-rank path with every rank
    # on one GPU (collectives on host tensors); the real run is RCCL, one GPU per rank
    backend = os.environ.get("GPX_BENCH_BACKEND", "nccl")
    torch.cuda.set_device(gpu)
    dev = torch.device(f"cuda:{gpu}")
    cdev = dev if backend == "nccl" else torch.device("cpu")
    if world > 1:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)

    wk = FitWorker(args, 0, P, rank, gpu, admission)
    if args.warmup > 0:
        wk.run_steps(args.warmup)
    wk.reset_timing()
    torch.cuda.synchronize()
    collect(q, helpers, "ready", 1800)  # every host process of this GPU has warmed up
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    # trace markers (a ~1 us spin kernel) delimit the timed region in a rocprofv3 kernel trace,
    # so tools/trace_check.py can average the same launches the bench timed
    torch.cuda._sleep(1000)
    if start is not None:
        start.set()                     # the helpers start their steps
    nfev, summary = wk.run_steps(args.steps)
    torch.cuda._sleep(1000)
    torch.cuda.synchronize()
    busy0 = time.perf_counter() - t0
    parts = [(0, nfev, summary, wk.timing(), wk.driver_stats[-1] if wk.driver_stats else None, busy0,
              wk.wave_records())]
    parts += collect(q, helpers, "done", 1800)  # each sent after synchronising its device work
    parts.sort(key=lambda p: p[0])
    table = np.concatenate([p[2] for p in parts])
    if args.scaling == "strong":
        # the fixed batch's hand-off: one all_gather of every rank's rows (device tensors over
        # RCCL, distributed.all_gather_results), the table sorted by global fit index
        from portfoliooptgp_amd import distributed as D
        table = D.gather_table(table)
    elif world > 1:  # the per-asset hand-off: one all_gather of every fit's summary row
        t = torch.as_tensor(table, device=cdev)
        gathered = [torch.empty_like(t) for _ in range(world)]
        dist.all_gather(gathered, t)
        table = torch.cat(gathered).cpu().numpy()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    for h in helpers:
        h.join(timeout=120)
    if os.environ.get("GPX_SUBMIT_STATS"):
        wk.engines.clear()  # destroyed now: the library prints the per-batch submit phases

    tm = {f: sum(p[3][f] for p in parts) for f in SUM_FIELDS + NARROW_FIELDS}
    nfev_all = [n for p in parts for n in p[1]]
    if world > 1:
        t = torch.tensor([elapsed], device=cdev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        nf = torch.tensor([float(sum(nfev_all)), float(len(nfev_all)), tm["evals"]], device=cdev,
                          dtype=torch.float64)
        dist.all_reduce(nf)
        nfev_mean = float(nf[0] / nf[1])
        evals_all = float(nf[2])  # device evaluations over all ranks
    else:
        nfev_mean = float(np.mean(nfev_all))
        evals_all = tm["evals"]
    if args.scaling == "strong":
        total_fits = args.total_fits * args.steps
        assert table.shape[0] == total_fits and np.array_equal(table[:, 0], np.arange(total_fits)), table.shape
    else:
        total_fits = args.fits * args.steps * world
    assert table.shape[0] == total_fits, (table.shape, total_fits)
    value = total_fits / elapsed
    n = args.n

    # roofline: the banded sweep kernel with the most device time, when the fits' evaluations take
    # the banded path (C2: every evaluation); the dense contraction otherwise.
    #   band16 (16-row blocks, one wavefront per problem; most C2 evaluations): achieved = the
    #     MFMA flops its problems issue (2*16^3 per tile product; gpx_api.hip band16_flops) / the
    #     launch's HIP-event duration
    #   64-row fused sweeps (the wider bands): the 64^3 block products (leaf 2/3 of one)
    sweeps = {}
    # the 64-row pairs' kernels by the name rocprof records: band_fwd1_kernel / band_bwd1_kernel<1> (the
    # p <= 1 class) or band_fwd_kernel / band_bwd_kernel<1> (the p = 2 class, two 64-blocks per step)
    p2 = tm["band_fused_p2_launches"]
    f64n, b64n = (("band_fwd_kernel", "band_bwd_kernel<1>") if p2 >= tm["band_fused_launches"] > 0 else
                  ("band_fwd1_kernel", "band_bwd1_kernel<1>") if p2 == 0 else
                  ("band_fwd1_kernel+band_fwd_kernel", "band_bwd1_kernel<1>+band_bwd_kernel<1>"))
    for key, ms, fl, la in (("band16_fwd_kernel", tm["band16_fwd_ms_total"], tm["band16_fwd_flops"], tm["band16_launches"]),
                            ("band16_bwd_kernel", tm["band16_bwd_ms_total"], tm["band16_bwd_flops"], tm["band16_launches"]),
                            (f64n, tm["band_fwd_ms_total"], tm["band_fwd_flops"], tm["band_fused_launches"]),
                            (b64n, tm["band_bwd_ms_total"], tm["band_bwd_flops"], tm["band_fused_launches"]),
                            # the deferred part's Q = 4/5 classes, both sweeps per wavefront, one launch
                            ("band16_wide_kernel", tm["band16_wide_ms_total"], tm["band16_wide_flops"],
                             tm["band16_wide_launches"])):
        b_ms = ms / max(la, 1.0)
        b_fl = fl / max(la, 1.0)
        ach = b_fl / (b_ms * 1e-3) / 1e12 if b_ms > 0 else 0.0
        sweeps[key] = {"achieved": ach, "frac": ach / FP64_PEAK_TFLOPS, "avg_launch_ms": b_ms, "launches": la,
                       "alg_flops_per_launch": b_fl, "ms_total": ms}
    e16 = tm["band16_evals"]
    q_mean = tm["band16_q_sum"] / max(e16, 1.0)
    for key in ("band16_fwd_kernel", "band16_bwd_kernel"):
        k = sweeps[key]
        ppl = (e16 - tm["band16_wide_evals"]) / max(k["launches"], 1.0)  # problems per launch
        k["traffic"], k["traffic_source"] = band_traffic(key, ppl) if ppl > 0 else (None, None)
    k = sweeps["band16_wide_kernel"]
    ppl = tm["band16_wide_evals"] / max(k["launches"], 1.0)
    k["traffic"], k["traffic_source"] = band_traffic("band16_wide_kernel", ppl) if ppl > 0 else (None, None)
    for key, fwd in ((f64n, True), (b64n, False)):
        k = sweeps[key]
        pw = 2 if p2 >= tm["band_fused_launches"] > 0 else 1
        ppl = k["alg_flops_per_launch"] / band_problem_flops(n, pw, fwd)
        tkey = ("band_fwd1_kernel" if fwd else "band_bwd1_kernel")  # (the committed traffic passes: the p <= 1 pair)
        k["traffic"], k["traffic_source"] = band_traffic(tkey, ppl) if (ppl > 0 and pw == 1) else (None, None)
    # wave-time of each band16 kernel: problems per launch x launch ms, summed (one wavefront per
    # problem): the SIMD time it holds, which is what bounds the fits/s when thousands of problems
    # are in flight (the wide launch has the most device time — its few waves take ~10 ms each —
    # but holds a small share of the wave slots)
    for key in ("band16_fwd_kernel", "band16_bwd_kernel", "band16_wide_kernel"):
        k = sweeps[key]
        ev = tm["band16_wide_evals"] if key == "band16_wide_kernel" else e16 - tm["band16_wide_evals"]
        k["wave_s"] = ev * k["avg_launch_ms"] * 1e-3 if k["launches"] > 0 else 0.0
    from_p = tm["band_p_sum"] / max(tm["band_evals"], 1.0)
    # the whole chip over the timed region: the MFMA flops of every banded evaluation (band16
    # tile products + the 64-row sweeps' block products) / wall time
    # (the 64-row sweeps' flops are those of their timed launch pairs: the p <= 1 class's when the
    # call has one, else the p = 2 class's)
    chip_fl = (tm["band16_fwd_flops"] + tm["band16_bwd_flops"] + tm["band16_wide_flops"] + tm["band_fwd_flops"]
               + tm["band_bwd_flops"])
    chip_ach = chip_fl / elapsed / 1e12
    kname = max(sweeps, key=lambda k: sweeps[k]["ms_total"])
    if sweeps[kname]["ms_total"] > tm["contract_ms_total"]:
        k = sweeps[kname]
        b16 = kname.startswith("band16")
        roofline = {
            "kernel": ("band16_wide_kernel (the deferred Q = 4..8 classes: one wavefront walks a problem's 256 block "
                       "steps forward, then back)" if kname == "band16_wide_kernel" else
                       f"{kname}<Q> (16-row blocks, one wavefront walks a problem's 256 block steps; mean Q {q_mean:.2f})"
                       if b16 else f"{kname} (p<=1 class: one workgroup walks a problem's 64 block steps)"),
            # the sweeps are per-wave dependency chains, bounded by latency and by
            # how many of the chip's wave slots hold a sweep, not by the MFMA or HBM peak: the
            # MFMA fraction is reported as the contract's roofline, `occupancy` beside it
            "bound": "latency" if b16 else "mfma", "achieved": k["achieved"], "peak": FP64_PEAK_TFLOPS,
            "unit": "TFLOP/s", "frac": k["frac"], "traffic": k["traffic"], "traffic_source": k["traffic_source"],
            "trace_check": trace_check(kname),
            # NOT an occupancy: launch spans include the time a problem's wave is queued behind other
            # processes' work, so this can exceed 1. The measured residency is the wave trace's
            # (GPX_WAVE_TRACE=1: wave_trace.occupancy_2048; 0.67 of 2048 slots in round 5)
            "slot_demand": (tm["band16_wave_ms"] / (WAVE_SLOTS * elapsed * 1e3)) if b16 else None,
            "slot_demand_note": (f"sum over band16 launches of problems x HIP-event launch ms (queued time "
                                 f"included), over {WAVE_SLOTS} wave slots (256 CUs x 4 SIMDs x 2 sweeps per SIMD) "
                                 "x the timed wall ms; not a residency (see wave_trace.occupancy_2048)") if b16 else None,
            "traffic_unit": "bytes/launch", "avg_launch_ms": k["avg_launch_ms"], "launches": k["launches"],
            "alg_flops_per_launch": k["alg_flops_per_launch"], "mean_p_blocks": from_p,
            "band16_share_of_band_evals": e16 / max(tm["band_evals"], 1.0), "band16_mean_q": q_mean,
            "sweeps": {kk: {f: v.get(f) for f in ("achieved", "frac", "avg_launch_ms", "launches", "traffic", "wave_s")}
                       for kk, v in sweeps.items() if v["launches"] > 0},
            "by_wave_time": (lambda kw: {"kernel": kw, "frac": sweeps[kw]["frac"], "achieved": sweeps[kw]["achieved"],
                                         "wave_s_share": sweeps[kw]["wave_s"] / max(sum(sweeps[x].get("wave_s", 0.0)
                                                                                       for x in sweeps), 1e-30)})(
                max(("band16_fwd_kernel", "band16_bwd_kernel", "band16_wide_kernel"),
                    key=lambda x: sweeps[x].get("wave_s", 0.0))) if b16 else None,
            "chip_achieved": chip_ach, "chip_frac": chip_ach / FP64_PEAK_TFLOPS,
            "fp64_datapath": fp64_datapath(sweeps, elapsed) if b16 else None,
            "note": ("banded path (DESIGN.md §3c/§3d): the roofline kernel is the one with the most device time; "
                     "by_wave_time names the one holding the most wave-slot time (problems x launch ms), which bounds "
                     "the throughput; achieved = the MFMA flops a launch's problems issue (band16: "
                     "2*16^3 per 16x16x16 tile product, the 16x16 leaves' VALU work not counted; 64-row sweeps: "
                     "2*64^3 per block product, leaf 2/3 of one) / the launch's HIP-event duration; launches of "
                     "several device batches and host processes overlap on the GPU; traffic: the kernel's "
                     "profiles/<round>_band*_traffic.json x problems per launch"),
        }
    else:
        c_ms = tm["contract_ms_total"] / max(tm["contract_launches"], 1.0)
        c_fl = tm["contract_alg_flops"] / max(tm["contract_launches"], 1.0)
        ach = c_fl / (c_ms * 1e-3) / 1e12 if c_ms > 0 else 0.0
        traffic, src = contract_traffic(n, c_fl)
        roofline = {"kernel": "gemm_kernel<128,T,N,EPI_CONTRACT1> (K^-1 = W^T W fused with the gradient contraction)",
                    "bound": "mfma", "achieved": ach, "peak": FP64_PEAK_TFLOPS, "unit": "TFLOP/s",
                    "frac": ach / FP64_PEAK_TFLOPS, "traffic": traffic, "traffic_unit": "bytes/launch",
                    "traffic_source": src, "avg_launch_ms": c_ms, "launches": tm["contract_launches"],
                    "alg_flops_per_launch": c_fl}
    # host side: per process, the share of the timed region its one host thread was not waiting
    # for the device (driver stats), and its busy span
    host = []
    for p in parts:
        st = p[4] or {}
        # waiting for the device: the pipelined driver's device_wait, or (one batch per process)
        # the synchronous device calls, their submit/complete host work included
        wait = st.get("device_wait", 0.0) + st.get("device_call", 0.0)
        host.append({"proc": p[0], "fits": int(len(p[1])), "busy_s": p[5],
                     "host_share": (p[5] - wait) / p[5] if p[5] > 0 else None,
                     "rounds": st.get("rounds"), "fit_evals": st.get("fit_evals")})
    out = {
        "metric": "GP fits/sec (N=4096, 1-D RBF)",
        "value": value,
        "unit": "fits/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": args.scaling,
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic (C2 generator, seeded per rank/series)",
        "config": {"workload": "C2: exact GPR fit, synthetic 1-D series, N=4096, SquaredExponential, "
                               "fp64, sigma_n^2=1e-5 fixed, L-BFGS-B maxiter=100 + predict_f(X_train)",
                   "N": n, "fits_per_gpu_per_step": args.fits, "device_slots_per_gpu": args.width,
                   "host_processes_per_gpu": P, "device_batches_per_process": args.groups,
                   "admission_places": args.admission, "wide_slots_per_process": args.wide_slots,
                   "deferred_above_q": args.defer_q,
                   "slot_storage": args.storage, "kernel": "SquaredExponential",
                   "band_route": wk.engines[0].band_route,
                   "parallelism": f"independent fits, {world} rank(s) x 1 GPU x {P} host processes, "
                                  "RCCL all_gather of the per-fit results"},
        "nfev_mean": nfev_mean,
        "evals_per_s": evals_all / elapsed,
        "band_path": {"evals": tm["band_evals"], "dense_evals": tm["evals"] - tm["band_evals"],
                      "mean_p_blocks": from_p, "check_fallbacks": tm["band_fallbacks"],
                      "fallback_slot_evals": tm["shadow_evals"], "fallback_slot_predicts": tm["shadow_predicts"],
                      "ms_per_call": tm["band_ms_total"] / max(tm["band_calls"], 1.0),
                      "problems_per_call": tm["band_evals"] / max(tm["band_calls"], 1.0)},
        "host": host,
        "roofline": roofline,
        "box_cache": {"note": "the timed fits cycle over 512 resident series (12 fits each per step), marked immutable: "
                              "a rebind reuses the series' band boxes. Fresh series pay the box download and one stream "
                              "synchronise per call: GPX_BOX_CACHE=0 on the same box, 13431 vs 14192 fits/s (-5.3 %, "
                              "profiles/r05_ab.md)", "fresh_series_fits_per_s_same_box": 13431.2,
                      "cached_fits_per_s_same_box": 14191.8},
    }
    if args.scaling == "strong":
        out["config"]["fits_per_gpu_per_step"] = None
        out["config"]["total_fits_per_step"] = args.total_fits
        out["config"]["total_series"] = args.total_series
        out["data"] = "synthetic (C2 generator; one fixed batch of series split over the ranks)"
        hosts = [host]
        if world > 1:
            hosts = [None] * world
            dist.all_gather_object(hosts, host)
        plan = strong_fit_ids(args, world, P)
        out["strong"] = {
            "fits_per_rank_per_step": [sum(len(p) for p in pr) for pr in plan],
            "rank_host_share": [[h.get("host_share") for h in hr] for hr in hosts],
            "rank_busy_s_max": [max(h.get("busy_s") or 0.0 for h in hr) for hr in hosts],
            "note": ("a fixed batch of total_fits_per_step fits per step (the reference's per-asset loop is "
                     "fixed-size, Multi-Input_GPR/main.py:535-552) split by distributed.shard_lpt; the timed "
                     "region ends after the all_gather of the result table on every rank (max over ranks). "
                     "C3's own 20-series batch is bounded by secondary_c3_batch.ratio_wall_all_over_share: each "
                     "fit is a chain of ~20 dependent evaluations, so a batch of few fits cannot speed up past "
                     "that ratio; this batch holds thousands of fits per rank")}
    if parts[0][6] is not None:
        out["wave_trace"] = wave_trace_summary([p[6] for p in parts], elapsed)
        if os.environ.get("GPX_WAVE_TRACE_OUT"):  # raw records per host process (tools/wave_overlap.py)
            np.savez_compressed(os.environ["GPX_WAVE_TRACE_OUT"], **{f"proc{p[0]}": p[6] for p in parts})
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(n, nfev_mean)
    if rank == 0 and world == 1 and not args.no_secondary:
        for name, fn in (("secondary_c1_solo", lambda: secondary_c1_solo(gpu)),
                         ("secondary_solo", lambda: secondary_solo(gpu)),
                         ("secondary_c3_batch", lambda: secondary_c3(gpu)),
                         ("secondary_c4_dense", lambda: secondary_c4(gpu)),
                         ("secondary_c4_expxexp", lambda: secondary_c4(gpu, kind="expxexp")),
                         ("secondary_c5_svgp", lambda: secondary_c5(gpu))):
            try:
                out[name] = fn()
            except Exception as e:  # reported, never fatal to the headline line
                out[name] = {"error": f"{type(e).__name__}: {e}"}
    if rank == 0 and wk.driver_stats:
        out["driver_stats_last_call"] = wk.driver_stats[-1]
    if wk.traces and rank == 0:
        with open(os.environ.get("GPX_TRACE_OUT", "rounds_trace.json"), "w") as f:
            json.dump([[list(e) for e in tr] for tr in wk.traces], f)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
