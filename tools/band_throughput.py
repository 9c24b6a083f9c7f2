"""Device ceiling of the banded C2 evaluation, no L-BFGS-B host loop in the way: G band-storage
engines of B problems each (C2 series, N = 4096, SE at ℓ = 1.18, σn² = 1e-5: the p = 1 class),
evaluated back to back on their own streams (submit all, complete all) for `reps` rounds.
Prints evaluations/s, the fused sweeps' average launch times and the chip's block-product rate.

usage: python tools/band_throughput.py [--b 384] [--g 4] [--reps 20] [--ell 1.18]
       [--ells 1.18:0.89,1.6:0.05,1.9:0.06]   (a mix of width classes: ℓ:share, spread over every batch)
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from bench import band_problem_flops, synthetic_series, FP64_PEAK_TFLOPS  # noqa: E402
from portfoliooptgp_amd import kernels as K  # noqa: E402
from portfoliooptgp_amd.engine import Engine  # noqa: E402
from portfoliooptgp_amd.kernels import compile_spec  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--b", type=int, default=384)
    ap.add_argument("--g", type=int, default=4)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--ell", type=float, default=1.18)
    ap.add_argument("--series", type=int, default=64, help="distinct series (cycled over the slots)")
    ap.add_argument("--ells", default="", help="ℓ:share,... (a class mix; overrides --ell)")
    a = ap.parse_args()
    n = 4096
    data = [synthetic_series(n, s) for s in range(a.series)]
    spec = compile_spec(K.SquaredExponential(), 1)
    engs = []
    for g in range(a.g):
        idx = [(g * a.b + i) % a.series for i in range(a.b)]
        e = Engine([data[i][0] for i in idx], [data[i][1] for i in idx], [spec] * a.b, band_storage=True)
        engs.append(e)
    engs[0].ctx.set_profiling(True)
    streams = [torch.cuda.Stream() for _ in engs]
    th = np.ones((a.b, 16))
    th[:, :3] = [a.ell, 1.0, 1e-5]
    if a.ells:
        mix = [tuple(map(float, t.split(":"))) for t in a.ells.split(",")]
        w = np.array([m[1] for m in mix]) / sum(m[1] for m in mix)
        cnt = np.floor(w * a.b).astype(int)
        cnt[0] += a.b - cnt.sum()
        th[:, 0] = np.repeat([m[0] for m in mix], cnt)
    act = list(range(a.b))

    def rnd():
        for e, s in zip(engs, streams):
            with torch.cuda.stream(s):
                e.lml_grad_submit(act, th)
        for e in engs:
            e.lml_grad_complete()
    rnd()
    torch.cuda.synchronize()
    for e in engs:
        e.reset_timing()
    t0 = time.perf_counter()
    for _ in range(a.reps):
        rnd()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    tms = [e.last_timing() for e in engs]
    evals = sum(t.band_evals for t in tms)
    fl = lambda f: sum(getattr(t, f) for t in tms)  # noqa: E731
    per_eval = band_problem_flops(n, 1, True) + band_problem_flops(n, 1, False)
    out = {"B": a.b, "G": a.g, "reps": a.reps, "ell": a.ells or a.ell, "evals_per_s": evals / dt,
           "ms_per_round": dt / a.reps * 1e3, "band_evals": evals,
           "fwd1_avg_ms": fl("band_fwd_ms_total") / max(fl("band_fused_launches"), 1),
           "bwd1_avg_ms": fl("band_bwd_ms_total") / max(fl("band_fused_launches"), 1),
           "mean_p": fl("band_p_sum") / max(evals, 1), "check_fallbacks": fl("band_fallbacks"),
           "chip_tflops": evals * per_eval / dt / 1e12}
    out["chip_frac"] = out["chip_tflops"] / FP64_PEAK_TFLOPS
    e16 = fl("band16_evals")
    if e16 > 0:  # the band16 sweeps: launch times and the MFMA flops they issue
        la = max(fl("band16_launches"), 1)
        out.update({"band16_evals": e16, "band16_mean_q": fl("band16_q_sum") / e16,
                    "b16_fwd_avg_ms": fl("band16_fwd_ms_total") / la, "b16_bwd_avg_ms": fl("band16_bwd_ms_total") / la,
                    "b16_fwd_tflops": fl("band16_fwd_flops") / max(fl("band16_fwd_ms_total"), 1e-9) / 1e9,
                    "b16_bwd_tflops": fl("band16_bwd_flops") / max(fl("band16_bwd_ms_total"), 1e-9) / 1e9,
                    "b16_chip_mfma_tflops": (fl("band16_fwd_flops") + fl("band16_bwd_flops")) / dt / 1e12})
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
