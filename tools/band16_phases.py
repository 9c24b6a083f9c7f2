"""Per-phase cycle breakdown of the band16 sweeps (csrc/gpx_band16.hip) on C2-shaped problems
(N = 4096, SE, unit-spaced inputs), from the diagnostic library libgpx_phases.so (`make phases`:
each wave times its steps with s_memtime). Prints per kernel the mean shader-clock cycles per
16-row step of each phase.

usage: python tools/band16_phases.py [B] [ell ...]      (GPU box; JSON lines to stdout)
"""
import ctypes
import json
import os
import sys
import time

ROOT = os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ["GPX_LIB"] = os.path.join(ROOT, "portfoliooptgp_amd", "libgpx_phases.so")
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

import portfoliooptgp_amd as gpx  # noqa: E402
from portfoliooptgp_amd.engine import Engine  # noqa: E402
from portfoliooptgp_amd.kernels import compile_spec  # noqa: E402

NAMES = {0: ["glds + y", "leaf", "W out, z_k", "panels, u", "window update", "new row reads", "drain", "stores, shift"],
         1: ["loads, frags, glds", "alpha_k", "G", "Z panel", "Z_kk, Z out", "contract", "stores, shift",
             "band check", "drain"]}


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 512
    ells = [float(v) for v in sys.argv[2:]] or [1.18]
    n = 4096
    lib = ctypes.CDLL(os.environ["GPX_LIB"])
    lib.gpx_debug_band16_phases.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int]
    buf = (ctypes.c_ulonglong * 32)()
    x = np.arange(n, dtype=np.float64)
    rng = np.random.default_rng(0)
    ys = [rng.standard_normal(n) * 0.01 for _ in range(B)]
    eng = Engine([x] * B, ys, [compile_spec(gpx.kernels.SquaredExponential(), 1)] * B, band_storage=True)
    eng.ctx.set_profiling(True)
    for ell in ells:
        th = np.zeros((B, 16))
        th[:, :3] = [ell, 1.0, 1e-5]
        eng.lml_grad(np.arange(B), th)  # warm
        torch.cuda.synchronize()
        lib.gpx_debug_band16_phases(buf, 1)
        eng.reset_timing()
        reps = 5
        t0 = time.perf_counter()
        for _ in range(reps):
            eng.lml_grad(np.arange(B), th)
        torch.cuda.synchronize()
        wall = (time.perf_counter() - t0) / reps
        lib.gpx_debug_band16_phases(buf, 1)
        tm = eng.last_timing()
        v = np.frombuffer(buf, dtype=np.uint64).astype(np.float64).reshape(2, 16)
        row = {"B": B, "ell": ell, "wall_ms_per_call": wall * 1e3, "q_mean": tm.band16_q_sum / max(tm.band16_evals, 1),
               "fwd_ms": tm.band16_fwd_ms_total / max(tm.band16_launches, 1),
               "bwd_ms": tm.band16_bwd_ms_total / max(tm.band16_launches, 1), "kernels": {}}
        for kid in (0, 1):
            waves = v[kid, 15]
            if waves == 0:
                continue
            cyc = v[kid, :12] / (waves * (n // 16))
            tot = cyc.sum()
            row["kernels"][["fwd", "bwd"][kid]] = {
                "waves": int(waves), "cycles_per_step": round(tot, 1),
                "phases": {NAMES[kid][i]: [round(c, 1), round(c / tot, 3)] for i, c in enumerate(cyc[:len(NAMES[kid])])}}
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
