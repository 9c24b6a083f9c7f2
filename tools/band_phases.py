"""Per-phase cycle breakdown of the fused banded sweeps (band_fwd1/bwd1 for p <= 1,
band_fwd/bwd for p = 2) on C2-shaped problems (N = 4096, SE kernel, unit-spaced inputs).

Loads the diagnostic library libgpx_phases.so (`make phases`: gpx_band.hip compiled with
-DGPX_BAND_PHASES, thread 0 of each workgroup timing its block steps with s_memtime) and
prints, per kernel, the mean shader-clock cycles per block step of each phase and the share
of the step. Phase names follow the PH(i) markers in gpx_band.hip.

usage: python tools/band_phases.py [B] [ell ...]      (GPU box; writes JSON to stdout)
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

NAMES = {
    0: ["stage A_kk", "leaf", "W out, z_k, panel in", "P = A W^T", "P out", "u, SYRK", "tail", "", "", "", "", ""],
    1: ["alpha_k", "W^TW, G", "Z_k+1,k, Z_kk", "Z out, prefetch", "contract diag", "contract off",
        "sums, check", "", "", "", "", ""],
    2: ["stage", "leaf", "W out, z_k", "panels", "u, window update", "", "", "", "", "", "", ""],
    3: ["alpha_k", "W^TW, G", "Z blocks", "prefetch", "contract", "sums, check", "", "", "", "", "", ""],
}


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    ells = [float(v) for v in sys.argv[2:]] or [1.0]
    n = 4096
    lib = ctypes.CDLL(os.environ["GPX_LIB"])
    lib.gpx_debug_band_phases.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int]
    buf = (ctypes.c_ulonglong * 72)()
    x = np.arange(n, dtype=np.float64)
    rng = np.random.default_rng(0)
    ys = [rng.standard_normal(n) * 0.01 for _ in range(B)]
    eng = Engine([x] * B, ys, [compile_spec(gpx.kernels.SquaredExponential(), 1)] * B)
    eng.ctx.set_profiling(True)
    out = []
    for ell in ells:
        th = np.zeros((B, 16))
        th[:, :3] = [ell, 1.0, 1e-5]
        eng.lml_grad(np.arange(B), th)  # warm
        torch.cuda.synchronize()
        lib.gpx_debug_band_phases(buf, 1)
        reps = 5
        t0 = time.perf_counter()
        for _ in range(reps):
            eng.lml_grad(np.arange(B), th)
        torch.cuda.synchronize()
        wall = (time.perf_counter() - t0) / reps
        lib.gpx_debug_band_phases(buf, 1)
        tm = eng.last_timing()
        allv = np.frombuffer(buf, dtype=np.uint64).astype(np.float64)
        v = allv[:64].reshape(4, 16)
        lv = allv[64:]
        row = {"B": B, "ell": ell, "wall_ms_per_call": wall * 1e3, "band_p_sum": tm.band_p_sum,
               "band_fwd_ms": tm.band_fwd_ms_total, "band_bwd_ms": tm.band_bwd_ms_total, "kernels": {}}
        if lv[7] > 0:
            lc = lv[:4] / lv[7]
            row["leaf"] = {"leaves": int(lv[7]), "cycles": round(lc.sum(), 1),
                           "phases": {nm: round(c, 1) for nm, c in zip(["diag", "panel", "trailing", "inverse"], lc)}}
        for kid in (0, 1, 2, 3):
            wgs = v[kid, 15]
            if wgs == 0:
                continue
            steps = wgs * (n // 64)
            cyc = v[kid, :12] / steps
            tot = cyc.sum()
            row["kernels"][["fwd1", "bwd1", "fwd2", "bwd2"][kid]] = {
                "workgroups": int(wgs), "cycles_per_step": round(tot, 1),
                "phases": {NAMES[kid][i] or f"ph{i}": [round(c, 1), round(c / tot, 3)]
                           for i, c in enumerate(cyc) if c > 0}}
        out.append(row)
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
