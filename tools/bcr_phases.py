"""Per-phase shader-clock cycles of the block-cyclic-reduction kernels (csrc/gpx_bcr.hip) from the
diagnostic library libgpx_phases.so (`make phases`, -DGPX_BCR_PHASES: thread 0 of every
workgroup times its phases with s_memtime). One C2-shaped problem (N, SE, unit-spaced inputs)
evaluated `reps` times at each ℓ; prints per kernel and level the mean cycles per workgroup.

usage: python tools/bcr_phases.py [N] [problems] [ell ...]      (GPU box; JSON lines to stdout)"""
import ctypes
import json
import os
import sys

ROOT = os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ["GPX_LIB"] = os.path.join(ROOT, "portfoliooptgp_amd", "libgpx_phases.so")
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402

import portfoliooptgp_amd as gpx  # noqa: E402
from portfoliooptgp_amd.engine import Engine  # noqa: E402
from portfoliooptgp_amd.kernels import compile_spec  # noqa: E402

NAMES = {0: ["loads", "rhs init", "sweep", "stores", "updates"],
         1: ["loads", "alpha", "G, WtW", "Z loads", "Z panels", "-", "Z_XX, stores"],
         2: ["stage", "elements", "reduce, out"]}


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
    B = int(sys.argv[2]) if len(sys.argv) > 2 else 1
    ells = [float(v) for v in sys.argv[3:]] or [1.18, 1.9]
    lib = ctypes.CDLL(os.environ["GPX_LIB"])
    lib.gpx_debug_bcr_phases.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int]
    buf = (ctypes.c_ulonglong * (3 * 16 * 16))()
    x = np.arange(n, dtype=np.float64)
    rng = np.random.default_rng(0)
    ys = [rng.standard_normal(n) for _ in range(B)]
    eng = Engine([x] * B, ys, [compile_spec(gpx.kernels.SquaredExponential(), 1)] * B)
    reps = 20
    for ell in ells:
        th = np.ones((B, 16))
        th[:, 0] = ell
        th[:, 2] = 1e-5
        eng.lml_grad(list(range(B)), th)
        lib.gpx_debug_bcr_phases(buf, 1)
        for _ in range(reps):
            eng.lml_grad(list(range(B)), th)
        lib.gpx_debug_bcr_phases(buf, 1)
        a = np.frombuffer(buf, dtype=np.uint64).reshape(3, 16, 16).astype(np.float64)
        for k in range(3):
            for lev in range(16):
                cnt = a[k, lev, 15]
                if cnt == 0:
                    continue
                ph = {NAMES[k][i]: round(a[k, lev, i] / cnt) for i in range(len(NAMES[k]))}
                print(json.dumps({"ell": ell, "N": n, "kernel": ["fwd", "bwd", "contract"][k], "level": lev,
                                  "wgs_per_eval": cnt / reps, "cycles_per_wg": ph,
                                  "total_per_wg": round(sum(a[k, lev, :8]) / cnt)}), flush=True)


if __name__ == "__main__":
    main()
