"""Config C4 (bench.py secondary_c4: D = 5, N = 4096, fp64, dense path) over device-batch layouts:
the 32 fits in 1, 2 or 4 concurrent batches, Matern52 and the reference's Exp x Exp product.
usage: python tools/c4_layouts.py [groups ...]   (GPU box; JSON lines)"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

for g in [int(v) for v in sys.argv[1:]] or [1, 2, 4]:
    for kind in ("m52",):
        r = bench.secondary_c4(0, kind=kind, groups=g)
        print(json.dumps({"groups": g, "kind": kind, "fits_per_s": r["fits_per_s"], "eval_alg_tflops": r["eval_alg_tflops"],
                          "nfev_mean": r["nfev_mean"], "nfev_max": r["nfev_max"], "seconds": r["seconds"], "contraction_frac": r["contraction_roofline"]["frac"]}), flush=True)
