"""Rebind cost while another stream keeps every CU busy with banded sweeps (the bench's
situation): host-staged rebind from numpy vs from device tensors, and a bare tiny-kernel sync."""
import os
import sys
import threading
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
import portfoliooptgp_amd as gpx  # noqa: E402
from portfoliooptgp_amd.engine import Engine  # noqa: E402
from portfoliooptgp_amd.kernels import compile_spec  # noqa: E402

n = 4096
x, y = bench.synthetic_series(n, 0)
xd, yd = torch.as_tensor(x, device="cuda:0"), torch.as_tensor(y, device="cuda:0")
spec = compile_spec(gpx.kernels.SquaredExponential(), 1)
big = Engine([xd] * 256, [yd] * 256, [spec] * 256, device=0)
small = Engine([xd] * 4, [yd] * 4, [spec] * 4, device=0)
th = np.ones((256, 16))
th[:, :3] = [1.2, 0.6, 1e-5]
stop = threading.Event()


def load():
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        while not stop.is_set():
            big.lml_grad(list(range(256)), th)


def timeit(label, fn, reps=50):
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    print(f"{label}: {(time.perf_counter() - t0) / reps * 1e6:.1f} us", flush=True)


s2 = torch.cuda.Stream()
with torch.cuda.stream(s2):
    timeit("idle: rebind from numpy", lambda: small.rebind(1, x, y, spec))
    timeit("idle: rebind from device tensors", lambda: small.rebind(1, xd, yd, spec))
    t = threading.Thread(target=load, daemon=True)
    t.start()
    time.sleep(0.5)
    timeit("loaded: rebind from numpy", lambda: small.rebind(1, x, y, spec))
    timeit("loaded: rebind from device tensors", lambda: small.rebind(1, xd, yd, spec))
    z = torch.zeros(16, device="cuda:0")

    def tiny():
        z.add_(1.0)
        torch.cuda.current_stream().synchronize()
    timeit("loaded: tiny kernel + sync", tiny)
    hb = torch.empty(2 * n, dtype=torch.float64, pin_memory=True)

    def d2h():
        hb[:n].copy_(yd.reshape(-1), non_blocking=True)
        torch.cuda.current_stream().synchronize()
    timeit("loaded: D2H 32 KB to pinned + sync", d2h)
    yd2 = torch.empty_like(yd)

    def h2d():
        yd2.reshape(-1).copy_(hb[:n], non_blocking=True)
        torch.cuda.current_stream().synchronize()
    timeit("loaded: H2D 32 KB from pinned + sync", h2d)

    hb2 = torch.empty(2 * n, dtype=torch.float64, pin_memory=True)

    def d2h_both():
        hb2[:n].copy_(xd.reshape(-1), non_blocking=True)
        hb2[n:].copy_(yd.reshape(-1), non_blocking=True)
        torch.cuda.current_stream().synchronize()
    timeit("loaded: D2H X and Y to pinned + one sync", d2h_both)

    def d2h_x():
        hb2[:n].copy_(xd.reshape(-1), non_blocking=True)
        torch.cuda.current_stream().synchronize()
    timeit("loaded: D2H X ([n,1]) to pinned + sync", d2h_x)
    import ctypes
    from portfoliooptgp_amd import _native as N

    def c_dev():
        rc = small.lib.gpx_batch_rebind_device(small.handle, 1, n, ctypes.c_void_p(xd.data_ptr()),
                                               ctypes.c_void_p(yd.data_ptr()), ctypes.byref(spec),
                                               small._stream())
        assert rc == 0
    timeit("loaded: gpx_batch_rebind_device", c_dev)

    def rb_sync():
        small.rebind(1, x, y, spec)
        torch.cuda.current_stream().synchronize()
    timeit("loaded: rebind from numpy + sync", rb_sync)
    stop.set()
    t.join()
