"""Probe vendor-library fp64 rates on the GPU box (context numbers only, never the product path)."""
import time, torch
dev = "cuda:0"
print(torch.cuda.get_device_name(0), torch.version.hip)
def timeit(f, reps=5):
    f(); torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps): f()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / reps
n = 4096
a = torch.randn(n, n, dtype=torch.float64, device=dev)
b = torch.randn(n, n, dtype=torch.float64, device=dev)
t = timeit(lambda: a @ b)
print(f"DGEMM {n}^3 rocBLAS: {t*1e3:.2f} ms  {2*n**3/t/1e12:.2f} TFLOP/s")
x = torch.arange(n, dtype=torch.float64, device=dev)
K = torch.exp(-0.5 * (x[:, None] - x[None, :]) ** 2 / 64.0**2) + 1e-5 * torch.eye(n, dtype=torch.float64, device=dev)
t = timeit(lambda: torch.linalg.cholesky(K))
print(f"potrf {n} single: {t*1e3:.2f} ms  {n**3/3/t/1e12:.2f} TFLOP/s")
Kb = K.unsqueeze(0).repeat(8, 1, 1).contiguous()
t = timeit(lambda: torch.linalg.cholesky(Kb), reps=3)
print(f"potrf {n} batch8: {t*1e3:.2f} ms  {8*n**3/3/t/1e12:.2f} TFLOP/s")
L = torch.linalg.cholesky(K)
t = timeit(lambda: torch.cholesky_inverse(L), reps=3)
print(f"potri {n}: {t*1e3:.2f} ms  {2*n**3/3/t/1e12:.2f} TFLOP/s")
print("bandwidth probe:")
big = torch.empty(2**28, dtype=torch.float64, device=dev)
t = timeit(lambda: big.mul_(1.0000001))
print(f"  in-place scale 2 GiB: {2*big.numel()*8/t/1e12:.2f} TB/s")
