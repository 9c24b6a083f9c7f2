import torch, time
for n in (4096, 8192):
    a = torch.randint(-120, 120, (n, n), dtype=torch.int8, device="cuda")
    b = torch.randint(-120, 120, (n, n), dtype=torch.int8, device="cuda")
    for _ in range(3): c = torch._int_mm(a, b)
    torch.cuda.synchronize(); t = time.perf_counter(); r = 10
    for _ in range(r): c = torch._int_mm(a, b)
    torch.cuda.synchronize(); dt = (time.perf_counter() - t) / r
    print(f"torch._int_mm n={n}: {dt*1e3:.3f} ms  {2*n**3/dt/1e12:.0f} TOPS")
    x = torch.randn(n, n, dtype=torch.float64, device="cuda"); y = torch.randn(n, n, dtype=torch.float64, device="cuda")
    for _ in range(2): z = x @ y
    torch.cuda.synchronize(); t = time.perf_counter()
    for _ in range(5): z = x @ y
    torch.cuda.synchronize(); dt = (time.perf_counter() - t) / 5
    print(f"fp64 matmul n={n}: {dt*1e3:.3f} ms  {2*n**3/dt/1e12:.1f} TFLOPS")
