"""Vendor-library reference points on the same MI355X (rocBLAS/hipBLASLt dgemm, rocSOLVER potrf,
triangular inverse) for the FP64 work of one PSO step at N=4096, P=64. Diagnostics only."""
import time
import torch

def timeit(f, reps=5):
    f(); torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        f()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / reps

dev = "cuda"
for n in (4096, 8192):
    a = torch.randn(n, n, dtype=torch.float64, device=dev); b = torch.randn(n, n, dtype=torch.float64, device=dev)
    dt = timeit(lambda: a @ b)
    print(f"dgemm {n}^3: {2*n**3/dt/1e12:.1f} TFLOP/s ({dt*1e3:.1f} ms)")
N, P = 4096, 16
x = torch.rand(P, 3, N, dtype=torch.float64, device=dev)
d2 = ((x[:, :, :, None] - x[:, :, None, :]) ** 2).sum(1) / 0.09
K = torch.exp(-0.5 * d2) + 0.01 * torch.eye(N, dtype=torch.float64, device=dev)
dt = timeit(lambda: torch.linalg.cholesky(K), reps=3)
print(f"batched potrf P={P} N={N}: {dt*1e3:.1f} ms, {P*N**3/3/dt/1e12:.1f} TFLOP/s, per particle {dt/P*1e3:.2f} ms")
L = torch.linalg.cholesky(K)
I = torch.eye(N, dtype=torch.float64, device=dev).expand(P, N, N)
dt2 = timeit(lambda: torch.linalg.solve_triangular(L, I, upper=False), reps=3)
print(f"batched trsm (L^-1 via N RHS) P={P}: {dt2*1e3:.1f} ms, {P*N**3/dt2/1e12:.1f} TFLOP/s (N^3 flops/particle)")
print(f"vendor potrf+trsm per particle: {(dt+dt2)/P*1e3:.2f} ms -> {P/(dt+dt2):.0f} evals/s upper bound")
