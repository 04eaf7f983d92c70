"""GPU diagnostics: per-block factor errors vs NumPy, MFMA peak, rocBLAS dgemm rate."""
import os, sys, time
os.environ.setdefault("OMP_NUM_THREADS", "1")
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gaussian-process_amd")]
import torch  # initialise the HIP runtime through torch first
import gpfit
from oracle import ref_cpu

ctx = gpfit.Context(0)
for N in [65, 100, 128, 200, 300]:
    rng = np.random.default_rng(N)
    x = rng.uniform(size=(2, N)); y = np.sin(3 * x[0]) + x[1]; e = np.full(N, 0.1)
    ls = np.array([0.3, 0.4])
    ctx.set_data(x, y, e)
    L, U, z, al = ctx.debug_factor(ls)
    npad = L.shape[0]
    K = np.eye(npad); K[:N, :N] = ref_cpu.kernel_func(x, x, ls) + np.diag(e ** 2)
    Lr = np.linalg.cholesky(K); Ur = np.linalg.inv(Lr)
    yp = np.zeros(npad); yp[:N] = y
    zr = Ur @ yp
    Lg = np.tril(L); Ug = np.tril(U)
    print(f"N={N} npad={npad}")
    for bi in range(npad // 64):
        for bj in range(bi + 1):
            sl = (slice(bi * 64, bi * 64 + 64), slice(bj * 64, bj * 64 + 64))
            el = np.abs(Lg[sl] - Lr[sl]).max(); eu = np.abs(Ug[sl] - Ur[sl]).max()
            print(f"  block ({bi},{bj}) |dL|={el:.2e} |dU|={eu:.2e}")
    print(f"  |dz| per 64: {[float(np.abs(z[i:i+64]-zr[i:i+64]).max()) for i in range(0, npad, 64)]}")
    ar = Ur[:, :N].T @ zr
    print(f"  |dalpha|={np.abs(al - ar[:N]).max():.2e}")
print("mfma f64 peak TFLOP/s:", [round(ctx.mfma_peak(blocks=b, iters=2048), 2) for b in (256, 1024, 2048)])
import torch
for n in (4096, 8192):
    a = torch.randn(n, n, dtype=torch.float64, device="cuda"); b = torch.randn(n, n, dtype=torch.float64, device="cuda")
    for _ in range(2): c = a @ b
    torch.cuda.synchronize(); t = time.perf_counter()
    for _ in range(5): c = a @ b
    torch.cuda.synchronize(); dt = (time.perf_counter() - t) / 5
    print(f"torch/rocBLAS dgemm {n}^3: {2 * n**3 / dt / 1e12:.1f} TFLOP/s")
