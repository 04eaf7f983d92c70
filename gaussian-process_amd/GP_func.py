"""Drop-in for the reference's GP_func.py, computed on the MI355X.

Same public surface as /GP_func.py of rferguson22/Gaussian-Process:
    GP(x_known, y_known, e_known, x_fit, lengths, batch_size=10000) -> (mu, sigma)
        (GP_func.py:12-45)
    kernel_func(x1, x2, l) -> (N1, N2) array                       (GP_func.py:49-65)

Both run through libgpfit (include/gpfit.h: gpf_predict, gpf_kernel); a
non-positive-definite covariance raises numpy.linalg.LinAlgError like
numpy.linalg.cholesky does at GP_func.py:22. There is no CPU fallback.
"""
import numpy as np

from gpfit._lib import default_context

__all__ = ["GP", "kernel_func"]


def GP(x_known, y_known, e_known, x_fit, lengths, batch_size=10000):
    """GP regression mean / sd at x_fit (GP_func.py:12-45).

    K = k(x,x) + diag(e^2) is factorised once on the device (L and L^-1);
    every query column gets mu = K_s^T alpha and
    sd = sqrt(clip(1 - ||L^-1 K_s||^2, 1e-12)) without materialising
    L^-1 K_s. ``batch_size`` is accepted for signature parity; on the device
    the query set is chunked by available memory and the chunking does not
    change the result (as in the reference).
    """
    x_known = np.asarray(x_known, dtype=np.float64)
    x_fit = np.asarray(x_fit, dtype=np.float64)
    if x_fit.ndim != 2 or x_fit.shape[0] != x_known.shape[0]:
        raise ValueError("x_fit must be (d, M) with the same d as x_known")
    ctx = default_context()
    ctx.set_data(x_known, y_known, e_known)
    return ctx.predict(lengths, x_fit, batch_size)


def kernel_func(x1, x2, l):
    """Unit-amplitude squared-exponential kernel between column sets (GP_func.py:49-65)."""
    x1 = np.asarray(x1, dtype=np.float64)
    x2 = np.asarray(x2, dtype=np.float64)
    return default_context().kernel(x1, x2, np.asarray(l, dtype=np.float64))
