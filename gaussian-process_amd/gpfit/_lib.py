"""ctypes binding of libgpfit.so (the C-ABI in include/gpfit.h).

There is deliberately no CPU fallback: if the HIP library is missing or no
device is visible, every entry point raises. The checker (oracle/) is a
separate, test-only tree.
"""
from __future__ import annotations

import ctypes
import hashlib
import os
from pathlib import Path

import numpy as np

PKG_DIR = Path(__file__).resolve().parent.parent
LIB_PATH = Path(os.environ.get("GPFIT_LIB", PKG_DIR / "libgpfit.so"))

GPF_OK, GPF_NOT_PD, GPF_HIP_ERROR, GPF_BAD_ARG = 0, 1, 2, 3
GPF_COMM_RCCL, GPF_COMM_HOST = 1, 2
GPF_OP_SUM, GPF_OP_MAX = 0, 1
ABI_VERSION = 2

_dp = ctypes.POINTER(ctypes.c_double)
_ip = ctypes.POINTER(ctypes.c_int)
_vp = ctypes.c_void_p

# name -> (restype, argtypes); mirrors include/gpfit.h
SIGNATURES = {
    "gpf_version": (ctypes.c_int, []),
    "gpf_tile": (ctypes.c_int, []),
    "gpf_open": (ctypes.c_int, [ctypes.c_int, ctypes.POINTER(_vp)]),
    "gpf_close": (None, [_vp]),
    "gpf_last_error": (ctypes.c_char_p, [_vp]),
    "gpf_set_data": (ctypes.c_int, [_vp, _dp, _dp, _dp, ctypes.c_int64, ctypes.c_int]),
    "gpf_set_grid": (ctypes.c_int, [_vp, _dp, _dp, ctypes.c_int, _dp, _dp]),
    "gpf_eval_batch": (ctypes.c_int, [_vp, _dp, ctypes.c_int, _dp, _dp, _dp, _ip]),
    "gpf_predict": (ctypes.c_int, [_vp, _dp, _dp, ctypes.c_int64, ctypes.c_int64, _dp, _dp]),
    "gpf_kernel": (ctypes.c_int, [_vp, _dp, ctypes.c_int64, _dp, ctypes.c_int64, ctypes.c_int, _dp, _dp]),
    "gpf_log_marginal_likelihood": (ctypes.c_int, [_vp, _dp, _dp]),
    "gpf_set_profiling": (ctypes.c_int, [_vp, ctypes.c_int]),
    "gpf_get_profile": (ctypes.c_int, [_vp, _dp, ctypes.c_int]),
    "gpf_reset_profile": (ctypes.c_int, [_vp]),
    "gpf_selftest_mfma": (ctypes.c_int, [_vp, _dp, _dp, _dp]),
    "gpf_debug_factor": (ctypes.c_int, [_vp, _dp, _dp, _dp, _dp, _dp]),
    "gpf_debug_factor128": (ctypes.c_int, [_vp, _dp, _dp, ctypes.c_int, _dp, _dp, _dp, _dp, _dp, _ip, _dp]),
    "gpf_mfma_peak": (ctypes.c_int, [_vp, ctypes.c_int, ctypes.c_int, _dp]),
    "gpf_prob_surface": (ctypes.c_int, [_vp, _dp, ctypes.c_int64, ctypes.c_int, _dp, _dp,
                                        ctypes.POINTER(ctypes.c_int)]),
    "gpf_hull_fill": (ctypes.c_int, [_vp, _dp, ctypes.c_int64, ctypes.c_int, _dp, ctypes.POINTER(ctypes.c_int),
                                     ctypes.POINTER(ctypes.c_int64)]),
    "gpf_hull_fetch": (ctypes.c_int, [_vp, _dp]),
    "gpf_gemm_bench": (ctypes.c_int, [_vp, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                      ctypes.c_int, _dp]),
    "gpf_build_info": (ctypes.c_char_p, []),
    "gpf_sync": (ctypes.c_int, [_vp]),
    "gpf_comm_open": (ctypes.c_int, [_vp, ctypes.c_int, ctypes.c_int, ctypes.c_char_p, ctypes.c_int, ctypes.c_int,
                                     ctypes.POINTER(_vp)]),
    "gpf_comm_close": (None, [_vp]),
    "gpf_comm_rank": (ctypes.c_int, [_vp]),
    "gpf_comm_size": (ctypes.c_int, [_vp]),
    "gpf_comm_last_error": (ctypes.c_char_p, [_vp]),
    "gpf_comm_stats": (ctypes.c_int, [_vp, _dp, ctypes.POINTER(ctypes.c_longlong)]),
    "gpf_comm_allreduce": (ctypes.c_int, [_vp, _dp, ctypes.c_int64, ctypes.c_int]),
    "gpf_comm_exchange_scores": (ctypes.c_int, [_vp, ctypes.c_int, _dp, ctypes.c_int, ctypes.c_int, _dp, _ip]),
    "gpf_eval_batch_sharded": (ctypes.c_int, [_vp, _vp, _dp, ctypes.c_int, _dp, _ip]),
    "gpf_plan_check": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_longlong),
                                      ctypes.c_char_p, ctypes.c_int]),
    "gpf_bench_clock": (ctypes.c_int, [_vp, _dp]),
    "gpf_kmeans_set": (ctypes.c_int, [_vp, _dp, ctypes.c_int64, ctypes.c_int]),
    "gpf_kmeans_step": (ctypes.c_int, [_vp, _dp, ctypes.c_int, ctypes.c_int, _ip, _dp, _dp, _dp]),
}

_LIB = None


class GPFitError(RuntimeError):
    """HIP runtime failure inside libgpfit."""


def load_library():
    """Load libgpfit.so (raises OSError with a build hint if it is missing)."""
    global _LIB
    if _LIB is not None:
        return _LIB
    if not LIB_PATH.exists():
        raise OSError(f"{LIB_PATH} not found: build it with `python -c 'import __graft_entry__ as g; g.build()'`")
    lib = ctypes.CDLL(str(LIB_PATH))
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if lib.gpf_version() != ABI_VERSION:
        raise OSError(f"libgpfit ABI {lib.gpf_version()} != expected {ABI_VERSION}")
    _LIB = lib
    return lib


def build_info():
    """Provenance string baked into the loaded library (gpf_build_info)."""
    return load_library().gpf_build_info().decode()


def plan_check(particles, nt):
    """Host-side check of the k_step dispatch plan (gpf_plan_check); raises AssertionError
    naming the first violation, else returns the stats dict. Reads the GPF_* environment."""
    lib = load_library()
    stats = (ctypes.c_longlong * 11)()
    msg = ctypes.create_string_buffer(256)
    rc = lib.gpf_plan_check(int(particles), int(nt), stats, msg, 256)
    if rc != GPF_OK:
        raise AssertionError(f"plan_check(pc={particles}, nt={nt}): {msg.value.decode()}")
    keys = ("launches", "workgroups", "whole_tiles", "split_tiles", "S", "Smax", "groups", "diag_workgroups",
            "syrk_workgroups", "persistent", "lead_launches")
    return dict(zip(keys, list(stats)))


def _f64(a):
    return np.ascontiguousarray(a, dtype=np.float64)


def _ptr(a):
    return a.ctypes.data_as(_dp)


def _digest(*arrays):
    """sha256 over the arrays' shapes and bytes: the key that decides whether an upload can be
    skipped (a Python hash() collision would silently score stale data)."""
    h = hashlib.sha256()
    for a in arrays:
        h.update(repr(a.shape).encode())
        h.update(a.tobytes())
    return h.digest()


def default_device():
    """One process per GPU: torch.distributed launchers export LOCAL_RANK."""
    return int(os.environ.get("GPFIT_DEVICE", os.environ.get("LOCAL_RANK", "0")))


class Context:
    """One HIP device, one stream, device-resident training data (gpf_ctx)."""

    def __init__(self, device=None):
        self.lib = load_library()
        self.device = default_device() if device is None else int(device)
        h = _vp()
        rc = self.lib.gpf_open(self.device, ctypes.byref(h))
        if rc != GPF_OK or not h.value:
            raise GPFitError(f"gpf_open(device={self.device}) failed (rc={rc}); is a GPU visible?")
        self._h = h
        self.N = 0
        self.d = 0
        self._data_key = None
        self._grid_key = None

    def close(self):
        if getattr(self, "_h", None) is not None and self._h.value:
            self.lib.gpf_close(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # -- error mapping: same exception types as the reference's numpy path --
    def _check(self, rc, what, bad=None):
        if rc == GPF_OK:
            return
        msg = self.lib.gpf_last_error(self._h).decode(errors="replace")
        if rc == GPF_NOT_PD:
            err = np.linalg.LinAlgError("Matrix is not positive definite")
            # the batch row of the first failing particle (gpf_eval_batch's bad_idx), or None
            err.particle = None if bad is None or bad.value < 0 else int(bad.value)
            raise err
        if rc == GPF_BAD_ARG:
            raise ValueError(f"{what}: {msg}")
        raise GPFitError(f"{what}: {msg}")

    def set_data(self, x_dN, y, e):
        x = _f64(x_dN)
        if x.ndim != 2:
            raise ValueError("x must be (d, N)")
        y, e = _f64(y), _f64(e)
        d, n = x.shape
        key = _digest(x, y, e)
        if key == self._data_key:
            return
        self._check(self.lib.gpf_set_data(self._h, _ptr(x), _ptr(y), _ptr(e), n, d), "gpf_set_data")
        self.N, self.d = n, d
        self._data_key = key
        self._grid_key = None

    def set_grid(self, sigma_vals, expected, lo, hi):
        s, ex = _f64(sigma_vals), _f64(expected)
        lo, hi = _f64(lo).reshape(-1), _f64(hi).reshape(-1)
        key = _digest(s, ex, lo, hi)
        if key == self._grid_key:
            return
        self._check(self.lib.gpf_set_grid(self._h, _ptr(s), _ptr(ex), s.shape[0], _ptr(lo), _ptr(hi)),
                    "gpf_set_grid")
        self._grid_key = key

    def eval_batch(self, positions, want_mu_sd=False):
        P = _f64(positions)
        if P.ndim == 1:
            P = P.reshape(1, -1)
        n = P.shape[0]
        loss = np.empty(n)
        mu = np.empty((n, self.N)) if want_mu_sd else None
        sd = np.empty((n, self.N)) if want_mu_sd else None
        bad = ctypes.c_int(-1)
        rc = self.lib.gpf_eval_batch(self._h, _ptr(P), n, _ptr(loss),
                                     _ptr(mu) if want_mu_sd else None,
                                     _ptr(sd) if want_mu_sd else None, ctypes.byref(bad))
        self._check(rc, "gpf_eval_batch", bad)
        return (loss, mu, sd) if want_mu_sd else loss

    def eval_batch_sharded(self, comm, positions):
        """This rank's rows of the (P, d) batch on this GPU, then the swarm exchange
        (gpf_eval_batch_sharded): every rank returns the same (P,) scores, or raises the same
        error (LinAlgError for a non-PD particle on any rank)."""
        P = _f64(positions)
        if P.ndim == 1:
            P = P.reshape(1, -1)
        loss = np.empty(P.shape[0])
        bad = ctypes.c_int(-1)
        rc = self.lib.gpf_eval_batch_sharded(self._h, comm.handle, _ptr(P), P.shape[0], _ptr(loss), ctypes.byref(bad))
        self._check(rc, "gpf_eval_batch_sharded", bad)
        return loss

    def synchronize(self):
        """Device-wide fence (gpf_sync): all queued work on this context's GPU has finished."""
        self._check(self.lib.gpf_sync(self._h), "gpf_sync")

    def predict(self, lengths, x_fit, batch_size=10000):
        ls = _f64(lengths).reshape(-1)
        xf = _f64(x_fit)
        m = xf.shape[1]
        mu, sd = np.empty(m), np.empty(m)
        self._check(self.lib.gpf_predict(self._h, _ptr(ls), _ptr(xf), m, int(batch_size), _ptr(mu), _ptr(sd)),
                    "gpf_predict")
        return mu, sd

    def kernel(self, x1, x2, l):
        a, b = _f64(x1), _f64(x2)
        ls = _f64(l).reshape(-1)
        out = np.empty((a.shape[1], b.shape[1]))
        self._check(self.lib.gpf_kernel(self._h, _ptr(a), a.shape[1], _ptr(b), b.shape[1], a.shape[0],
                                        _ptr(ls), _ptr(out)), "gpf_kernel")
        return out

    def log_marginal_likelihood(self, lengths):
        ls = _f64(lengths).reshape(-1)
        out = ctypes.c_double(0.0)
        self._check(self.lib.gpf_log_marginal_likelihood(self._h, _ptr(ls), ctypes.byref(out)),
                    "gpf_log_marginal_likelihood")
        return out.value

    # -- measurement hooks --
    def set_profiling(self, on=True):
        self._check(self.lib.gpf_set_profiling(self._h, int(bool(on))), "gpf_set_profiling")

    def reset_profile(self):
        self._check(self.lib.gpf_reset_profile(self._h), "gpf_reset_profile")

    def profile(self):
        buf = np.zeros(27)
        self.lib.gpf_get_profile(self._h, _ptr(buf), 27)
        keys = ["panel_ms", "panel_launches", "panel_flops", "diag_ms", "diag_launches", "diag_flops",
                "build_ms", "build_launches", "build_bytes", "loss_ms", "loss_launches", "evals",
                "factor_wall_ms", "factor_calls", "factor_flops", "predict_ms", "predict_launches",
                "predict_flops", "predict_cov_ms", "predict_cov_launches", "predict_cov_bytes",
                "psurf_ms", "psurf_launches", "psurf_bytes", "factor_sclk_mhz", "cus", "fp64_ceiling_at_sclk_tflops"]
        return dict(zip(keys, buf.tolist()))

    def debug_factor(self, lengths):
        """(L, U, z, alpha) of one particle: Npad x Npad factor and inverse (diagnostic)."""
        ls = _f64(lengths).reshape(-1)
        t = self.lib.gpf_tile()
        npad = -(-self.N // t) * t
        L, U = np.empty((npad, npad)), np.empty((npad, npad))
        z, al = np.empty(npad), np.empty(self.N)
        rc = self.lib.gpf_debug_factor(self._h, _ptr(ls), _ptr(L), _ptr(U), _ptr(z), _ptr(al))
        if rc not in (GPF_OK, GPF_NOT_PD):
            self._check(rc, "gpf_debug_factor")
        return L, U, z, al

    def debug_factor128(self, a, y):
        """factor128 on n 128x128 blocks a[n,128,128] with right-hand sides y[n,128] (diagnostic):
        dict of L, U, z, s2, sz, bad, cycles (shader cycles per block)."""
        a = np.ascontiguousarray(a, dtype=np.float64).reshape(-1, 128, 128)
        n = a.shape[0]
        y = np.ascontiguousarray(y, dtype=np.float64).reshape(n, 128)
        L, U = np.empty_like(a), np.empty_like(a)
        z, s2, sz, cyc = np.empty((n, 128)), np.empty((n, 128)), np.empty((n, 128)), np.empty(n)
        bad = np.zeros(n, dtype=np.int32)
        self._check(self.lib.gpf_debug_factor128(self._h, _ptr(a), _ptr(y), n, _ptr(L), _ptr(U), _ptr(z), _ptr(s2),
                                                 _ptr(sz), bad.ctypes.data_as(_ip), _ptr(cyc)), "gpf_debug_factor128")
        return {"L": L, "U": U, "z": z, "s2": s2, "sz": sz, "bad": bad, "cycles": cyc}

    def mfma_peak(self, blocks=1024, iters=4096):
        out = ctypes.c_double(0.0)
        self._check(self.lib.gpf_mfma_peak(self._h, int(blocks), int(iters), ctypes.byref(out)), "gpf_mfma_peak")
        return out.value

    def bench_clock(self):
        """Shader clock (MHz) the last mfma_peak / gemm_bench held (gpf_bench_clock)."""
        out = ctypes.c_double(0.0)
        self._check(self.lib.gpf_bench_clock(self._h, ctypes.byref(out)), "gpf_bench_clock")
        return out.value

    def kmeans_set(self, X):
        """Keep the (n, d) centred points on the device for kmeans_step (gpf_kmeans_set)."""
        X = np.ascontiguousarray(X, dtype=np.float64)
        self._check(self.lib.gpf_kmeans_set(self._h, _ptr(X), X.shape[0], X.shape[1]), "gpf_kmeans_set")
        self._km_n = X.shape[0]

    def kmeans_step(self, centers, update=True, want_dist=False):
        """One Lloyd E-step (+ M-step sums) against centers (k, d) (gpf_kmeans_step):
        (labels, sums, counts, dist or None)."""
        C = np.ascontiguousarray(centers, dtype=np.float64)
        k, d = C.shape
        labels = np.empty(self._km_n, dtype=np.int32)
        sums = np.empty((k, d)) if update else None
        counts = np.empty(k) if update else None
        dist = np.empty(self._km_n) if want_dist else None
        nul = ctypes.POINTER(ctypes.c_double)()
        self._check(self.lib.gpf_kmeans_step(self._h, _ptr(C), k, int(bool(update)),
                                             labels.ctypes.data_as(ctypes.POINTER(ctypes.c_int)),
                                             _ptr(sums) if update else nul, _ptr(counts) if update else nul,
                                             _ptr(dist) if want_dist else nul), "gpf_kmeans_step")
        return labels, sums, counts, dist

    def prob_surface(self, tails):
        """(y (M,100), p (M,100), ok (M,) bool) for each row of tail entries (gpf_prob_surface)."""
        t = _f64(tails)
        if t.ndim != 2:
            raise ValueError("tails must be (M, E)")
        m, e = t.shape
        y, p = np.empty((m, 100)), np.empty((m, 100))
        ok = np.empty(m, dtype=np.int32)
        self._check(self.lib.gpf_prob_surface(self._h, _ptr(t), m, e, _ptr(y), _ptr(p),
                                              ok.ctypes.data_as(ctypes.POINTER(ctypes.c_int))), "gpf_prob_surface")
        return y, p, ok.astype(bool)

    def hull_fill(self, shell_rows, res, decimals):
        """The d sort + scan-fill passes of fill_convex_hull on the GPU (gpf_hull_fill): rows
        (m, d) sorted lexicographically."""
        rows = _f64(shell_rows)
        n, d = rows.shape
        r = _f64(res).reshape(-1)
        dec = np.ascontiguousarray(decimals, dtype=np.int32).reshape(-1)
        if r.shape[0] != d or dec.shape[0] != d:
            raise ValueError("res and decimals need one entry per dimension")
        m = ctypes.c_int64(0)
        self._check(self.lib.gpf_hull_fill(self._h, _ptr(rows), n, d, _ptr(r),
                                           dec.ctypes.data_as(ctypes.POINTER(ctypes.c_int)), ctypes.byref(m)),
                    "gpf_hull_fill")
        out = np.empty((m.value, d))
        self._check(self.lib.gpf_hull_fetch(self._h, _ptr(out)), "gpf_hull_fetch")
        return out

    def gemm_bench(self, mode=0, npad=4096, particles=64, tiles=15, depth=2048, iters=5):
        """TF/s of the block-column GEMM core alone (gpf_gemm_bench)."""
        out = ctypes.c_double(0.0)
        self._check(self.lib.gpf_gemm_bench(self._h, int(mode), int(npad), int(particles), int(tiles), int(depth),
                                            int(iters), ctypes.byref(out)), "gpf_gemm_bench")
        return out.value

    def selftest_mfma(self, a, b):
        a, b = _f64(a), _f64(b)
        c = np.empty((16, 16))
        self._check(self.lib.gpf_selftest_mfma(self._h, _ptr(a), _ptr(b), _ptr(c)), "gpf_selftest_mfma")
        return c


class Comm:
    """Rank `rank` of `nranks` in a swarm-exchange group (gpf_comm, include/gpfit.h).

    transport "rccl": ncclAllReduce on `ctx`'s GPU (one process per GPU); "host": the same
    exchange over the TCP rendezvous sockets (no device; CPU tests and tools).
    """

    def __init__(self, rank, nranks, host="127.0.0.1", port=29600, transport="rccl", ctx=None):
        self.lib = load_library()
        kind = {"rccl": GPF_COMM_RCCL, "host": GPF_COMM_HOST}[transport]
        if kind == GPF_COMM_RCCL and ctx is None:
            raise ValueError("the rccl transport needs the rank's Context")
        h = _vp()
        rc = self.lib.gpf_comm_open(ctx._h if ctx is not None else None, int(rank), int(nranks), host.encode(),
                                    int(port), kind, ctypes.byref(h))
        if rc != GPF_OK or not h.value:
            why = ctx.lib.gpf_last_error(ctx._h).decode(errors="replace") if ctx is not None else ""
            raise GPFitError(f"gpf_comm_open(rank={rank}, nranks={nranks}, {host}:{port}, {transport}) failed "
                             f"(rc={rc}) {why}")
        self.handle = h
        self.rank, self.size, self.transport = int(rank), int(nranks), transport

    @classmethod
    def from_env(cls, ctx=None, transport=None):
        """torchrun-style environment: RANK, WORLD_SIZE, MASTER_ADDR; the rendezvous port is
        GPF_COMM_PORT, else MASTER_PORT + 1 (MASTER_PORT itself is the launcher's store)."""
        rank = int(os.environ.get("RANK", "0"))
        world = int(os.environ.get("WORLD_SIZE", "1"))
        host = os.environ.get("MASTER_ADDR", "127.0.0.1")
        port = int(os.environ.get("GPF_COMM_PORT", int(os.environ.get("MASTER_PORT", "29599")) + 1))
        transport = transport or os.environ.get("GPF_COMM_TRANSPORT", "rccl" if ctx is not None else "host")
        return cls(rank, world, host, port, transport, ctx)

    def close(self):
        if getattr(self, "handle", None) is not None and self.handle.value:
            self.lib.gpf_comm_close(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _err(self):
        return self.lib.gpf_comm_last_error(self.handle).decode(errors="replace")

    def allreduce(self, values, op="sum"):
        buf = np.array(values, dtype=np.float64, copy=True).reshape(-1)
        rc = self.lib.gpf_comm_allreduce(self.handle, _ptr(buf), buf.shape[0],
                                         {"sum": GPF_OP_SUM, "max": GPF_OP_MAX}[op])
        if rc != GPF_OK:
            raise GPFitError(f"gpf_comm_allreduce: {self._err()}")
        return buf

    def barrier(self):
        self.allreduce(np.zeros(1))

    def stats(self):
        """(ms, count): cumulative wall time this rank spent in the score exchange
        (gpf_comm_exchange_scores: the all-reduce, including the wait for the slowest rank)."""
        ms = ctypes.c_double(0.0)
        n = ctypes.c_longlong(0)
        if self.lib.gpf_comm_stats(self.handle, ctypes.byref(ms), ctypes.byref(n)) != GPF_OK:
            raise GPFitError("gpf_comm_stats failed")
        return ms.value, n.value

    def rows(self, P):
        """This rank's contiguous rows [rP/G, (r+1)P/G) of a P-particle swarm."""
        return self.rank * P // self.size, (self.rank + 1) * P // self.size

    def exchange_scores(self, P, local, local_rc=GPF_OK, local_bad=-1):
        """gpf_comm_exchange_scores: this rank's scores of its rows -> the full (P,) vector on
        every rank; a non-PD particle on any rank raises LinAlgError on every rank."""
        loss = np.empty(P)
        loc = _f64(local) if local is not None else np.zeros(0)
        bad = ctypes.c_int(-1)
        rc = self.lib.gpf_comm_exchange_scores(self.handle, int(P), _ptr(loc), int(local_rc), int(local_bad),
                                               _ptr(loss), ctypes.byref(bad))
        if rc == GPF_NOT_PD:
            err = np.linalg.LinAlgError("Matrix is not positive definite")
            err.bad_index = bad.value  # the smallest failing row of the whole swarm
            raise err
        if rc == GPF_BAD_ARG:
            raise ValueError(f"gpf_comm_exchange_scores: {self._err()}")
        if rc != GPF_OK:
            raise GPFitError(f"gpf_comm_exchange_scores: {self._err()}")
        return loss


_DEFAULT = {}
_COMM = {}


def default_comm(ctx=None):
    """The process-wide swarm-exchange group when the launcher started several ranks
    (WORLD_SIZE > 1 in the environment), else None. Created on first use: RCCL on this
    process's GPU context, or the host transport when no context is given."""
    if int(os.environ.get("WORLD_SIZE", "1")) <= 1:
        return None
    key = "ctx" if ctx is not None else "host"
    if key not in _COMM:
        _COMM[key] = Comm.from_env(ctx)
    return _COMM[key]


def default_context():
    """Process-wide context on this process's GPU (created on first use)."""
    dev = default_device()
    ctx = _DEFAULT.get(dev)
    if ctx is None:
        ctx = Context(dev)
        _DEFAULT[dev] = ctx
    return ctx
