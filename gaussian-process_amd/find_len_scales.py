"""Drop-in for the reference's find_len_scales.py, computed on the MI355X.

Public surface of find_len_scales.py (rferguson22/Gaussian-Process):
    len_scale_opt(x_known, y_known, e_known, PSO_progress)        :22-150
    wass_loss(ls, x, y, e, sigma_vals, expected, lower, upper)     :154-177
    evaluate_loss(lengths, ...)                                    :181-182
    evaluate_loss_helper(args)                                     :186-188
    sigma_to_percent(x)                                            :192-201

Every objective evaluation runs in libgpfit (gpf_eval_batch): the reference's
fork pool over particles becomes one batched call per PSO iteration.
len_scale_opt keeps the reference defaults (40 particles, 500 iterations,
KMeans subsample above 100 points) and adds keyword-only overrides used by the
benchmarks and the tests: num_particles, max_iter, max_points,
init_positions, seed.
"""
import numpy as np

from gpfit._lib import default_context
from gpfit.swarm import particle_swarm
from gpfit.swarm import sigma_to_percent as _sigma_to_percent

__all__ = ["len_scale_opt", "wass_loss", "evaluate_loss", "evaluate_loss_helper", "sigma_to_percent"]


def len_scale_opt(x_known, y_known, e_known, PSO_progress, *, num_particles=40, max_iter=500,
                  max_points=100, init_positions=None, seed=None):
    """PSO search for the per-dimension length scales (find_len_scales.py:22-150)."""
    best, _ = particle_swarm(np.asarray(x_known, dtype=np.float64), np.asarray(y_known, dtype=np.float64),
                             np.asarray(e_known, dtype=np.float64), PSO_progress,
                             num_particles=num_particles, max_iter=max_iter, max_points=max_points,
                             init_positions=init_positions, seed=seed)
    return best


def wass_loss(ls, x_known, y_known, e_known, sigma_vals, expected_percents, lower_bounds, upper_bounds):
    """Negated calibration loss of one particle (find_len_scales.py:154-177)."""
    return -evaluate_loss(ls, x_known, y_known, e_known, sigma_vals, expected_percents,
                          lower_bounds, upper_bounds)


def evaluate_loss(lengths, x_known, y_known, e_known, sigma_vals, expected_percents, lower_bounds, upper_bounds):
    """find_len_scales.py:181-182: W + 0.01 * proximity, or 1e13 outside the box."""
    ctx = default_context()
    ctx.set_data(x_known, y_known, e_known)
    ctx.set_grid(sigma_vals, expected_percents, lower_bounds, upper_bounds)
    return float(ctx.eval_batch(np.asarray(lengths, dtype=np.float64).reshape(1, -1))[0])


def evaluate_loss_helper(args):
    """find_len_scales.py:186-188 (tuple-unpacking task body)."""
    return evaluate_loss(*args)


def sigma_to_percent(x):
    """Phi(x) - Phi(-x) (find_len_scales.py:192-201)."""
    return _sigma_to_percent(x)
