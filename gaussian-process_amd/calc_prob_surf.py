"""Drop-in for the reference's calc_prob_surf.py, computed on the MI355X.

For every grid row, the finite (mean, sd) pairs of its experiments define an
equal-weight Gaussian mixture; its bin probabilities on 100 points spanning
[min(mu - 3 sd), max(mu + 3 sd)] are written as (x..., quantity, prob) rows.
The per-row arithmetic runs in `k_prob_surf` (gpf_prob_surface, csrc/gpf_probsurf.hip,
following calc_prob_surf.py:15-30,67-81 operation by operation); output naming,
skipping rules and the CSV layout follow calc_prob_surf.py:39-88.
"""
import os

import numpy as np
import pandas as pd
import yaml

from gpfit import default_context

__all__ = ["generate_prob_surf", "sum_gaussians"]

POINTS = 100


def sum_gaussians(temp_y, temp_gaus):
    """Mean probability mass of bins of width dy centred on temp_y under the Gaussians
    (mu_0, sd_0, mu_1, sd_1, ...) (calc_prob_surf.py:15-30). temp_y must be the row's
    100-point grid (as the reference always calls it); computed on the GPU."""
    temp_y = np.asarray(temp_y, dtype=np.float64)
    if temp_y.shape != (POINTS,):
        raise ValueError(f"temp_y must hold the row's {POINTS}-point grid")
    gaus = np.asarray(temp_gaus, dtype=np.float64).reshape(1, -1)
    y, p, ok = default_context().prob_surface(gaus)
    if not ok[0]:
        raise ValueError("temp_gaus must hold (mu, sd) pairs")
    if not np.array_equal(y[0], temp_y):  # a grid of another span: not the reference's call pattern
        raise ValueError("temp_y is not numpy.linspace(min(mu - 3 sd), max(mu + 3 sd), 100)")
    return p[0]


def _output_path(options_path):
    out = "prob_surf.txt"
    if os.path.exists(options_path):
        with open(options_path, "r") as f:
            opts = yaml.safe_load(f) or {}
        target = opts.get("out_file_name", "").strip()
        if target:
            out = os.path.join(target, "prob_surf.txt") if os.path.isdir(target) else target
    return out


def generate_prob_surf(df, ndims, options_path="options.yaml"):
    """Probability surface of a merged GP results frame, written to CSV
    (calc_prob_surf.py:39-88; output location from options.yaml out_file_name)."""
    print("Calculating Probability")
    output_file = _output_path(options_path)
    values = df.to_numpy()
    tails = np.ascontiguousarray(values[:, ndims:], dtype=np.float64)
    ys, ps, ok = default_context().prob_surface(tails)
    keep = np.nonzero(ok)[0]
    cols = df.columns[:ndims].tolist() + ["quantity", "prob"]
    data = np.empty((len(keep) * POINTS, ndims + 2), dtype=object)
    if len(keep):
        data[:, :ndims] = np.repeat(values[keep, :ndims], POINTS, axis=0)
        data[:, ndims] = ys[keep].reshape(-1)
        data[:, ndims + 1] = ps[keep].reshape(-1)
    pd.DataFrame(data.tolist(), columns=cols).to_csv(output_file, index=False)
    print(f"Probability results written to {output_file}")
