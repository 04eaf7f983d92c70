"""Drop-in for the reference's calc_prob_surf.py (host post-processing).

For every grid row, the finite (mean, sd) pairs of its experiments define an
equal-weight Gaussian mixture; its bin probabilities on 100 points spanning
[min(mu - 3 sd), max(mu + 3 sd)] are written as (x..., quantity, prob) rows.
Per-element operations and their order follow calc_prob_surf.py:15-30,67-81.
"""
import os

import numpy as np
import pandas as pd
import yaml
from scipy.stats import norm

__all__ = ["generate_prob_surf", "sum_gaussians"]

POINTS = 100


def sum_gaussians(temp_y, temp_gaus):
    """Mean probability mass of bins of width dy centred on temp_y under the
    Gaussians (mu_0, sd_0, mu_1, sd_1, ...) (calc_prob_surf.py:15-30)."""
    temp_y = np.asarray(temp_y)
    k = len(temp_gaus) // 2
    dy = abs(max(temp_y) - min(temp_y)) / len(temp_y)
    z = np.zeros(len(temp_y))
    for i in range(k):
        mu, sd = temp_gaus[2 * i], temp_gaus[2 * i + 1]
        z += norm.cdf(temp_y + dy / 2, loc=mu, scale=sd)
        z -= norm.cdf(temp_y - dy / 2, loc=mu, scale=sd)
    return z / k


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
    blocks = []
    for row in values:
        tail = row[ndims:]
        gaus = tail[np.isfinite(tail)]
        if len(gaus) < 2 or len(gaus) % 2:
            continue
        mus, sds = gaus[::2], gaus[1::2]
        y = np.linspace(min(mus - 3 * sds), max(mus + 3 * sds), POINTS)
        p = sum_gaussians(y, gaus)
        block = np.empty((POINTS, ndims + 2), dtype=object)
        block[:, :ndims] = row[:ndims]
        block[:, ndims] = y
        block[:, ndims + 1] = p
        blocks.append(block)
    cols = df.columns[:ndims].tolist() + ["quantity", "prob"]
    data = np.concatenate(blocks) if blocks else np.empty((0, ndims + 2))
    pd.DataFrame(data.tolist(), columns=cols).to_csv(output_file, index=False)
    print(f"Probability results written to {output_file}")
