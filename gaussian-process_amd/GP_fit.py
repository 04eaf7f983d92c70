"""Drop-in for the reference's GP_fit.py: per-experiment fit + prediction + CSV writers.

Orchestration stays on the host; the two calls that matter
run on the MI355X: len_scale_opt (batched PSO objective, gpf_eval_batch) and GP on
the hull grid (gpf_predict). Column naming, file naming, merge semantics and
messages follow GP_fit.py:20-164.

Optional options.yaml keys (absent = reference behaviour): pso_num_particles (40),
pso_max_iter (500), pso_max_points (100), pso_seed (none: unseeded global RNG).
"""
from functools import reduce
from pathlib import Path

import pandas as pd
import yaml

from convex_hull import fill_convex_hull
from find_len_scales import len_scale_opt
from GP_func import GP
from read_in import read_yaml

__all__ = ["process_experiment", "write_individual_file", "write_grouped_file", "write_combined_file",
           "create_GP"]

_PSO_KEYS = {"pso_num_particles": "num_particles", "pso_max_iter": "max_iter", "pso_max_points": "max_points",
             "pso_seed": "seed"}


def _pso_overrides(options_path="options.yaml"):
    try:
        with open(options_path, "r") as f:
            opts = yaml.safe_load(f) or {}
    except OSError:
        return {}
    return {kw: opts[key] for key, kw in _PSO_KEYS.items() if opts.get(key) is not None}


def _merge(frames, on):
    return reduce(lambda a, b: pd.merge(a, b, on=on, how="outer"), frames).fillna(float("inf"))


def process_experiment(x_known, y_known, e_known, resolution, dim_labels, filename, exp_idx, total_exps,
                       PSO_progress, **pso):
    """Length scales by PSO, hull grid, GP prediction -> DataFrame (GP_fit.py:20-46)."""
    if x_known.shape[1] == 0:
        print("  Skipping experiment: no valid data points")
        return None
    ls = len_scale_opt(x_known, y_known, e_known, PSO_progress, **pso)
    grid = fill_convex_hull(x_known.T, resolution)
    mu, sd = GP(x_known, y_known, e_known, grid.T, ls)
    frame = pd.DataFrame(grid, columns=dim_labels)
    if total_exps == 1:
        qcol, ecol = f"{filename}", f"{filename}_unc"
    else:
        qcol, ecol = f"{filename}_exp{exp_idx}", f"{filename}_unc{exp_idx}"
    frame[qcol] = mu.flatten()
    frame[ecol] = sd.flatten()
    return frame


def write_individual_file(df, filename, out_path, total_exps, exp_idx):
    """One experiment per file (GP_fit.py:50-66)."""
    folder = out_path if out_path.is_dir() else out_path.parent
    folder.mkdir(parents=True, exist_ok=True)
    name = f"{filename}_GP_results.txt" if total_exps == 1 else f"{filename}_exp{exp_idx}_GP_results.txt"
    target = folder / name
    df.to_csv(target, index=False)
    print(f"Written individual output file: {target}")


def write_grouped_file(file_dfs, filename, out_path, dim_labels):
    """All experiments of one input file merged on the grid (GP_fit.py:70-85)."""
    folder = out_path if out_path.is_dir() else out_path.parent
    folder.mkdir(parents=True, exist_ok=True)
    target = folder / f"{filename}_GP_results.txt"
    _merge(file_dfs, dim_labels).to_csv(target, index=False)
    print(f"Written grouped output file: {target}")


def write_combined_file(experiment_dfs, out_path, dim_labels):
    """Every experiment merged into one file (GP_fit.py:89-108)."""
    if str(out_path).endswith("/"):
        out_path.mkdir(parents=True, exist_ok=True)
        target = out_path / "GP_results.txt"
    else:
        target = out_path
        target.parent.mkdir(parents=True, exist_ok=True)
    merged = _merge(experiment_dfs, dim_labels)
    merged.to_csv(target, index=False)
    print(f"Combined results written to {target}")
    return merged


def create_GP():
    """Fit every experiment of every configured file and write the outputs (GP_fit.py:112-164).

    Returns (merged DataFrame, number of kinematic dimensions).
    """
    resolution, progress, out_name, labels, data_list, write_ind, group_exps = read_yaml()
    pso = _pso_overrides()
    nd = len(resolution)
    dim_labels = labels[:nd]
    out_path = Path(out_name) if out_name else Path("GP_results.txt")

    if write_ind:
        print("Writing individual output files")
        print("Writing experiments from the same file together" if group_exps
              else "Writing experiments from the same file separately")
    else:
        print("Writing combined output file")

    all_dfs = []
    for file_idx, (file_path, xs, pairs, _labels) in enumerate(data_list, start=1):
        stem = Path(file_path).stem
        n_exp = len(xs)
        file_dfs = []
        for idx, (x, (y, e)) in enumerate(zip(xs, pairs), start=1):
            print(f"Processing experiment {idx}/{n_exp} from file {file_idx}/{len(data_list)}: {stem}")
            df = process_experiment(x, y, e, resolution, dim_labels, stem, idx, n_exp, progress, **pso)
            if df is None:
                continue
            all_dfs.append(df)
            file_dfs.append(df)
            if write_ind and not group_exps:
                write_individual_file(df, stem, out_path, n_exp, idx)
        if write_ind and group_exps and file_dfs:
            write_grouped_file(file_dfs, stem, out_path, dim_labels)

    if not write_ind and all_dfs:
        return write_combined_file(all_dfs, out_path, dim_labels), nd
    if all_dfs:
        return _merge(all_dfs, dim_labels), nd
    print("No experiment data to return")
    return pd.DataFrame(), nd
