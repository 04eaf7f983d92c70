"""Drop-in for the reference's main.py: `python main.py` in a directory holding options.yaml.

gp_fit: true  -> create_GP() (PSO + prediction on the MI355X)
gp_fit: false -> reload precomputed GP result files and merge them
run_prob_surf (default true, main.py:67) -> generate_prob_surf on the merged frame
Flow and messages follow main.py:20-101.
"""
import os
import sys
from functools import reduce
from pathlib import Path

# the drop-in modules sit next to this file; keep them ahead of any other tree on sys.path
_HERE = os.path.dirname(os.path.abspath(__file__))
if sys.path[0] != _HERE:
    sys.path.insert(0, _HERE)

import pandas as pd  # noqa: E402
import yaml  # noqa: E402

from calc_prob_surf import generate_prob_surf  # noqa: E402
from GP_fit import create_GP  # noqa: E402
from read_in import check_data, expand_file_paths  # noqa: E402

__all__ = ["load_and_merge_gp_results", "main_gp_flow", "main"]


def load_and_merge_gp_results(file_entries, resolution, labels):
    """Reload GP result files and merge them on the grid (main.py:20-52)."""
    data_list = check_data(expand_file_paths(file_entries), resolution, labels)
    if not data_list:
        print("No files loaded.")
        return pd.DataFrame(), len(resolution)
    dim_labels = None
    frames = []
    for file_path, xs, pairs, labels_out in data_list:
        if dim_labels is None:
            dim_labels = labels_out[:len(resolution)]
        for k, (x, (y, e)) in enumerate(zip(xs, pairs), start=1):
            df = pd.DataFrame(x.T, columns=dim_labels)
            q = f"{Path(file_path).stem}_exp{k}"
            df[q] = y
            df[f"{q}_unc"] = e
            frames.append(df)
    merged = reduce(lambda a, b: pd.merge(a, b, on=dim_labels, how="outer"), frames).fillna(float("inf"))
    print("All GP results loaded and merged.")
    return merged, len(resolution)


def main_gp_flow():
    """Fit (or reload) per options.yaml in the working directory (main.py:57-77)."""
    with open("options.yaml", "r") as f:
        opts = yaml.safe_load(f)
    if opts.get("gp_fit", True):
        df, nd = create_GP()
    else:
        df, nd = load_and_merge_gp_results(opts["file_name"], opts["resolution"], opts.get("labels", None))
    return df, nd, opts.get("run_prob_surf", True)


def main():
    """Entry point (main.py:81-94)."""
    df, nd, run_prob_surf = main_gp_flow()
    if run_prob_surf:
        print("Generating probability surface...")
        generate_prob_surf(df, nd)
    else:
        print("Skipping probability surface generation as per options.yaml")


if __name__ == "__main__":
    main()
