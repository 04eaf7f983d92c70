"""Drop-in for the reference's read_in.py: options.yaml + input files (host I/O).

Input files are CSV with optional header: d kinematic columns, then (quantity,
error) pairs, one pair per experiment; rows whose pair is not finite are
dropped per experiment. Behaviour, messages and return shapes follow
read_in.py:16-254 (x is returned (d, N), as a transposed view).
"""
from pathlib import Path

import numpy as np
import pandas as pd
import yaml

__all__ = ["file_has_header", "expand_file_paths", "header_labels", "check_data", "read_yaml", "read_data",
           "read_csv"]


def _is_number(v):
    try:
        float(v)
    except (ValueError, TypeError):
        return False
    return True


def file_has_header(file_path):
    """True when some cell of the first row does not parse as a float (read_in.py:16-31)."""
    first = pd.read_csv(file_path, nrows=1, header=None).iloc[0]
    return not all(_is_number(v) for v in first)


def expand_file_paths(file_entries):
    """Files stay, folders expand to their sorted regular files (read_in.py:35-58)."""
    found = []
    for entry in file_entries:
        p = Path(entry)
        if p.is_file():
            found.append(str(p))
        elif p.is_dir():
            inside = sorted(str(q) for q in p.glob("*") if q.is_file())
            if not inside:
                raise ValueError(f"The folder '{entry}' is empty or contains no readable files.")
            found.extend(inside)
        else:
            raise ValueError(f"'{entry}' is not a valid file or directory.")
    if not found:
        raise ValueError("No valid input files found. Please check 'file_name' entries.")
    return found


def header_labels(file_paths, num_kin_dims):
    """Kinematic labels shared (case/space-insensitively) by every headed file, else None
    (read_in.py:62-100)."""
    raw, norm = [], []
    for fp in file_paths:
        try:
            if not file_has_header(fp):
                continue
            cols = list(pd.read_csv(fp, nrows=0, header=0).columns)
        except Exception:
            continue
        if len(cols) < num_kin_dims:
            print(f"  File '{fp}' has insufficient header columns ({len(cols)}), skipping.")
            continue
        raw.append(cols[:num_kin_dims])
        norm.append([c.strip().lower() for c in cols[:num_kin_dims]])
    if not norm:
        return None
    if any(n != norm[0] for n in norm[1:]):
        print("Warning: File header labels are inconsistent across files.")
        return None
    return raw[0]


def read_csv(file_path):
    """CSV with or without a header row (read_in.py:243-254)."""
    return pd.read_csv(file_path, header=0 if file_has_header(file_path) else None)


def read_data(file_path, labels, resolution):
    """Per-experiment (x (d, N_valid), (y, e)) from one file (read_in.py:204-239)."""
    table = read_csv(file_path)
    nd = len(resolution)
    extra = table.shape[1] - nd
    if extra % 2 != 0:
        raise ValueError(f"File '{file_path}' must have pairs of columns for quantity and error after kinematic dimensions.")
    vals = table.values
    xs, pairs = [], []
    for k in range(extra // 2):
        y = vals[:, nd + 2 * k]
        e = vals[:, nd + 2 * k + 1]
        keep = np.isfinite(y) & np.isfinite(e)
        xs.append(vals[:, :nd].T[:, keep])
        pairs.append((y[keep], e[keep]))
    return xs, pairs, labels


def check_data(file_paths, resolution, labels):
    """Load every file and check its kinematic dimension (read_in.py:104-130)."""
    out = []
    for fp in file_paths:
        try:
            xs, pairs, labels_out = read_data(fp, labels, resolution)
            for x in xs:
                if len(resolution) != x.shape[0]:
                    raise ValueError(f"File '{fp}' appears to have kinematic dimension {x.shape[0]}, "
                                     f"but resolution list has {len(resolution)} elements.")
            out.append((fp, xs, pairs, labels_out))
        except Exception as err:
            raise ValueError(f"Failed to load file '{fp}': {err}")
    print("All datafile paths are readable.")
    return out


def read_yaml():
    """Parse ./options.yaml and load the data it names (read_in.py:134-200).

    Returns (resolution, PSO_progress, out_file_name, labels, data_list,
    write_individual_files, group_experiments_per_file).
    """
    with open("options.yaml", "r") as f:
        opts = yaml.safe_load(f)
    entries = opts["file_name"]
    resolution = opts["resolution"]
    progress = opts.get("PSO_progress", False)
    out_name = opts.get("out_file_name", None)
    labels = opts.get("labels", None)
    individual = opts.get("write_individual_files", False)
    grouped = opts.get("group_experiments_per_file", False)

    if not isinstance(entries, list):
        raise ValueError("Expected 'file_name' to be a list of file paths or folder paths.")
    paths = expand_file_paths(entries)
    data = check_data(paths, resolution, labels)
    if not all(isinstance(r, (float, int)) for r in resolution):
        raise ValueError("All resolution values must be floats or integers.")

    if out_name is None:
        out_name = "GP_results.txt"
    out_path = Path(out_name)
    if individual:
        if not out_path.exists():
            print(f"Output folder '{out_path}' does not exist — creating it.")
            out_path.mkdir(parents=True, exist_ok=True)
        elif out_path.is_file():
            print(f"Warning: Individual file output requested, but out_file_name points to a file."
                  "Will write a single combined output file: {out_file_name}")
            individual = False
    elif out_path.is_dir():
        out_name = str(out_path / "GP_results.txt")

    nd = len(resolution)
    print(f"Number of Kinematic Dimensions: {nd}")
    if labels is not None:
        if len(labels) == nd:
            kin = labels
            print(f"Using kinematic dimension labels from options.yaml: {kin}")
        else:
            kin = [f"dim{i+1}" for i in range(nd)]
            print(f"Warning: The number of kinematic dimension labels ({len(labels)}) does not match the expected number "
                  f"({nd}). Using generic kinematic dimension labels instead: {kin}")
    else:
        inferred = header_labels(paths, nd)
        if inferred is not None:
            kin = inferred
            print(f"Using kinematic dimension labels from file headers: {kin}")
        else:
            kin = [f"dim{i+1}" for i in range(nd)]
            print(f"Using generic kinematic dimension labels: {kin}")

    return resolution, progress, str(out_name), kin + ["quantity", "error"], data, individual, grouped
