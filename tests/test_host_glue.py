"""Host-side drop-in modules (read_in, convex_hull, calc_prob_surf, GP_fit, main)
against fixtures captured from the reference (tests/golden/make_golden.py)."""
import os
import shutil
from pathlib import Path

import numpy as np
import pandas as pd
import pytest

from conftest import GOLDEN, load_golden

INPUTS = GOLDEN / "inputs"


def test_fill_convex_hull_matches_reference_grids():
    from convex_hull import fill_convex_hull
    f6 = load_golden("f6_hull.npz")
    for i in range(int(f6["ncases"])):
        pts, res = f6[f"c{i}_points"], list(f6[f"c{i}_res"])
        got = fill_convex_hull(pts, res)
        want = f6[f"c{i}_grid"]
        assert got.shape == want.shape, i
        assert np.array_equal(got, want), i


def test_round_to_res_quirks():
    from convex_hull import round_to_res
    assert round_to_res(0.125, 0.01) == 0.12  # round half to even on value/res
    assert round_to_res(1.2349, 0.25) == 1.25
    assert round_to_res(7.0, 2) == 8


def test_prob_surface_matches_reference(tmp_path):
    from calc_prob_surf import generate_prob_surf
    f7 = load_golden("f7_prob_surf.npz")
    df = pd.DataFrame(f7["frame"], columns=[str(c) for c in f7["columns"]])
    out = tmp_path / "ps.txt"
    opt = tmp_path / "options.yaml"
    opt.write_text(f"out_file_name: '{out}'\n")
    generate_prob_surf(df, 2, options_path=str(opt))
    got = pd.read_csv(out)
    assert list(got.columns) == [str(c) for c in f7["out_columns"]]
    np.testing.assert_array_equal(got.values, f7["out"])


def test_read_in_matches_reference_loader(f2, tmp_path, monkeypatch):
    import read_in
    shutil.copytree(INPUTS, tmp_path / "in")
    monkeypatch.chdir(tmp_path / "in")
    Path("options.yaml").write_text('file_name: ["Test_file1.txt", "Test_folder"]\nresolution: [0.01, 0.01]\n'
                                    'out_file_name: "out/"\nwrite_individual_files: true\n'
                                    'group_experiments_per_file: true\n')
    res, prog, out, labels, data, ind, grp = read_in.read_yaml()
    assert labels == ["energy", "angle", "quantity", "error"] and ind and grp and prog is False
    got = [(x, y, e) for _, xs, pairs, _ in data for x, (y, e) in zip(xs, pairs)]
    assert len(got) == int(f2["ncases"])
    for i, (x, y, e) in enumerate(got):
        assert np.array_equal(x, f2[f"c{i}_x"]) and x.flags["F_CONTIGUOUS"]
        assert np.array_equal(y, f2[f"c{i}_y"]) and np.array_equal(e, f2[f"c{i}_e"])


def test_read_in_errors(tmp_path):
    import read_in
    with pytest.raises(ValueError, match="not a valid file or directory"):
        read_in.expand_file_paths([str(tmp_path / "missing.txt")])
    (tmp_path / "empty").mkdir()
    with pytest.raises(ValueError, match="is empty"):
        read_in.expand_file_paths([str(tmp_path / "empty")])
    bad = tmp_path / "bad.txt"
    bad.write_text("1,2,3\n4,5,6\n")
    with pytest.raises(ValueError, match="Failed to load file"):
        read_in.check_data([str(bad)], [0.1, 0.1], None)


@pytest.mark.gpu
def test_main_end_to_end_on_gpu(f4, tmp_path, monkeypatch, capsys):
    """`python main.py` flow on the bundled inputs: PSO + hull grid + GP on the GPU,
    grouped per-file outputs named and laid out like the committed reference outputs."""
    import main as dropin_main
    from oracle import ref_cpu
    shutil.copytree(INPUTS, tmp_path / "run")
    monkeypatch.chdir(tmp_path / "run")
    Path("options.yaml").write_text('file_name: ["Test_file1.txt","Test_folder"]\nresolution: [0.01, 0.01]\n'
                                    'gp_fit: true\nrun_prob_surf: true\nout_file_name: "output_folder/"\n'
                                    'labels: ["Plab", "cosTheta"]\nPSO_progress: false\nwrite_individual_files: true\n'
                                    'group_experiments_per_file: true\npso_seed: 3\npso_max_iter: 60\n')
    dropin_main.main()
    capsys.readouterr()
    f6 = load_golden("f6_hull.npz")
    headers = {"Test_file1": "Plab,cosTheta,Test_file1,Test_file1_unc",
               "Test_file2": "Plab,cosTheta,Test_file2,Test_file2_unc",
               "Test_file3": "Plab,cosTheta,Test_file3_exp1,Test_file3_unc1,Test_file3_exp2,Test_file3_unc2"}
    for stem, hdr in headers.items():
        path = Path("output_folder") / f"{stem}_GP_results.txt"
        assert path.read_text().splitlines()[0] == hdr
        df = pd.read_csv(path)
        assert np.all(np.isfinite(df.iloc[:, 2].values[np.isfinite(df.iloc[:, 2].values)]))
    # grids equal the reference's hull grids; values equal GP at the found scales
    df1 = pd.read_csv("output_folder/Test_file1_GP_results.txt")
    assert np.array_equal(df1.iloc[:, :2].values, f6["c0_grid"])
    assert Path("output_folder/prob_surf.txt").exists()
