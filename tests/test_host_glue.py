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


def test_hull_oracle_matches_reference_grids():
    """The host restatement (checker of gpf_hull_fill) reproduces the reference's grids F6."""
    from oracle.ref_hull import fill_convex_hull
    f6 = load_golden("f6_hull.npz")
    for i in range(int(f6["ncases"])):
        pts, res = f6[f"c{i}_points"], list(f6[f"c{i}_res"])
        got = fill_convex_hull(pts, res)
        want = f6[f"c{i}_grid"]
        assert got.shape == want.shape, i
        assert np.array_equal(got, want), i


@pytest.mark.gpu
def test_fill_convex_hull_on_gpu_matches_reference_grids():
    """fill_convex_hull with the fill passes on the MI355X: the reference's grids F6 point for
    point, same order (2-D and 3-D cases)."""
    from convex_hull import fill_convex_hull
    f6 = load_golden("f6_hull.npz")
    for i in range(int(f6["ncases"])):
        pts, res = f6[f"c{i}_points"], list(f6[f"c{i}_res"])
        got = fill_convex_hull(pts, res)
        want = f6[f"c{i}_grid"]
        assert got.shape == want.shape, i
        assert np.array_equal(got, want), i


@pytest.mark.gpu
def test_fill_convex_hull_on_gpu_matches_oracle_off_grid():
    """Off-grid hull vertices (raw values that round_to_res moves, resolutions >= 1 and with
    different decimals, 3-D and 4-D): GPU fill == host restatement."""
    from convex_hull import fill_convex_hull
    from oracle.ref_hull import fill_convex_hull as ref_fill
    rng = np.random.default_rng(5)
    for d, res in [(2, [0.05, 0.1]), (2, [0.25, 2.0]), (3, [0.1, 0.2, 0.15]), (4, [0.5, 0.5, 0.5, 0.5])]:
        pts = rng.uniform(-1.3, 2.7, size=(12, d)) * np.array([1, 2, 1, 3][:d])
        got = fill_convex_hull(pts, res)
        want = ref_fill(pts, res)
        assert got.shape == want.shape, (d, res)
        assert np.array_equal(got, want), (d, res)


def test_round_to_res_quirks():
    from convex_hull import round_to_res
    assert round_to_res(0.125, 0.01) == 0.12  # round half to even on value/res
    assert round_to_res(1.2349, 0.25) == 1.25
    assert round_to_res(7.0, 2) == 8


def test_host_rasterisation_matches_oracle():
    """The drop-in's facet rasterisation (Python-float walks, scalar trim instead of np.around)
    against the oracle's numpy-scalar restatement (oracle/ref_hull.py, pinned to the
    reference's grids F6): round_to_res on random values and exact ties, and every facet's
    shell of random off-grid hulls in 2-4 dimensions, bit for bit and in the same order."""
    from scipy.spatial import ConvexHull
    import convex_hull as ch
    from oracle import ref_hull as rh
    rng = np.random.default_rng(29)
    resolutions = [0.005, 0.01, 0.02, 0.25, 0.1, 1e-05, 0.3, 1.0, 2.0, 0.125]
    for r in resolutions:
        vals = np.concatenate([rng.uniform(-3, 3, 200), (np.arange(-20, 20) + 0.5) * r,
                               rng.integers(-50, 50, 40) * r, [0.0, -0.0]])
        for v in vals:
            got, want = ch.round_to_res(v, r), rh.round_to_res(v, r)
            assert got == want and np.signbit(got) == np.signbit(want), (v, r)
    cases = [(2, 15, [0.005, 0.01]), (2, 9, [0.25, 0.1]), (3, 10, [0.02, 0.05, 0.04]),
             (3, 8, [0.1, 0.3, 0.2]), (4, 9, [0.1, 0.2, 0.25, 0.1]), (2, 7, [1.0, 2.0])]
    for d, n, res in cases:
        pts = rng.uniform(-1.0, 2.0, size=(n, d)) * (np.max(res) * 20 if max(res) >= 1 else 1.0)
        res = np.asarray(res)
        for simplex in ConvexHull(pts).simplices:
            corners = pts[list(simplex)]
            got, want = ch._facet_surface(corners, res), rh._facet_surface(corners, res)
            assert got.shape == want.shape and np.array_equal(got, want), (d, n, list(res))


def test_prob_surface_oracle_matches_reference(tmp_path):
    """The host restatement (checker of the GPU kernel), written through the same object-frame
    to_csv as calc_prob_surf.py:84-86, equals the reference's output file F7 bit for bit."""
    from oracle import ref_cpu
    f7 = load_golden("f7_prob_surf.npz")
    rows, ys, ps = ref_cpu.prob_surface(f7["frame"], 2)
    data = np.empty((len(rows) * 100, 4), dtype=object)
    data[:, :2] = np.repeat(f7["frame"][rows, :2], 100, axis=0)
    data[:, 2] = ys.reshape(-1)
    data[:, 3] = ps.reshape(-1)
    pd.DataFrame(data.tolist(), columns=[str(c) for c in f7["out_columns"]]).to_csv(tmp_path / "o.csv", index=False)
    np.testing.assert_array_equal(pd.read_csv(tmp_path / "o.csv").values, f7["out"])


@pytest.mark.gpu
def test_prob_surface_on_gpu_matches_reference(tmp_path):
    """generate_prob_surf (k_prob_surf on the MI355X) vs the reference's output F7: same rows,
    columns and grid (bitwise: same linspace arithmetic), probabilities to 1e-12 (erf/erfc are
    not scipy's implementations)."""
    from calc_prob_surf import generate_prob_surf, sum_gaussians
    f7 = load_golden("f7_prob_surf.npz")
    df = pd.DataFrame(f7["frame"], columns=[str(c) for c in f7["columns"]])
    out = tmp_path / "ps.txt"
    opt = tmp_path / "options.yaml"
    opt.write_text(f"out_file_name: '{out}'\n")
    generate_prob_surf(df, 2, options_path=str(opt))
    got = pd.read_csv(out)
    assert list(got.columns) == [str(c) for c in f7["out_columns"]]
    ref = f7["out"]
    assert got.values.shape == ref.shape
    np.testing.assert_array_equal(got.values[:, :3], ref[:, :3])
    np.testing.assert_allclose(got.values[:, 3], ref[:, 3], rtol=1e-12, atol=1e-15)
    # the scalar helper on one row, and its argument checks
    row = next(r for r in f7["frame"] if np.isfinite(r[2:]).sum() >= 2 and np.isfinite(r[2:]).sum() % 2 == 0)
    gaus = row[2:][np.isfinite(row[2:])]
    y = np.linspace(min(gaus[::2] - 3 * gaus[1::2]), max(gaus[::2] + 3 * gaus[1::2]), 100)
    from oracle import ref_cpu
    np.testing.assert_allclose(sum_gaussians(y, gaus), ref_cpu.sum_gaussians(y, gaus), rtol=1e-12, atol=1e-15)
    with pytest.raises(ValueError):
        sum_gaussians(y[:50], gaus)


@pytest.mark.gpu
def test_prob_surface_on_gpu_edge_rows():
    """Skipped rows (no finite pair, odd count), misaligned compaction, a single Gaussian, zero span."""
    import gpfit
    from oracle import ref_cpu
    inf = np.inf
    tails = np.array([[0.5, 0.1, inf, inf],      # one experiment
                      [inf, inf, inf, inf],      # nothing finite: skipped
                      [0.5, inf, 0.7, 0.2],      # odd count: skipped
                      [0.5, 0.1, 0.7, 0.2],      # two experiments
                      [inf, 0.3, 0.4, inf],      # compaction pairs (0.3, 0.4)
                      [1e3, 1e-3, -2.0, 5.0]])   # wide span
    vals = np.concatenate([np.zeros((len(tails), 2)), tails], axis=1)
    rows, ys, ps = ref_cpu.prob_surface(vals, 2)
    y, p, ok = gpfit.default_context().prob_surface(tails)
    assert list(np.nonzero(ok)[0]) == list(rows)
    np.testing.assert_array_equal(y[ok], ys)
    np.testing.assert_allclose(p[ok], ps, rtol=1e-12, atol=1e-15)


@pytest.mark.gpu
@pytest.mark.parametrize("keep_mb", ["2048", "0"])
def test_prob_surface_buffer_reuse(monkeypatch, keep_mb):
    """The row-chunk buffers kept between calls (grow-only; freed after the call above
    GPF_PREDICT_KEEP_MB): a small call, a larger one with a wider tail, then the small one again
    all equal fresh-context results bit for bit, and the oracle to 1e-12."""
    import gpfit
    from oracle import ref_cpu
    monkeypatch.setenv("GPF_PREDICT_KEEP_MB", keep_mb)
    rng = np.random.default_rng(7)

    def frame(m, E):
        t = np.empty((m, E))
        t[:, 0::2] = rng.normal(size=(m, E // 2))
        t[:, 1::2] = rng.uniform(0.05, 0.5, size=(m, E // 2))
        t[rng.uniform(size=m) < 0.2, E - 2:] = np.inf
        t[rng.uniform(size=m) < 0.05, 1] = np.nan  # odd count: skipped
        return t

    small, big = frame(300, 4), frame(5000, 8)
    ctx = gpfit.Context(0)
    try:
        runs = [ctx.prob_surface(small), ctx.prob_surface(big), ctx.prob_surface(small)]
    finally:
        ctx.close()
    fresh = []
    for t in (small, big):
        c2 = gpfit.Context(0)
        try:
            fresh.append(c2.prob_surface(t))
        finally:
            c2.close()
    for got, ref in zip(runs, [fresh[0], fresh[1], fresh[0]]):
        np.testing.assert_array_equal(got[2], ref[2])  # (skipped rows' y, p are not written)
        np.testing.assert_array_equal(got[0][got[2]], ref[0][ref[2]])
        np.testing.assert_array_equal(got[1][got[2]], ref[1][ref[2]])
    y, p, ok = runs[1]
    rows, ys, ps = ref_cpu.prob_surface(np.concatenate([np.zeros((len(big), 2)), big], axis=1), 2)
    assert 0 < len(rows) < len(big)
    assert list(np.nonzero(ok)[0]) == list(rows)
    np.testing.assert_array_equal(y[ok], ys)
    np.testing.assert_allclose(p[ok], ps, rtol=1e-12, atol=1e-15)


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
