"""Pin the CPU oracle against the reference's golden vectors (no GPU).

The fixtures were produced by executing the reference itself
(tests/golden/make_golden.py); the oracle must reproduce them bit for bit,
because it issues the same NumPy/LAPACK calls in the same order.
"""
import numpy as np
import pytest

from oracle import ref_cpu


def _fx(x):
    # read_in.py:229 hands the reference a transposed (F-order) view; keep the
    # same layout so BLAS takes the same path.
    return np.asfortranarray(x)


def test_sigma_grid_matches_fixture(f2):
    s, ex = ref_cpu.sigma_grid()
    assert np.array_equal(s, f2["sigma_vals"])
    assert np.array_equal(ex, f2["expected"])


def test_gp_bitwise_vs_reference(f1):
    for i in range(int(f1["ncases"])):
        x, y, e, ls = _fx(f1[f"c{i}_x"]), f1[f"c{i}_y"], f1[f"c{i}_e"], f1[f"c{i}_ls"]
        xfit = f1[f"c{i}_xfit"]
        mu, sd = ref_cpu.GP(x, y, e, xfit, ls)
        assert np.array_equal(mu, f1[f"c{i}_mu"]), i
        assert np.array_equal(sd, f1[f"c{i}_sd"]), i
        mu7, sd7 = ref_cpu.GP(x, y, e, xfit, ls, batch_size=7)
        assert np.array_equal(mu7, f1[f"c{i}_mu_b7"]), i
        assert np.array_equal(sd7, f1[f"c{i}_sd_b7"]), i


def test_gp_matches_committed_outputs(f1):
    """The reference's own committed output files (output_folder/, output_file)."""
    for i in range(int(f1["ncases"])):
        n = int(f1[f"c{i}_ntrain"])
        mu, sd = f1[f"c{i}_mu"][n:], f1[f"c{i}_sd"][n:]
        cm, cs = f1[f"c{i}_committed_mu"], f1[f"c{i}_committed_sd"]
        assert np.max(np.abs(mu - cm) / np.maximum(np.abs(cm), 1e-3)) < 1e-9
        assert np.max(np.abs(sd - cs) / cs) < 1e-9


def test_identity_formulation_matches_reference(f1, f3):
    """The GPU's exact identity (mu = y - e^2 alpha, var = e^2 - e^4 diag K^-1)."""
    for i in range(int(f1["ncases"])):
        x, y, e, ls = _fx(f1[f"c{i}_x"]), f1[f"c{i}_y"], f1[f"c{i}_e"], f1[f"c{i}_ls"]
        n = x.shape[1]
        mu, sd = ref_cpu.GP_train_identity(x, y, e, ls)
        np.testing.assert_allclose(mu, f1[f"c{i}_mu"][:n], rtol=1e-9, atol=1e-12)
        np.testing.assert_allclose(sd, f1[f"c{i}_sd"][:n], rtol=1e-8)
    for i in range(int(f3["ncases"])):
        x, y, e, P = f3[f"c{i}_x"], f3[f"c{i}_y"], f3[f"c{i}_e"], f3[f"c{i}_P"]
        mu, sd = ref_cpu.GP_train_identity(x, y, e, P[0])
        np.testing.assert_allclose(mu, f3[f"c{i}_mu0"], rtol=1e-7, atol=1e-9)
        np.testing.assert_allclose(sd, f3[f"c{i}_sd0"], rtol=1e-6)


def test_evaluate_loss_bitwise_testfiles(f2):
    s, ex = f2["sigma_vals"], f2["expected"]
    for i in range(int(f2["ncases"])):
        x, y, e = _fx(f2[f"c{i}_x"]), f2[f"c{i}_y"], f2[f"c{i}_e"]
        lo, hi, P = f2[f"c{i}_lo"], f2[f"c{i}_hi"], f2[f"c{i}_P"]
        got = np.array([ref_cpu.evaluate_loss(p, x, y, e, s, ex, lo, hi) for p in P])
        assert np.array_equal(got, f2[f"c{i}_loss"]), str(f2[f"c{i}_tag"])


def test_evaluate_loss_bitwise_synthetic_small(f3):
    s, ex = f3["sigma_vals"], f3["expected"]
    for i in range(int(f3["ncases"])):
        N = int(f3[f"c{i}_meta"][0])
        if N > 256:
            continue  # the 1024 cases run in the slow suite below
        x, y, e = f3[f"c{i}_x"], f3[f"c{i}_y"], f3[f"c{i}_e"]
        lo, hi, P = f3[f"c{i}_lo"], f3[f"c{i}_hi"], f3[f"c{i}_P"]
        got = np.array([ref_cpu.evaluate_loss(p, x, y, e, s, ex, lo, hi) for p in P])
        assert np.array_equal(got, f3[f"c{i}_loss"]), i


def test_sentinel_and_degenerate_bounds(f2):
    """Test_file3 has 2 distinct energies -> lower == upper."""
    for i in range(int(f2["ncases"])):
        if "Test_file3" in str(f2[f"c{i}_tag"]):
            assert np.all(f2[f"c{i}_loss"] == ref_cpu.SENTINEL)
            lo, hi = ref_cpu.search_bounds(_fx(f2[f"c{i}_x"]))
            assert np.any(lo >= hi)


@pytest.mark.parametrize("k", [0, 1, 2])
def test_pso_trajectory_bitwise(f4, k, capsys):
    x, y, e = _fx(f4[f"c{k}_x"]), f4[f"c{k}_y"], f4[f"c{k}_e"]
    np.random.seed(int(f4[f"c{k}_seed"]))
    best = ref_cpu.len_scale_opt(x, y, e, True, init_positions=f4[f"c{k}_init"])
    out = capsys.readouterr().out
    assert np.array_equal(best, f4[f"c{k}_best"])
    assert out == str(f4[f"c{k}_log"])


def test_pairwise_sum_order():
    """numpy's float64 add.reduce order, used by np.trapezoid (find_len_scales.py:166)."""
    from oracle.pairwise import pairwise_sum
    rng = np.random.default_rng(0)
    for n in [1, 5, 8, 9, 127, 128, 129, 999, 1000, 4097]:
        a = rng.standard_normal(n) * 10.0 ** rng.integers(-8, 8, size=n)
        assert pairwise_sum(a) == a.sum()


def test_evaluate_loss_bitwise_configB_fixture():
    """F11 (the reference's evaluate_loss on config B's data, N=1024 d=2, seed 0): the oracle
    reproduces the losses and the recorded GP() mean/sd bit for bit; the inputs regenerate
    from the seed (sha256 stored with the fixture)."""
    from conftest import fixture_data, load_golden
    fx = load_golden("f11_configB.npz")
    x, y, e = fixture_data(fx["meta"], fx["data_sha256"])
    lo, hi = ref_cpu.search_bounds(x)
    np.testing.assert_array_equal(lo, fx["lo"])
    np.testing.assert_array_equal(hi, fx["hi"])
    s, ex = fx["sigma_vals"], fx["expected"]
    for k, p in enumerate(fx["P"][:3]):  # ~0.3 s each on one core
        assert ref_cpu.evaluate_loss(p, x, y, e, s, ex, lo, hi) == fx["loss"][k], k
        mu, sd = ref_cpu.GP(x, y, e, x, p, batch_size=x.shape[1])
        np.testing.assert_array_equal(mu, fx["mu"][k])
        np.testing.assert_array_equal(sd, fx["sd"][k])


def test_configE_fixtures_share_inputs():
    """F9 and F9b score particles on the same regenerated config-E inputs."""
    from conftest import load_golden
    a, b = load_golden("f9_configE.npz"), load_golden("f9b_configE.npz")
    assert str(a["data_sha256"]) == str(b["data_sha256"])
    np.testing.assert_array_equal(a["lo"], b["lo"])
    assert b["mu"].shape == (2, 16384) and np.all(np.isfinite(b["loss"]))
