"""Host logic of the product package, checked on CPU with the oracle injected
as the objective (the oracle is only the checker; the code under test is
gpfit.swarm, the drop-in PSO driver)."""
import numpy as np
import pytest

from oracle import ref_cpu


def _fx(x):
    return np.asfortranarray(x)


@pytest.mark.parametrize("k", [0, 1, 2])
def test_swarm_driver_reproduces_reference_trajectory(f4, k, capsys):
    from gpfit.swarm import particle_swarm
    x, y, e = _fx(f4[f"c{k}_x"]), f4[f"c{k}_y"], f4[f"c{k}_e"]
    best, info = particle_swarm(x, y, e, True, init_positions=f4[f"c{k}_init"], seed=int(f4[f"c{k}_seed"]),
                                evaluator=lambda args: [ref_cpu.evaluate_loss_helper(a) for a in args])
    out = capsys.readouterr().out
    assert np.array_equal(best, f4[f"c{k}_best"])
    assert out == str(f4[f"c{k}_log"])
    assert info["evals"] == 40 * (501 + info["restarts"])


def test_search_bounds_match_oracle(f2):
    from gpfit.swarm import search_bounds
    for i in range(int(f2["ncases"])):
        x = _fx(f2[f"c{i}_x"])
        lo, hi = search_bounds(x)
        rlo, rhi = ref_cpu.search_bounds(x)
        assert np.array_equal(lo, rlo) and np.array_equal(hi, rhi)
        assert np.array_equal(lo, f2[f"c{i}_lo"]) and np.array_equal(hi, f2[f"c{i}_hi"])


def test_sigma_grid_matches_reference(f2):
    from gpfit.swarm import sigma_grid
    s, ex = sigma_grid()
    assert np.array_equal(s, f2["sigma_vals"]) and np.array_equal(ex, f2["expected"])


def test_centred_lhs_is_latin_and_leaves_global_rng_alone():
    from gpfit.swarm import centred_lhs
    np.random.seed(3)
    before = np.random.get_state()[1].copy()
    lo, hi = np.array([0.1, 1.0, -2.0]), np.array([0.5, 3.0, 2.0])
    P = centred_lhs(lo, hi, 40, seed=11)
    assert np.array_equal(np.random.get_state()[1], before)
    for k in range(3):
        u = np.sort((P[:, k] - lo[k]) / (hi[k] - lo[k]))
        np.testing.assert_allclose(u, (np.arange(40) + 0.5) / 40, atol=1e-12)
    np.testing.assert_array_equal(P, centred_lhs(lo, hi, 40, seed=11))


def test_kmeans_representatives_match_oracle():
    from gpfit.swarm import kmeans_representatives
    rng = np.random.default_rng(0)
    x = rng.uniform(size=(2, 300))
    y, e = rng.standard_normal(300), np.full(300, 0.1)
    a = kmeans_representatives(x, y, e, 100)
    b = ref_cpu.kmeans_subsample(x, y, e, 100)
    for u, v in zip(a, b):
        assert np.array_equal(u, v)


def test_kmeans_subsample_matches_reference_fixture():
    """F10 (tests/golden/make_golden_big.py): the points the reference's len_scale_opt keeps
    (find_len_scales.py:25-47, sklearn KMeans n_init='auto', random_state=0) at N = 300..4096,
    d = 2..4, and the search box it derives from them (:56-61). The drop-in's prepare() must
    keep exactly the same points in the same order."""
    from conftest import fixture_data, load_golden
    from gpfit.swarm import prepare
    f = load_golden("f10_kmeans.npz")
    for i in range(int(f["ncases"])):
        x, y, e = fixture_data(f[f"c{i}_meta"], f[f"c{i}_data_sha256"])
        xs, ys, es, lo, hi, _, _ = prepare(_fx(x), y, e, max_points=100, verbose=False)
        idx = f[f"c{i}_idx"]
        assert np.array_equal(xs, x[:, idx]) and np.array_equal(ys, y[idx]) and np.array_equal(es, e[idx])
        assert np.array_equal(lo, f[f"c{i}_lo"]) and np.array_equal(hi, f[f"c{i}_hi"])


def test_kmeans_path_taken_above_max_points(capsys):
    from gpfit.swarm import particle_swarm
    rng = np.random.default_rng(1)
    x = rng.uniform(size=(2, 130))
    y, e = np.sin(4 * x[0]) + 0.1 * rng.standard_normal(130), np.full(130, 0.1)
    seen = []

    def ev(args):
        seen.append(args[0][1].shape[1])
        return [ref_cpu.evaluate_loss_helper(a) for a in args]

    particle_swarm(x, y, e, False, num_particles=4, max_iter=2, max_points=100, seed=0, evaluator=ev)
    assert "Subsampling to 100" in capsys.readouterr().out
    assert set(seen) == {100}


class _NumpyKMeansSteps:
    """Test stand-in for Context.kmeans_step (csrc/gpf_kmeans.hip's arithmetic in NumPy): lets the
    host half of gpfit.kmeans — sklearn's Lloyd loop around the device steps — run without a GPU."""

    def kmeans_set(self, X):
        self.X = np.array(X, dtype=np.float64)

    def kmeans_step(self, centers, update=True, want_dist=False):
        X, C = self.X, np.asarray(centers, dtype=np.float64)
        d2 = np.einsum("ij,ij->i", C, C)[None, :] + (-2.0 * (X @ C.T))
        labels = np.argmin(d2, axis=1).astype(np.int32)
        sums = counts = dist = None
        if update:
            k = C.shape[0]
            sums = np.zeros_like(C)
            np.add.at(sums, labels, X)
            counts = np.bincount(labels, minlength=k).astype(np.float64)
        if want_dist:
            dist = np.sum((X - C[labels]) ** 2, axis=1)
        return labels, sums, counts, dist


@pytest.mark.parametrize("n,d,k,dup", [(300, 2, 100, 0), (1024, 3, 100, 0), (2000, 4, 50, 0), (500, 2, 100, 300),
                                       (4096, 3, 100, 0)])
def test_kmeans_fit_loop_matches_sklearn(n, d, k, dup):
    """gpfit.kmeans.kmeans_fit (sklearn's seeding and Lloyd loop, the E/M-steps delegated — here to
    a NumPy stand-in of the device steps): labels equal to sklearn's KMeans(k, n_init='auto',
    random_state=0).fit, centres to rounding; with many duplicate points too (empty clusters get
    relocated as sklearn's _relocate_empty_clusters_dense does)."""
    from sklearn.cluster import KMeans
    from gpfit.kmeans import kmeans_fit
    rng = np.random.default_rng(n + d + k + dup)
    X = rng.uniform(size=(n, d))
    if dup:
        X[-dup:] = X[:8][rng.integers(0, 8, size=dup)]
    km = KMeans(n_clusters=k, n_init="auto", random_state=0).fit(X)
    labels, centres = kmeans_fit(_NumpyKMeansSteps(), X, k)
    assert np.array_equal(labels, km.labels_)
    np.testing.assert_allclose(centres, km.cluster_centers_, rtol=0, atol=1e-12)


def test_kmeans_fit_keeps_the_reference_points_f10():
    """F10 (the points the reference's len_scale_opt keeps, N = 300..4096) through the GPU path's
    host loop (NumPy stand-in for the device steps): the same points in the same order."""
    from conftest import fixture_data, load_golden
    from gpfit.kmeans import kmeans_representatives_gpu
    f = load_golden("f10_kmeans.npz")
    for i in range(int(f["ncases"])):
        x, y, e = fixture_data(f[f"c{i}_meta"], f[f"c{i}_data_sha256"])
        xs, ys, es = kmeans_representatives_gpu(_NumpyKMeansSteps(), _fx(x), y, e, 100)
        idx = f[f"c{i}_idx"]
        assert np.array_equal(xs, x[:, idx]) and np.array_equal(ys, y[idx]) and np.array_equal(es, e[idx])


def test_kmeans_above_device_cap_uses_host_fit():
    """max_points x (d + 1) > 8192 (gpf_kmeans_step's LDS bound) keeps sklearn's host fit instead of
    raising: prepare() with a context stand-in that must not be asked for a step; just
    under the cap the device path (here its NumPy stand-in) is taken and keeps the same points."""
    from gpfit.kmeans import fits_device
    from gpfit.swarm import kmeans_representatives, prepare

    class _Refuse(_NumpyKMeansSteps):
        def kmeans_step(self, *a, **k):
            raise AssertionError("device KMeans step above its cap")

    assert not fits_device(1000, 9) and not fits_device(300, 32) and fits_device(1000, 7)
    rng = np.random.default_rng(3)
    x = rng.uniform(size=(9, 1200))
    y, e = np.sin(3 * x[0]), np.full(1200, 0.1)
    xs, ys, es = prepare(x, y, e, max_points=1000, verbose=False, ctx=_Refuse())[:3]
    want = kmeans_representatives(x, y, e, 1000)
    assert np.array_equal(xs, want[0]) and np.array_equal(ys, want[1]) and np.array_equal(es, want[2])
    x7 = x[:7, :1100]
    xs7 = prepare(x7, y[:1100], e[:1100], max_points=1000, verbose=False, ctx=_NumpyKMeansSteps())[0]
    assert np.array_equal(xs7, kmeans_representatives(x7, y[:1100], e[:1100], 1000)[0])
