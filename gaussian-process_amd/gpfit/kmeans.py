"""KMeans subsample of len_scale_opt (find_len_scales.py:25-47) with the Lloyd iterations on the GPU.

The reference calls ``KMeans(n_clusters=max_points, n_init='auto', random_state=0).fit_predict``
on the points and keeps, per cluster, the member nearest its centre. ``kmeans_fit`` reproduces
that fit: sklearn's own data preparation and k-means++ seeding (``sklearn.cluster.kmeans_plusplus``
on the mean-centred points with ``RandomState(random_state)`` — the draws ``KMeans.fit`` makes, so
the seeds are the reference's), then sklearn's Lloyd loop (``_kmeans_single_lloyd``: relocation of
empty clusters, averaging, centre shift, strict or tolerance convergence, the final E-step) with
every E-step and M-step sum over the points on the device (``Context.kmeans_step``,
csrc/gpf_kmeans.hip). Per iteration only O(k d) numbers cross to the host.

Floating point: sklearn forms ``||c||^2 - 2 x.c`` through BLAS and sums each cluster in chunk /
thread order (its own result depends on the OpenMP thread count); here the dot products run in
feature order and the sums in a fixed per-cluster order. Labels and the kept points agree with the
reference's on its fixtures (F10) and on the test sweep; the centres to rounding.
"""
import numpy as np

KM_MAXKD = 8192  # gpf_kmeans_step's LDS bound on k x (d + 1) (csrc/gpf_kmeans.hip)


def fits_device(n_clusters, d):
    """Whether gpf_kmeans_step can stage n_clusters centres of dimension d (and their norms)."""
    return n_clusters * (d + 1) <= KM_MAXKD


def kmeans_fit(ctx, X, n_clusters, *, random_state=0, max_iter=300, tol=1e-4):
    """labels, cluster_centers_ of KMeans(n_clusters, n_init='auto', random_state).fit(X) (X: n x d)."""
    from sklearn.cluster import kmeans_plusplus
    X = np.ascontiguousarray(X, dtype=np.float64)
    n, d = X.shape
    tol_abs = float(np.mean(np.var(X, axis=0)) * tol)  # sklearn's _tolerance, on the uncentred data
    mean = X.mean(axis=0)
    Xc = X - mean
    x_sq = np.einsum("ij,ij->i", Xc, Xc)  # sklearn's row_norms(X, squared=True)
    centers, _ = kmeans_plusplus(Xc, n_clusters, x_squared_norms=x_sq,
                                 random_state=np.random.RandomState(random_state))
    centers = np.ascontiguousarray(centers, dtype=np.float64)
    ctx.kmeans_set(Xc)
    labels_old = np.full(n, -1, dtype=np.int32)
    strict = False
    for _ in range(max_iter):
        labels, sums, counts, _ = ctx.kmeans_step(centers, update=True)
        empty = np.nonzero(counts == 0)[0]
        if empty.size:  # _relocate_empty_clusters_dense: the points farthest from their centres
            _, _, _, dist = ctx.kmeans_step(centers, update=False, want_dist=True)
            if np.max(dist) != 0:
                far = np.argpartition(dist, -empty.size)[:-empty.size - 1:-1]
                for new_id, idx in zip(empty, far):
                    old_id = labels[idx]
                    sums[old_id] -= Xc[idx]
                    sums[new_id] = Xc[idx]
                    counts[new_id] = 1.0
                    counts[old_id] -= 1.0
        # _average_centers (empty clusters, if any are left, at the heaviest cluster's centre)
        heaviest = int(np.argmax(counts))
        new = sums.copy()
        for j in range(n_clusters):
            if counts[j] > 0:
                new[j] = sums[j] * (1.0 / counts[j])
            else:
                new[j] = new[heaviest]
        shift = np.sqrt(np.sum((new - centers) ** 2, axis=1))  # _center_shift
        centers = new
        if np.array_equal(labels, labels_old):
            strict = True
            break
        if float(np.sum(shift ** 2)) <= tol_abs:
            break
        labels_old = labels
    if not strict:  # the final E-step, so that the labels match the centres
        labels, _, _, _ = ctx.kmeans_step(centers, update=False)
    return labels, centers + mean


def kmeans_representatives_gpu(ctx, x_known, y_known, e_known, max_points):
    """find_len_scales.py:25-47 with the fit on the GPU: the member nearest each centre."""
    pts = x_known.T
    labels, centres = kmeans_fit(ctx, pts, max_points)
    pick = []
    for k in range(max_points):
        members = np.where(labels == k)[0]
        if len(members) == 0:
            continue
        dist2 = np.sum((pts[members] - centres[k]) ** 2, axis=1)
        pick.append(members[np.argmin(dist2)])
    pick = np.array(pick)
    return x_known[:, pick], y_known[pick], e_known[pick]
