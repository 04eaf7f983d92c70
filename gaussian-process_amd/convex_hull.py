"""Drop-in for the reference's convex_hull.py: the prediction grid of GP_fit.py:31.

SURVEY.md §8f row 3. The Qhull facets are rasterised onto the per-dimension resolution
grid on the host (short sequential walks, convex_hull.py:38-174); the d sort + scan-fill
passes over the whole grid, where the reference spends ~95% of its time, run on the
MI355X (gpf_hull_fill, csrc/gpf_hull.hip). Same snapping rule and traversal order as
convex_hull.py:13-224, so the grid is identical point for point (tests/test_host_glue.py,
fixtures F6).
"""
import functools

import numpy as np
from scipy.spatial import ConvexHull

from gpfit import default_context

__all__ = ["fill_convex_hull", "round_to_res"]


def _decimals(res):
    """Digits after the decimal point of str(res) (0.01 -> 2, 0.25 -> 2)."""
    txt = str(res)
    return len(txt) - 1 - txt.index(".") if "." in txt else -1


@functools.lru_cache(maxsize=64)
def _trim(res):
    """(decimals of res, 10.0 ** decimals) for the trim step of round_to_res."""
    d = _decimals(res)
    return d, 10.0 ** d


def round_to_res(value, res):
    """Nearest multiple of res (Python round: half to even), then trimmed to res's
    decimals when res < 1 (convex_hull.py:13-24).

    The trim is numpy's float rounding (np.around: multiply by 10**d, round half to even,
    divide) done on the scalar directly; np.around on one scalar costs ~8 us, and the facet
    rasterisation calls this once per coordinate of every point it walks
    (tests/test_host_glue.py::test_host_rasterisation_matches_oracle pins it to the oracle's
    np.around form)."""
    if res < 1:
        d, p10 = _trim(float(res))
        if d >= 0:  # the same IEEE operations on Python floats
            r = float(res)
            return round(round(float(value) / r) * r * p10) / p10
    snapped = round(value / res) * res
    if res < 1:
        snapped = np.around(snapped, _decimals(res))
    return snapped


def _unique_rows(rows):
    """Distinct rows in lexicographic order (the reference's sorted(set(tuples)))."""
    return np.array(sorted({tuple(r) for r in rows.tolist()}))


def _segment(a, b, res):
    """Grid points from a to b, stepping along the dimension that needs most steps
    (convex_hull.py:38-72). The walk runs on Python floats (same operations and order as the
    reference's numpy scalars, a fraction of their per-operation cost)."""
    lead = int(np.argmax(np.abs((a - b) / res)))
    lo, hi = (a, b) if a[lead] < b[lead] else (b, a)
    span = (hi - lo).tolist()
    lo, hi, rs = lo.tolist(), hi.tolist(), np.asarray(res, dtype=np.float64).tolist()
    others = [k for k in range(len(lo)) if k != lead]
    pts = [lo]
    cur = list(lo)
    while cur[lead] < hi[lead]:
        cur[lead] = round_to_res(cur[lead] + rs[lead], rs[lead])
        frac = (cur[lead] - lo[lead]) / span[lead]
        for k in others:
            cur[k] = round_to_res((frac * span[k]) + lo[k], rs[k])
        pts.append(list(cur))
    return np.array(pts, dtype=np.float64)


def _polygon_outline(corners, res):
    """Rasterised closed polygon through the corners in order (convex_hull.py:76-97)."""
    n = len(corners)
    pieces = [_segment(corners[0], corners[1], res)]
    for k in range(1, n):
        nxt = corners[0] if k == n - 1 else corners[k + 1]
        pieces.append(_segment(corners[k], nxt, res))
    return _unique_rows(np.concatenate(pieces))


def _scanfill(axis, pts, res):
    """Fill the gaps between consecutive (sorted) points that differ only along
    `axis`, stepping by res[axis] (convex_hull.py:122-155); Python floats, as in _segment."""
    d = pts.shape[1]
    rows, rs = pts.tolist(), np.asarray(res, dtype=np.float64).tolist()
    stride = [rs[axis] if j == axis else 0.0 for j in range(d)]
    others = [k for k in range(d) if k != axis]
    out = []
    for k in range(len(rows) - 1):
        a, b = rows[k], rows[k + 1]
        if any(a[j] != b[j] for j in others):
            continue
        cur = list(a)
        out.append(cur)
        while cur[axis] < b[axis]:
            cur = [round_to_res(cur[j] + stride[j], rs[j]) for j in range(d)]
            out.append(cur)
        out.append(list(b))
    out.append(rows[-1])
    return _unique_rows(np.concatenate((np.array(out, dtype=np.float64), pts)))


def _facet_surface(corners, res):
    """Outline of one hull facet, filled along its last non-flat axis
    (convex_hull.py:159-174: the axis index starts at len(corners) - 1)."""
    outline = _polygon_outline(corners, res)
    axis = len(corners) - 1
    while np.max(corners[:, axis]) - np.min(corners[:, axis]) == 0:
        axis -= 1
    return _scanfill(axis, outline, res)


def fill_convex_hull(points, step):
    """Grid points (rows) filling the convex hull of `points` (n, d) at resolution `step`
    (convex_hull.py:203-224)."""
    points = np.asarray(points)
    res = np.asarray(step, dtype=np.float64).reshape(-1)
    hull = ConvexHull(points)
    shells = np.concatenate([_facet_surface(points[list(simplex)], res) for simplex in hull.simplices])
    decimals = [_decimals(r) for r in res]
    # d passes: fill along the last column, rotate the columns left by one (convex_hull.py:218-223)
    return default_context().hull_fill(shells.astype(np.float64), res, decimals)
