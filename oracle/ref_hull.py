"""CPU oracle for the convex-hull grid — TEST INFRASTRUCTURE ONLY.

A restatement of convex_hull.py:13-224: Qhull facets rasterised onto the resolution grid,
then the hull filled by scan lines, one dimension at a time, with the reference's snapping
rule and traversal order. Pinned to fixtures F6 (the reference's own output, point for
point); the checker of gpf_hull_fill. Only tests/ and bench.py's CPU baseline leg use it.
"""
import numpy as np
from scipy.spatial import ConvexHull

__all__ = ["fill_convex_hull", "round_to_res"]


def _decimals(res):
    """Digits after the decimal point of str(res) (0.01 -> 2, 0.25 -> 2)."""
    txt = str(res)
    return len(txt) - 1 - txt.index(".") if "." in txt else -1


def round_to_res(value, res):
    """Nearest multiple of res (Python round: half to even), then trimmed to res's
    decimals when res < 1 (convex_hull.py:13-24)."""
    snapped = round(value / res) * res
    if res < 1:
        snapped = np.around(snapped, _decimals(res))
    return snapped


def _unique_rows(rows):
    """Distinct rows in lexicographic order (the reference's sorted(set(tuples)))."""
    return np.array(sorted({tuple(r) for r in rows}))


def _segment(a, b, res):
    """Grid points from a to b, stepping along the dimension that needs most steps
    (convex_hull.py:38-72)."""
    lead = int(np.argmax(np.abs((a - b) / res)))
    lo, hi = (a, b) if a[lead] < b[lead] else (b, a)
    span = hi - lo
    pts = [lo]
    cur = np.array(lo, dtype=np.float64, copy=True)
    while cur[lead] < hi[lead]:
        cur[lead] = round_to_res(cur[lead] + res[lead], res[lead])
        frac = (cur[lead] - lo[lead]) / span[lead]
        for k in range(cur.shape[0]):
            if k != lead:
                cur[k] = round_to_res((frac * span[k]) + lo[k], res[k])
        pts.append(cur.copy())
    return np.array(pts)


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
    `axis`, stepping by res[axis] (convex_hull.py:122-155)."""
    stride = np.zeros(pts.shape[1])
    stride[axis] = res[axis]
    others = [k for k in range(pts.shape[1]) if k != axis]
    out = []
    for k in range(len(pts) - 1):
        a, b = pts[k], pts[k + 1]
        if not np.all(a[others] == b[others]):
            continue
        cur = a.copy()
        out.append(cur.copy())
        while cur[axis] < b[axis]:
            cur = cur + stride
            for j in range(cur.shape[0]):
                cur[j] = round_to_res(cur[j], res[j])
            out.append(cur.copy())
        out.append(b.copy())
    out.append(pts[-1])
    return _unique_rows(np.concatenate((np.array(out), pts)))


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
    res = step
    hull = ConvexHull(points)
    shells = [_facet_surface(points[list(simplex)], res) for simplex in hull.simplices]
    grid = _unique_rows(np.concatenate(shells))
    for _ in range(grid.shape[1]):
        # fill along the last column, then rotate the columns left by one (and the steps with them)
        grid = _scanfill(grid.shape[1] - 1, grid, res)
        grid = _unique_rows(np.concatenate((grid[:, 1:].T, grid[:, :1].T)).T)
        res = np.concatenate((res[1:], res[:1]))
    return grid
