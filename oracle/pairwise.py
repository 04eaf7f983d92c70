"""NumPy's float64 pairwise summation order — TEST INFRASTRUCTURE ONLY.

``np.trapezoid`` (the reference's ``np.trapz``, find_len_scales.py:166) ends in
``(...).sum()``, i.e. numpy's ``pairwise_sum``: blocks of <= 128 are summed
with 8 interleaved accumulators combined as ((r0+r1)+(r2+r3))+((r4+r5)+(r6+r7))
plus a sequential tail; longer runs split at n/2 rounded down to a multiple
of 8. The HIP loss kernel reproduces this order so the calibration loss is
bit-identical; this restatement is what the test checks the order with.
"""


def pairwise_sum(a):
    n = len(a)
    if n < 8:
        r = 0.0
        for v in a:
            r += float(v)
        return r
    if n <= 128:
        acc = [float(v) for v in a[:8]]
        i = 8
        stop = n - (n % 8)
        while i < stop:
            for j in range(8):
                acc[j] += float(a[i + j])
            i += 8
        r = ((acc[0] + acc[1]) + (acc[2] + acc[3])) + ((acc[4] + acc[5]) + (acc[6] + acc[7]))
        while i < n:
            r += float(a[i])
            i += 1
        return r
    half = n // 2
    half -= half % 8
    return pairwise_sum(a[:half]) + pairwise_sum(a[half:])
