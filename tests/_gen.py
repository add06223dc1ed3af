"""Seeded random bitmaps whose containers sit on the reference's type thresholds.

Thresholds exercised (RB/ = RoaringBitmap/src/main/java/org/roaringbitmap/):
  4096 array/bitmap boundary (RB/ArrayContainer.java:27), the run-vs-array
  threshold of 32 (RB/RunContainer.java:576,2412), toEfficientContainer ties
  (RB/RunContainer.java:2326-2335), full containers (RB/RunContainer.java:1663),
  run containers that are not space-efficient, and the 2047-run bitmap limit.
"""
import numpy as np

from _fmt import A, B, R, encode

MODES = ["a_tiny", "a_32", "a_small", "a_mid", "a_edge", "b_edge", "b_mid", "b_dense", "full_b", "full_r",
         "r_few", "r_mid", "r_many", "r_tiny", "r_tie", "r_single", "r_dense", "b_sparse_runs"]


def _choice(rng, n, k):
    return np.sort(rng.choice(n, size=k, replace=False)).astype(np.uint16)


def _runs(rng, nr, min_len=1, max_len=None, span=65536):
    """nr disjoint, non-adjacent runs inside [0, span)."""
    seg = span // nr
    vals = []
    for i in range(nr):
        hi = (i + 1) * seg - 1  # leave a gap before the next segment
        s = i * seg + int(rng.integers(0, max(1, seg // 2)))
        room = max(1, hi - s)
        ml = room if max_len is None else min(room, max_len)
        ln = int(rng.integers(min(min_len, ml), ml + 1)) if ml > 1 else 1
        vals.append(np.arange(s, min(s + ln, hi)))
    v = np.unique(np.concatenate(vals)).astype(np.uint16)
    return v


def container(rng, mode):
    """-> (kind, sorted unique uint16 values)"""
    if mode == "a_tiny":
        return A, _choice(rng, 65536, int(rng.integers(1, 32)))
    if mode == "a_32":
        return A, _choice(rng, 65536, int(rng.integers(32, 41)))
    if mode == "a_small":
        return A, _choice(rng, 65536, int(rng.integers(1, 200)))
    if mode == "a_mid":
        return A, _choice(rng, 65536, int(rng.integers(200, 4097)))
    if mode == "a_edge":
        return A, _choice(rng, 65536, int(rng.integers(4080, 4097)))
    if mode == "b_edge":
        return B, _choice(rng, 65536, int(rng.integers(4097, 4121)))
    if mode == "b_mid":
        return B, _choice(rng, 65536, int(rng.integers(4097, 60000)))
    if mode == "b_dense":
        return B, np.setdiff1d(np.arange(65536), rng.choice(65536, int(rng.integers(1, 40)), replace=False)).astype(
            np.uint16)
    if mode == "full_b":
        return B, np.arange(65536, dtype=np.uint16)
    if mode == "full_r":
        return R, np.arange(65536, dtype=np.uint16)
    if mode == "r_few":
        return R, _runs(rng, int(rng.integers(1, 9)), min_len=100)
    if mode == "r_mid":
        return R, _runs(rng, int(rng.integers(100, 600)), max_len=40)
    if mode == "r_many":  # > 2047 runs: never space-efficient as a run container
        return R, _runs(rng, int(rng.integers(2048, 3000)), max_len=6)
    if mode == "r_tiny":  # few short runs, small cardinality
        return R, _runs(rng, int(rng.integers(1, 8)), max_len=4)
    if mode == "r_tie":  # runs of exactly 2 values: 2+4r == 2+2c (toEfficientContainer keeps R)
        nr = int(rng.integers(1, 40))
        starts = np.sort(rng.choice(65536 // 4, nr, replace=False)) * 4
        return R, np.unique(np.concatenate([starts, starts + 1])).astype(np.uint16)
    if mode == "r_single":  # singleton runs: array is smaller than runs
        nr = int(rng.integers(1, 60))
        return R, (np.sort(rng.choice(65536 // 2, nr, replace=False)) * 2).astype(np.uint16)
    if mode == "r_dense":  # long runs separated by small gaps
        gaps = np.sort(rng.choice(65536, int(rng.integers(1, 30)), replace=False))
        return R, np.setdiff1d(np.arange(65536), gaps).astype(np.uint16)
    if mode == "b_sparse_runs":  # bitmap whose content has ~1000 runs
        return B, _runs(rng, 1000, min_len=6, max_len=30)
    raise ValueError(mode)


def bitmap(rng, keys, modes=None, p_present=0.8):
    ctrs = []
    for k in keys:
        if rng.random() > p_present:
            continue
        m = modes[int(rng.integers(len(modes)))] if modes else MODES[int(rng.integers(len(MODES)))]
        kind, vals = container(rng, m)
        ctrs.append((int(k), kind, vals))
    return encode(ctrs)


def perturbed_pair(rng, keys):
    """Two bitmaps whose shared keys hold identical or near-identical containers
    (empty XOR/ANDNOT results, results landing exactly on thresholds)."""
    c1, c2 = [], []
    for k in keys:
        kind, vals = container(rng, MODES[int(rng.integers(len(MODES)))])
        c1.append((int(k), kind, vals))
        r = rng.random()
        if r < 0.3:
            c2.append((int(k), kind, vals))  # identical
        elif r < 0.6:
            drop = rng.choice(vals.size, size=min(vals.size - 1, int(rng.integers(1, 40))), replace=False) \
                if vals.size > 1 else []
            v2 = np.delete(vals, drop)
            k2 = kind if not (kind == B and v2.size <= 4096) else A
            c2.append((int(k), k2 if kind != R else R, v2))
        else:
            kind2, v2 = container(rng, MODES[int(rng.integers(len(MODES)))])
            c2.append((int(k), kind2, v2))
    return encode(c1), encode(c2)


def random_values(rng, n, universe=1 << 32):
    return rng.integers(0, universe, size=n, dtype=np.int64).astype(np.uint32)
