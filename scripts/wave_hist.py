"""Per-wave start/end spread of one pairwise launch (stamps build + RBG_WAVE_DUMP)."""
import os, sys
import numpy as np
d = np.fromfile(sys.argv[1], dtype=np.uint32).reshape(-1, 16384, 4)
for i, r in enumerate(d):
    n = int((r[:, 1] != 0).sum())
    r = r[:n].astype(np.int64)
    print('waves', n)
    t0 = r[:, 0].min()
    end = (r[:, 1] - t0) / 100.0
    life = (r[:, 1] - r[:, 0]) / 100.0
    xcc = r[:, 2] & 0xF
    cu = (r[:, 3] >> 8) & 0xF
    se = (r[:, 3] >> 13) & 0x7
    simd = (r[:, 3] >> 4) & 0x3
    print(f"launch {i}: end us pct 0/10/50/90/99/100:", np.percentile(end, [0, 10, 50, 90, 99, 100]).round(1))
    print("  by XCC mean end:", [round(end[xcc == x].mean(), 1) for x in range(8)],
          "max:", [round(end[xcc == x].max(), 1) for x in range(8)])
    print("  by blockIdx%8 mean end:", [round(end[(np.arange(n) // 4) % 8 == x].mean(), 1) for x in range(8)])
    print("  by SE mean end:", [round(end[se == x].mean(), 1) for x in range(8) if (se == x).any()])
    print("  by SIMD mean end:", [round(end[simd == x].mean(), 1) for x in range(4)])
    wv = np.arange(n) % 4
    print("  by wave-in-WG mean end:", [round(end[wv == x].mean(), 1) for x in range(4)])
    # waves per (xcc, se, cu)
    key = xcc * 1000 + se * 100 + cu
    u, c = np.unique(key, return_counts=True)
    print("  CUs used", len(u), "waves/CU min/max", c.min(), c.max())
    hist, edges = np.histogram(end, bins=12)
    print("  hist", list(zip(edges.round(0).astype(int).tolist(), hist.tolist())))
