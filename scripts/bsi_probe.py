"""Per-workgroup timing of C5's k_bsi_reg (compare(RANGE) + sum over 10^9 rows) under the RBG_WAVE_PROBE
build (scripts/build_variant.sh probe "-DRBG_WAVE_PROBE=1"; RBG_LIB=..., RBG_DEBUG_BSI=1): each workgroup
stores its start / end on the 100 MHz clock, XCC_ID, HW_ID and unit count at its end.  Prints the query
time (wall, 20 queries) and the spread of workgroup end times: overall, by XCD, and by the dispatch order
of the workgroups sharing a CU."""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import ctypes
import numpy as np
import torch
from roaringbitmap_amd import Engine
from roaringbitmap_amd._lib import lib
torch.cuda.set_device(0)
e = Engine(0)
rows = 10 ** 9
b = e.synth(4, 0xC5, rows, 0, (rows + 65535) // 65536)
mn, mx = e.batch_minmax(b)
lo, hi = 1 << 29, 1 << 30
for _ in range(5):
    e.bsi(b, "RANGE", 31, lo, hi, mn, mx, want_sum=True)
e.sync()
t0 = time.perf_counter()
for _ in range(20):
    e.bsi(b, "RANGE", 31, lo, hi, mn, mx, want_sum=True)
e.sync()
print(f"lib={os.path.basename(os.environ.get('RBG_LIB', 'default'))} query ms {(time.perf_counter() - t0) / 20 * 1e3:.4f}",
      flush=True)
if "probe" in os.environ.get("RBG_LIB", ""):
    os.environ["RBG_DEBUG_BSI"] = "1"
    buf = (ctypes.c_uint64 * 20)()
    path = "gpurun_out/bsi_probe.bin"
    if os.path.exists(path):
        os.remove(path)
    for rep in range(3):
        os.environ.pop("RBG_WAVE_DUMP", None)
        lib().rbg_debug_stamps(buf, 1)
        e.bsi(b, "RANGE", 31, lo, hi, mn, mx, want_sum=True)
        e.sync()
        os.environ["RBG_WAVE_DUMP"] = path
        lib().rbg_debug_stamps(buf, 0)
        os.environ.pop("RBG_WAVE_DUMP")
    raw = np.fromfile(path, dtype=np.uint32).reshape(3, 4096, 2, 4)
    for rep in range(3):
        w = raw[rep]
        live = w[:, 1, 3] == 1
        r0 = w[live, 0, 0].astype(np.uint64) | (w[live, 0, 1].astype(np.uint64) << np.uint64(32))
        r1 = w[live, 0, 2].astype(np.uint64) | (w[live, 0, 3].astype(np.uint64) << np.uint64(32))
        xcc, hw, nu = w[live, 1, 0] & 0xF, w[live, 1, 1], w[live, 1, 2]
        base = r0.min()
        end = (r1 - base).astype(np.float64) / 100.0
        start = (r0 - base).astype(np.float64) / 100.0
        print(f"launch {rep}: {live.sum()} workgroups, units {int(nu.min())}-{int(nu.max())}, last end {end.max():.1f} us; "
              f"end p10 / p50 / p90 / p99 " + " / ".join(f"{np.percentile(end, q):.1f}" for q in (10, 50, 90, 99))
              + f"; starts spread {start.max():.1f} us", flush=True)
        # workgroups sharing a CU (same XCC and HW_ID CU / SH / SE fields), in start order
        cu = (xcc.astype(np.int64) << 16) | ((hw >> 8) & 0xFF).astype(np.int64)
        order_ends = {}
        for c in np.unique(cu):
            idx = np.where(cu == c)[0]
            idx = idx[np.argsort(r0[idx])]
            for k, i in enumerate(idx):
                order_ends.setdefault(k, []).append(end[i])
        print("  mean end by dispatch order within a CU: "
              + " / ".join(f"{np.mean(v):.1f} (n={len(v)})" for k, v in sorted(order_ends.items())), flush=True)
