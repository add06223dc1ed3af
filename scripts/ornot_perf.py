"""orNot kernel timing on the GPU box (rocprofv3 --kernel-trace --stats around it).

Two resident operands of N keys each (tests/_gen mixed container modes, 70% of keys present in each),
RoaringBitmap.orNot(x1, x2, N << 16) run `reps` times; one fetch at the end checks the bytes against
the oracle.  Prints the input payload bytes and the result size for the roofline arithmetic.
"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, ROOT)

import _gen  # noqa: E402
import _oracle as O  # noqa: E402
import roaringbitmap_amd as rb  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
mode = sys.argv[3] if len(sys.argv) > 3 else "mixed"
inplace = mode == "inplace"
rng = np.random.default_rng(5)
keys = np.arange(n)
if mode == "empty":  # every key x2-free and x1-free: full run containers only (the trivial-task floor)
    a = b = O.from_values(np.zeros(0, dtype=np.uint32))
elif mode == "bitmaps":  # every key a bitmap in both operands
    a = _gen.bitmap(rng, keys, modes=["b_mid"], p_present=1.0)
    b = _gen.bitmap(rng, keys, modes=["b_mid"], p_present=1.0)
else:
    a = _gen.bitmap(rng, keys, p_present=0.7)
    b = _gen.bitmap(rng, keys, p_present=0.7)
end = n << 16
eng = rb.Engine()
ia, ib = eng.load_pair(a, b)
eng.ornot(ia, ib, end, inplace)
got = eng.fetch().serialize()
want = O.ornot(a, b, end, inplace)
assert got == want, "orNot bytes differ from the oracle"
eng.sync()
t0 = time.perf_counter()
for _ in range(reps):
    eng.ornot(ia, ib, end, inplace)
    eng.serialize()
eng.sync()
dt = (time.perf_counter() - t0) / reps
print(f"mode={mode} keys={n} in_bytes={len(a) + len(b)} out_bytes={len(got)} inplace={inplace} host_ms_per_op={dt * 1e3:.3f}")
