"""ImmutableRoaringBitmap.and / andNot (RBG_AND_BUFFER / RBG_ANDNOT_BUFFER, k_pair_buf) on the C2 pair beside
the heap ops (k_pair_cu), for rocprofv3 --kernel-trace: 10 calls each + serialize."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from roaringbitmap_amd import Engine  # noqa: E402

eng = Engine(0)
a = eng.synth(0, 0xC2A0)
b = eng.synth(0, 0xC2B0)
for op in ("and", "and_buffer", "andnot", "andnot_buffer"):
    eng.pairwise(op, a, b)
    eng.serialize()
    eng.sync()
    t0 = time.perf_counter()
    for _ in range(10):
        eng.pairwise(op, a, b)
        eng.serialize()
    eng.sync()
    rs = eng.result_stats()
    print(f"{op}: {(time.perf_counter() - t0) / 10 * 1e3:.3f} ms per call (+ serialize), "
          f"{rs['containers']} containers, {rs['payload_bytes']} payload bytes")
