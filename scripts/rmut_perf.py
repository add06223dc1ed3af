"""Range-mutation timings on the C2 operand (65,536 mixed containers), for rocprofv3 --kernel-trace:
flip / add / remove over [0, 2^32) and over a range cutting keys 100..60000 mid-key, each + serialize."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from roaringbitmap_amd import Engine  # noqa: E402

eng = Engine(0)
a = eng.synth(0, 0xC2A0)
st = eng.batch_stats(a)
print("operand payload bytes", st["payload_bytes"], "containers", st["containers"])
for op, lo, hi in (("flip", 0, 1 << 32), ("flip", (100 << 16) + 5, (60000 << 16) + 7), ("add", (100 << 16) + 5,
                   (60000 << 16) + 7), ("remove", (100 << 16) + 5, (60000 << 16) + 7)):
    eng.range_mut(op, a, lo, hi)
    rs = eng.result_stats()
    eng.serialize()
    eng.sync()
    reps = 10
    t0 = time.perf_counter()
    for _ in range(reps):
        eng.range_mut(op, a, lo, hi)
        eng.serialize()
    eng.sync()
    dt = (time.perf_counter() - t0) / reps
    print(f"{op} [{lo}, {hi}): {dt * 1e3:.3f} ms per call (+ serialize), result {rs['containers']} containers, "
          f"{rs['payload_bytes']} payload bytes")
