"""addOffset timings on the C2 operand (65,536 mixed containers), for rocprofv3 --kernel-trace:
RoaringBitmap.addOffset(x, off) at a whole-key offset (clones), an offset inside a word and one at a
word edge, each + serialize."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from roaringbitmap_amd import Engine  # noqa: E402

eng = Engine(0)
a = eng.synth(0, 0xC2A0)
st = eng.batch_stats(a)
print("operand payload bytes", st["payload_bytes"], "containers", st["containers"])
for off in (3 << 16, 12345, 640, -(7 << 16) - 99):
    eng.add_offset(a, off)
    rs = eng.result_stats()
    eng.serialize()
    eng.sync()
    reps = 10
    t0 = time.perf_counter()
    for _ in range(reps):
        eng.add_offset(a, off)
        eng.serialize()
    eng.sync()
    dt = (time.perf_counter() - t0) / reps
    print(f"addOffset {off}: {dt * 1e3:.3f} ms per call (+ serialize), result {rs['containers']} containers, "
          f"{rs['payload_bytes']} payload bytes")
