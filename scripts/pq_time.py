"""Time FastAggregation.priorityqueue_or / naive_or on synthetic C3-shaped batches (device-resident).

usage: python scripts/pq_time.py KIND N [REPS]   (KIND 1 uniform, 2 clustered)
"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))

import torch  # noqa: E402

from roaringbitmap_amd.engine import Engine  # noqa: E402


def main():
    kind, n = int(sys.argv[1]), int(sys.argv[2])
    reps = int(sys.argv[3]) if len(sys.argv) > 3 else 3
    torch.cuda.init()
    eng = Engine(0)
    b = eng.synth(kind, 0xC3000000, n)
    st = eng.batch_stats(b)
    out = {"kind": kind, "n": n, "containers": st["containers"]}
    for op in ("or", "priorityqueue_or", "priorityqueue_xor"):
        eng.wide(op, b)
        eng.sync()
        t0 = time.perf_counter()
        for _ in range(reps):
            eng.wide(op, b)
            eng.sync()
        out[op + "_ms"] = round((time.perf_counter() - t0) / reps * 1e3, 3)
        rs = eng.result_stats()
        out[op + "_containers"] = rs["containers"]
        print(json.dumps(out), flush=True)
    eng.release(b)


if __name__ == "__main__":
    main()
