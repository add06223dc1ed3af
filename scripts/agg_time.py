"""Time every wide aggregation form on one synthetic C3-shaped batch (device-resident, synchronised).

usage: python scripts/agg_time.py KIND N [REPS [SKIP_OPS [ro]]]   (KIND 1 uniform, 2 clustered;
       ro: runOptimize the batch first)
"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))

import torch  # noqa: E402

from roaringbitmap_amd import _lib  # noqa: E402
from roaringbitmap_amd.engine import Engine  # noqa: E402


def main():
    kind, n = int(sys.argv[1]), int(sys.argv[2])
    reps = int(sys.argv[3]) if len(sys.argv) > 3 else 3
    skip = set(sys.argv[4].split(",")) if len(sys.argv) > 4 and sys.argv[4] else set()
    ro = len(sys.argv) > 5 and sys.argv[5] == "ro"
    torch.cuda.init()
    eng = Engine(0)
    b = eng.synth(kind, 0xC3000000, n)
    if ro:
        b0 = b
        b, _ = eng.run_optimize(b0)
        eng.release(b0)
    st = eng.batch_stats(b)
    print(json.dumps({"kind": kind, "n": n, "run_optimized": ro, "containers": st["containers"], "runs": st["run"],
                      "bitmaps": st["bitmap"], "payload_bytes": st["payload_bytes"]}), flush=True)
    for op in _lib.WIDE_OP:
        if op in skip:
            continue
        eng.wide(op, b)
        eng.sync()
        t0 = time.perf_counter()
        for _ in range(reps):
            eng.wide(op, b)
            eng.sync()
        ms = (time.perf_counter() - t0) / reps * 1e3
        rs = eng.result_stats()
        print(json.dumps({"op": op, "ms": round(ms, 3), "containers": rs["containers"],
                          "payload_bytes": rs["payload_bytes"]}), flush=True)
    eng.release(b)


if __name__ == "__main__":
    main()
