"""Time every BSI compare op (heap and buffer package) on the C5 synthetic index (device-resident).

usage: python scripts/bsi_time.py ROWS [REPS]
"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))

import torch  # noqa: E402

from roaringbitmap_amd.bsi import OPERATIONS  # noqa: E402
from roaringbitmap_amd.engine import Engine  # noqa: E402


def timed(eng, fn, reps):
    fn()
    eng.sync()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
        eng.sync()
    return round((time.perf_counter() - t0) / reps * 1e3, 3)


def main():
    rows = int(sys.argv[1])
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    torch.cuda.init()
    eng = Engine(0)
    b = eng.synth(4, 0xC5, rows)
    mn, mx = eng.batch_minmax(b)
    lo, hi = 1 << 29, 1 << 30
    print(json.dumps({"rows": rows, "stats": eng.batch_stats(b)}), flush=True)
    for op in OPERATIONS[:7]:
        out = {"op": op}
        out["heap_ms"] = timed(eng, lambda: eng.bsi(b, op, 31, lo, hi, mn, mx), reps)
        out["heap_containers"] = eng.result_stats()["containers"]
        out["heap_sum_ms"] = timed(eng, lambda: eng.bsi(b, op, 31, lo, hi, mn, mx, want_sum=True), reps)
        out["buffer_ms"] = timed(eng, lambda: eng.bsi_buffer(b, op, 31, lo, hi, mn, mx), reps)
        out["buffer_containers"] = eng.result_stats()["containers"]
        print(json.dumps(out), flush=True)
    eng.release(b)


if __name__ == "__main__":
    main()
