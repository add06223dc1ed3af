"""One BSI compare op repeated on the C5 synthetic index (for counter passes).

usage: python scripts/bsi_one.py ROWS OP SUM(0/1) REPS
"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))

import torch  # noqa: E402

from roaringbitmap_amd.engine import Engine  # noqa: E402


def main():
    rows, op, want_sum, reps = int(sys.argv[1]), sys.argv[2], sys.argv[3] == "1", int(sys.argv[4])
    torch.cuda.init()
    eng = Engine(0)
    b = eng.synth(4, 0xC5, rows)
    mn, mx = eng.batch_minmax(b)
    for _ in range(reps):
        eng.bsi(b, op, 31, 1 << 29, 1 << 30, mn, mx, want_sum=want_sum)
    eng.sync()
    eng.release(b)


if __name__ == "__main__":
    main()
