"""Phase timing of Engine.load for one serialized C2 operand (run with RBG_DEBUG_SYNC=1)."""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from roaringbitmap_amd import Engine
torch.cuda.set_device(0)
e = Engine(0)
a = e.synth(0, 0xC2A0)
x = e.batch_fetch(a).serialize()
for _ in range(3):
    t = time.perf_counter()
    b = e.load([x])
    print("load ms", (time.perf_counter() - t) * 1e3, file=sys.stderr)
    t = time.perf_counter()
    e.release(b)
    print("release ms", (time.perf_counter() - t) * 1e3, file=sys.stderr)
