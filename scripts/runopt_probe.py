"""runOptimize of a C2 operand, repeated (for a kernel trace of the runopt kernels)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from roaringbitmap_amd import Engine
torch.cuda.set_device(0)
e = Engine(0)
a = e.synth(0, 0xC2A0)
for _ in range(5):
    o, _ = e.run_optimize(a)
    e.release(o)
x = e.batch_fetch(a).serialize()
for _ in range(3):
    e.release(e.load([x]))
