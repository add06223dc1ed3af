"""Runs one pairwise op on one container-family pair repeatedly (for rocprofv3 counter passes)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from roaringbitmap_amd import Engine
ka, kb, op, reps = sys.argv[1], sys.argv[2], sys.argv[3], int(sys.argv[4]) if len(sys.argv) > 4 else 5
fam = {"A": 16, "B": 17, "R": 18, "M": 0}
torch.cuda.set_device(0)
e = Engine(0)
a = e.synth(fam[ka], 0xC2A0)
b = e.synth(fam[kb], 0xC2B0)
for _ in range(reps):
    if op == "card":
        e.and_cardinality(a, b)
    else:
        e.pairwise(op, a, b)
e.sync()
print("done")
