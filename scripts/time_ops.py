"""Times every pairwise op and andCardinality on a device-resident C2 pair (phase split)."""
import os, sys, json
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from roaringbitmap_amd import Engine
torch.cuda.set_device(0)
e = Engine(0)
a = e.synth(0, 0xC2A0); b = e.synth(0, 0xC2B0)
out = {}
for name, fn in [("and", lambda: e.pairwise("and", a, b)), ("or", lambda: e.pairwise("or", a, b)),
                 ("xor", lambda: e.pairwise("xor", a, b)), ("andnot", lambda: e.pairwise("andnot", a, b)),
                 ("and_card", lambda: e.and_cardinality(a, b))]:
    for _ in range(3):
        fn()
    e.sync()
    e.profile(10)
    for _ in range(10):
        fn()
    n, ph = e.profile_read()
    e.profile(0)
    out[name] = [round(x / n, 4) for x in ph]
print(json.dumps(out))
