"""Compute-kernel time per container family (65,536-key operands of one family each, the C2 generator)
and on the C2 mix, for AND and andCardinality: engine phase events, mean of N launches.  Prints one JSON
line tagged with the library in use (RBG_LIB)."""
import json, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch
from roaringbitmap_amd import Engine
torch.cuda.set_device(0)
e = Engine(0)
fam = {"A": 16, "B": 17, "R": 18, "mix": 0}
which = sys.argv[1].split(",") if len(sys.argv) > 1 else ["RR", "AR", "BR", "mix"]
N = 20
out = {"lib": os.path.basename(os.environ.get("RBG_LIB", "default"))}
bat = {}
for w in which:
    ka, kb = (w[0], w[1]) if w != "mix" else ("mix", "mix")
    a = bat.setdefault(ka + "a", e.synth(fam[ka], 0xC2A0))
    b = bat.setdefault(kb + "b", e.synth(fam[kb], 0xC2B0))
    for name, fn in [("and", lambda: e.pairwise("and", a, b)), ("card", lambda: e.and_cardinality(a, b))]:
        for _ in range(3):
            fn()
        e.sync()
        e.profile(N)
        for _ in range(N):
            fn()
        n, ph = e.profile_read()
        e.profile(0)
        out[f"{w}.{name}"] = round(ph[1] / n, 4)
print(json.dumps(out), flush=True)
