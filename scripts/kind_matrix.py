"""Per container-kind timing of the pairwise kernels (debugging aid, not a bench line).

Builds 65536-key operands from one container family each (A, B or R, same
generator as C2) and times and / and_card / or for every family pair.
"""
import os, sys, json
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from roaringbitmap_amd import Engine
torch.cuda.set_device(0)
e = Engine(0)
fam = {"A": 16, "B": 17, "R": 18}
bat = {k: (e.synth(v, 0xC2A0), e.synth(v, 0xC2B0)) for k, v in fam.items()}
bat["mix"] = (e.synth(0, 0xC2A0), e.synth(0, 0xC2B0))
out = {}
for ka in ["A", "B", "R", "mix"]:
    for kb in (["A", "B", "R"] if ka != "mix" else ["mix"]):
        a, b = bat[ka][0], bat[kb][1]
        st = e.batch_stats(a), e.batch_stats(b)
        for name, fn in [("and", lambda: e.pairwise("and", a, b)), ("and_card", lambda: e.and_cardinality(a, b)),
                         ("or", lambda: e.pairwise("or", a, b))]:
            for _ in range(3):
                fn()
            e.sync()
            e.profile(10)
            for _ in range(10):
                fn()
            n, ph = e.profile_read()
            e.profile(0)
            out[f"{ka}{kb}.{name}"] = [round(x / n, 4) for x in ph]
        out[f"{ka}{kb}.in_MB"] = round((st[0]["serialized_bytes"] + st[1]["serialized_bytes"]) / 1e6, 1)
for k, v in out.items():
    print(k, v)
