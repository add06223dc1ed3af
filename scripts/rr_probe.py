"""R AND R on C2's run family: which pairs take the run-domain path and what the results are
(debugging aid, not a bench line).  Prints the distribution of na + nb, and of the result
kind for the pairs that fit the wave's LDS (the others take the bitmap path)."""
import os, sys
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from roaringbitmap_amd import Engine


def parse(buf):
    """(key, kind, card, nruns) per container of a portable serialized bitmap."""
    b = memoryview(buf)
    c0 = int(np.frombuffer(b[:4], "<u4")[0])
    if c0 & 0xFFFF == 12347:
        n = (c0 >> 16) + 1
        nb = (n + 7) // 8
        flags = np.unpackbits(np.frombuffer(b[4:4 + nb], np.uint8), bitorder="little")[:n]
        p = 4 + nb
    else:
        n = int(np.frombuffer(b[4:8], "<u4")[0])
        flags = np.zeros(n, np.uint8)
        p = 8
    kc = np.frombuffer(b[p:p + 4 * n], "<u2").reshape(n, 2)
    p += 4 * n
    if c0 & 0xFFFF != 12347 or n >= 4:
        p += 4 * n
    out = []
    for i in range(n):
        key, card = int(kc[i, 0]), int(kc[i, 1]) + 1
        if flags[i]:
            nr = int(np.frombuffer(b[p:p + 2], "<u2")[0])
            out.append((key, "R", card, nr))
            p += 2 + 4 * nr
        elif card <= 4096:
            out.append((key, "A", card, 0))
            p += 2 * card
        else:
            out.append((key, "B", card, 0))
            p += 8192
    return out


torch.cuda.set_device(0)
e = Engine(0)
a, b = e.synth(18, 0xC2A0), e.synth(18, 0xC2B0)
ca = {k: (kd, c, r) for k, kd, c, r in parse(e.batch_fetch(a)._buf)}
cb = {k: (kd, c, r) for k, kd, c, r in parse(e.batch_fetch(b)._buf)}
e.pairwise("and", a, b)
res = {k: (kd, c, r) for k, kd, c, r in parse(e.fetch()._buf)}
both = sorted(set(ca) & set(cb))
kinds_in = {}
light = {"R": 0, "A": 0, "B": 0, "empty": 0}
heavy = {"R": 0, "A": 0, "B": 0, "empty": 0}
sums = []
for k in both:
    kinds_in[(ca[k][0], cb[k][0])] = kinds_in.get((ca[k][0], cb[k][0]), 0) + 1
    if ca[k][0] != "R" or cb[k][0] != "R":
        continue
    s = ca[k][2] + cb[k][2]
    sums.append(s)
    rk = res[k][0] if k in res else "empty"
    (light if s + 2 <= 2560 else heavy)[rk] += 1
sums = np.array(sums)
print("keys", len(both), "operand kinds", kinds_in)
print("na+nb percentiles 10/50/90/max", np.percentile(sums, [10, 50, 90]).tolist(), int(sums.max()))
print("light (run domain) result kinds", light)
print("heavy (bitmap path) result kinds", heavy)
rr = [res[k][2] for k in both if k in res and res[k][0] == "R"]
print("R result runs percentiles", np.percentile(rr, [10, 50, 90]).tolist() if rr else None)
cards = [res[k][1] for k in both if k in res]
print("result card percentiles", np.percentile(cards, [10, 50, 90]).tolist())
