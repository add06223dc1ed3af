"""Experiment: the C2 AND step (op + serialization) issued alternately on two engine contexts
(two HIP streams, separate device state), so one step's serialization can overlap the next
step's compute.  Prints ms per step for 1 and 2 contexts (debugging aid, not a bench line)."""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from roaringbitmap_amd import Engine
torch.cuda.set_device(0)
K = 40
engs = [Engine(0), Engine(0)]
pairs = [(e.synth(0, 0xC2A0), e.synth(0, 0xC2B0)) for e in engs]
sha = []
for e, (a, b) in zip(engs, pairs):
    e.pairwise("and", a, b)
    sha.append(hash(e.fetch().serialize()))
assert sha[0] == sha[1]
for nctx in (1, 2, 1, 2):
    for i in range(6):
        e = engs[i % nctx]; a, b = pairs[i % nctx]
        e.pairwise("and", a, b); e.serialize()
    for e in engs: e.sync()
    t0 = time.perf_counter()
    for i in range(K):
        e = engs[i % nctx]; a, b = pairs[i % nctx]
        e.pairwise("and", a, b); e.serialize()
    for e in engs: e.sync()
    dt = (time.perf_counter() - t0) / K
    print(f"contexts={nctx} ms_per_step={dt*1e3:.4f} input_GBps={0.717459586/dt:.1f}", flush=True)
