"""What the engine's HIP-event phase timing adds to the C2 headline step (op + serialization, back to
back): no events, two events per op around the compute kernel (profile compute_only), four per op (all
phases).  Alternating rounds on one box; the compute kernel time each form reads."""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from roaringbitmap_amd import Engine
torch.cuda.set_device(0)
e = Engine(0)
a, b = e.synth(0, 0xC2A0), e.synth(0, 0xC2B0)
N = 40
for _ in range(5):
    e.pairwise("and", a, b)
    e.serialize()
e.sync()
for rnd in range(3):
    for mode in ("none", "compute", "all"):
        if mode != "none":
            e.profile(N, compute_only=(mode == "compute"))
        t0 = time.perf_counter()
        for _ in range(N):
            e.pairwise("and", a, b)
            e.serialize()
        e.sync()
        st = (time.perf_counter() - t0) / N
        kern = 0.0
        if mode != "none":
            n, ph = e.profile_read()
            e.profile(0)
            kern = ph[1] / max(n, 1)
        print(f"round={rnd} events={mode} step_ms={st * 1e3:.4f} compute_kernel_ms={kern:.4f}", flush=True)
