"""The C2 headline step (RoaringBitmap.and + serialize) and its parts under the library in RBG_LIB (default:
the in-tree one): wall ms per step over 100 steps, the compute kernel's event time, the serialization's
event time, andCardinality's kernel time.  One JSON line tagged with the library (alternating comparisons)."""
import json, os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch
from roaringbitmap_amd import Engine
torch.cuda.set_device(0)
e = Engine(0)
a, b = e.synth(0, 0xC2A0), e.synth(0, 0xC2B0)
out = {"lib": os.path.basename(os.environ.get("RBG_LIB", "default"))}
N = 100
for _ in range(10):
    e.pairwise("and", a, b)
    e.serialize()
e.sync()
t0 = time.perf_counter()
for _ in range(N):
    e.pairwise("and", a, b)
    e.serialize()
e.sync()
out["step_ms"] = round((time.perf_counter() - t0) / N * 1e3, 4)
e.profile(N, compute_only=True)
for _ in range(N):
    e.pairwise("and", a, b)
    e.serialize()
n, ph = e.profile_read()
e.profile(0)
out["compute_ms"] = round(ph[1] / n, 4)
st = torch.cuda.ExternalStream(e.stream_ptr)
ser = 0.0
for _ in range(20):
    e.pairwise("and", a, b)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st)
    e.serialize()
    e1.record(st)
    e.sync()
    ser += e0.elapsed_time(e1)
out["serialize_ms"] = round(ser / 20, 4)
e.profile(N)
for _ in range(N):
    e.and_cardinality(a, b)
n, ph = e.profile_read()
e.profile(0)
out["card_ms"] = round(ph[1] / n, 4)
print(json.dumps(out), flush=True)
