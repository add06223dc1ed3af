"""C3 wide OR/AND timing probe: synth a C3 batch on the device, time the ops (phase split)."""
import json, os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from roaringbitmap_amd import Engine
torch.cuda.set_device(0)
kind = int(sys.argv[1]); n = int(sys.argv[2]); lo = int(sys.argv[3]) if len(sys.argv) > 3 else 0
hi = int(sys.argv[4]) if len(sys.argv) > 4 else 65536
e = Engine(0)
t0 = time.time()
b = e.synth(kind, 0xC3000000, n, lo, hi)
st = e.batch_stats(b)
gen = time.time() - t0
in_bytes = st["payload_bytes"] + 4 * st["containers"]
out = {"kind": kind, "n": n, "keys": [lo, hi], "gen_s": round(gen, 2), "stats": st, "in_GB": round(in_bytes / 1e9, 3)}
for op in ["or", "and", "xor"]:
    e.wide(op, b, lo, hi); e.sync()
    e.profile(3)
    for _ in range(3):
        e.wide(op, b, lo, hi)
    k, ph = e.profile_read(); e.profile(0)
    ms = [x / k for x in ph]
    rs = e.result_stats()
    out[op] = {"phase_ms": [round(x, 3) for x in ms], "GBps_in": round(in_bytes / (sum(ms) / 1e3) / 1e9, 1),
               "result": rs}
print(json.dumps(out))
