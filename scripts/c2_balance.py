"""Experiment: the C2 pairwise kernels with the tasks in key order (RBG_PW_BALANCE=0: the direct form) and
binned by estimated cost (k_plan_balanced + the rotated band walk), alternating on one box: AND compute
kernel (phase events), andCardinality kernel, the headline step (op + serialization), with the bytes
checked.  Also the per-family times (C2 generator forced to one family per operand)."""
import hashlib, os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from roaringbitmap_amd import Engine
torch.cuda.set_device(0)
e = Engine(0)
a, b = e.synth(0, 0xC2A0), e.synth(0, 0xC2B0)
os.environ["RBG_PW_BALANCE"] = "0"
e.pairwise("and", a, b)
ref = hashlib.sha256(e.fetch().serialize()).hexdigest()[:16]
N = 30


def kern(op, card=False, x=a, y=b):
    e.profile(N)
    for _ in range(N):
        if card:
            e.and_cardinality(x, y)
        else:
            e.pairwise(op, x, y)
    k, ph = e.profile_read()
    e.profile(0)
    return ph[0] / max(k, 1), ph[1] / max(k, 1)


for rnd in range(3):
    for bal in ("0", "1"):
        os.environ["RBG_PW_BALANCE"] = bal
        for _ in range(3):
            e.pairwise("and", a, b)
        e.sync()
        e.pairwise("and", a, b)
        ok = hashlib.sha256(e.fetch().serialize()).hexdigest()[:16] == ref
        pl, ka = kern("and")
        _, kc = kern("and", card=True)
        t0 = time.perf_counter()
        for _ in range(N):
            e.pairwise("and", a, b)
            e.serialize()
        e.sync()
        st = (time.perf_counter() - t0) / N
        print(f"round={rnd} balance={bal} plan_ms={pl:.4f} and_kernel_ms={ka:.4f} card_kernel_ms={kc:.4f} "
              f"step_ms={st * 1e3:.4f} sha_ok={ok}", flush=True)
fams = {"AA": (16, 16), "AB": (16, 17), "AR": (16, 18), "BB": (17, 17), "BR": (17, 18), "RR": (18, 18)}
for name, (fa, fb) in fams.items():
    x, y = e.synth(fa, 0xC2A0), e.synth(fb, 0xC2B0)
    row = []
    for bal in ("0", "1"):
        os.environ["RBG_PW_BALANCE"] = bal
        e.pairwise("and", x, y)
        e.sync()
        row.append(kern("and", x=x, y=y)[1])
    print(f"family {name}: and_kernel_ms key-order {row[0]:.4f} balanced {row[1]:.4f}", flush=True)
    e.release(x)
    e.release(y)
