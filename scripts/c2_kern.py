"""One line per task order: the C2 AND compute kernel and andCardinality kernel (engine phase events, N launches),
and the headline step (op + serialization), under the library in RBG_LIB (variant builds).  Bytes checked
against the default form's sha (argv[1], optional)."""
import hashlib, os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from roaringbitmap_amd import Engine
torch.cuda.set_device(0)
e = Engine(0)
a, b = e.synth(0, 0xC2A0), e.synth(0, 0xC2B0)
N = 30
lib = os.path.basename(os.environ.get("RBG_LIB", "default"))


def kern(card=False):
    e.profile(N)
    for _ in range(N):
        if card:
            e.and_cardinality(a, b)
        else:
            e.pairwise("and", a, b)
    k, ph = e.profile_read()
    e.profile(0)
    return ph[0] / max(k, 1), ph[1] / max(k, 1)


for bal in ("0", "1"):
    os.environ["RBG_PW_BALANCE"] = bal
    for _ in range(3):
        e.pairwise("and", a, b)
    e.pairwise("and", a, b)
    sha = hashlib.sha256(e.fetch().serialize()).hexdigest()[:16]
    pl, ka = kern()
    _, kc = kern(card=True)
    t0 = time.perf_counter()
    for _ in range(N):
        e.pairwise("and", a, b)
        e.serialize()
    e.sync()
    st = (time.perf_counter() - t0) / N
    print(f"lib={lib} balance={bal} plan_ms={pl:.4f} and_kernel_ms={ka:.4f} card_kernel_ms={kc:.4f} "
          f"step_ms={st * 1e3:.4f} sha={sha}", flush=True)
