"""Per-phase clock breakdown of the pairwise kernel (needs a -DRBG_STAMPS=1 library via RBG_LIB)."""
import ctypes, json, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from roaringbitmap_amd import Engine
from roaringbitmap_amd._lib import lib
torch.cuda.set_device(0)
e = Engine(0)
fam = {"A": 16, "B": 17, "R": 18, "M": 0}
names = ["mat_a", "comb_b", "card+kind", "store_B+rec", "map", "probe+out", "rec_f", "stage_AR", "copy+rec_AR",
         "wave_life", "tasks", "task_total"]
buf = (ctypes.c_uint64 * 16)()
for ka, kb in [("B", "B"), ("A", "B"), ("R", "R"), ("B", "R"), ("A", "A"), ("M", "M")]:
    a, b = e.synth(fam[ka], 0xC2A0), e.synth(fam[kb], 0xC2B0)
    for op in ["and", "card"]:
        for _ in range(2):
            (e.and_cardinality(a, b) if op == "card" else e.pairwise("and", a, b))
        e.sync()
        lib().rbg_debug_stamps(buf, 1)
        for _ in range(5):
            (e.and_cardinality(a, b) if op == "card" else e.pairwise("and", a, b))
        e.sync()
        lib().rbg_debug_stamps(buf, 1)
        n = max(buf[10], 1)
        d = {nm: round(buf[i] / n) for i, nm in enumerate(names) if nm and buf[i] and nm != "tasks"}
        d["tasks_per_wave"] = round(n / max(1, 1), 1)
        print(ka + kb, op, "per task:", d, "waves-total tasks:", n)
    e.release(a); e.release(b)
