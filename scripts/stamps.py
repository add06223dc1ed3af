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
buf = (ctypes.c_uint64 * 20)()
for ka, kb in [("B", "B"), ("A", "B"), ("R", "R"), ("B", "R"), ("A", "A"), ("M", "M")]:
    a, b = e.synth(fam[ka], 0xC2A0), e.synth(fam[kb], 0xC2B0)
    for op in ["and", "card"]:
        for _ in range(2):
            (e.and_cardinality(a, b) if op == "card" else e.pairwise("and", a, b))
        e.sync()
        lib().rbg_debug_stamps(buf, 1)
        spans = []
        acc = [0] * 20
        for _ in range(5):
            (e.and_cardinality(a, b) if op == "card" else e.pairwise("and", a, b))
            e.sync()
            lib().rbg_debug_stamps(buf, 1)
            w = max(buf[13], 1)
            spans.append((round((buf[15] - (~buf[14] & (2**64 - 1))) / 100, 1),
                          round(buf[16] / w / 100, 1), round((buf[17] - (~buf[14] & (2**64 - 1))) / 100, 1)))
            for i in range(20):
                acc[i] = max(acc[i], buf[i]) if i in (12, 14, 15, 17) else acc[i] + buf[i]
        buf = acc
        n = max(buf[10], 1)
        d = {nm: round(buf[i] / n) for i, nm in enumerate(names) if nm and buf[i] and nm != "tasks"}
        d["tasks_per_wave"] = round(n / max(1, 1), 1)
        print(ka + kb, op, "per task:", d, "waves-total tasks:", n,
              "| mean wave life", round(buf[9] / max(buf[13], 1)), "max", buf[12],
              "| us (span, mean wave life, last start):", spans)
        buf = (ctypes.c_uint64 * 20)()
    e.release(a); e.release(b)
