"""Dump per-wave start/end of pairwise AND launches (stamps build; see wave_hist.py)."""
import ctypes, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from roaringbitmap_amd import Engine
from roaringbitmap_amd._lib import lib
torch.cuda.set_device(0)
e = Engine(0)
buf = (ctypes.c_uint64 * 20)()
fams = {"BB": (17, 17), "MM": (0, 0), "AA": (16, 16)}
for name in sys.argv[1:]:
    fa, fb = fams[name]
    a, b = e.synth(fa, 0xC2A0), e.synth(fb, 0xC2B0)
    for _ in range(3):
        e.pairwise("and", a, b)
    e.sync()
    os.environ.pop("RBG_WAVE_DUMP", None)
    lib().rbg_debug_stamps(buf, 1)
    for i in range(2):
        e.pairwise("and", a, b)
        e.sync()
        os.environ["RBG_WAVE_DUMP"] = f"gpurun_out/waves_{name}.bin"
        lib().rbg_debug_stamps(buf, 1)
        os.environ.pop("RBG_WAVE_DUMP")
    e.release(a); e.release(b)
