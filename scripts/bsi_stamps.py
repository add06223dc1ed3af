"""Per-phase clocks of k_bsi_reg (diagnostic: needs an RBG_BSI_STAMPS=1 library via RBG_LIB)."""
import ctypes, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ["RBG_DEBUG_BSI"] = "1"
import torch
from roaringbitmap_amd import Engine
from roaringbitmap_amd._lib import lib
torch.cuda.set_device(0)
e = Engine(0)
rows = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000_000
b = e.synth(4, 0xC5, rows)
mn, mx = e.batch_minmax(b)
buf = (ctypes.c_uint64 * 20)()
for it in range(3):
    lib().rbg_debug_stamps(buf, 1)
    e.bsi(b, "RANGE", 31, 1 << 29, 1 << 30, mn, mx, want_sum=True)
    e.sync()
    lib().rbg_debug_stamps(buf, 1)
    tot = sum(buf[i] for i in range(7))
    print("iter", it, "phases(share):", [round(buf[i] / max(tot, 1), 3) for i in range(7)], "total Mcycles", tot / 1e6)
