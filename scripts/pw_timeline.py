"""One C2 AND with a timeline build (RBG_PWX & 16): placer chunk times vs kernel start (printf)."""
import os, sys
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "."))
import ctypes
from roaringbitmap_amd import Engine
eng = Engine(0)
a = eng.synth(0, 0xC2A0); b = eng.synth(0, 0xC2B0)
for _ in range(3):
    eng.pairwise("and", a, b)
eng.sync()
print("RUN", flush=True)
eng.pairwise("and", a, b)
eng.sync()
