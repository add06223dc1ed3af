"""Per-XCD wave timing of the C2 AND compute kernel at production speed.

Run under the default library (kernel time only) and under the RBG_WAVE_PROBE build
(scripts/build_variant.sh probe "-DRBG_WAVE_PROBE=1", loaded with RBG_LIB=...): that build adds three
16 B stores per wave at its end (start / end on the 100 MHz constant clock and on the shader clock,
XCC_ID, task count) and nothing per task.  Prints the kernel time (engine phase events, 20 launches)
and, for the probe build, per XCD: waves, tasks, mean / max wave end after the kernel's first wave
start, mean wave life, and the shader clock (delta s_memtime / delta s_memrealtime x 100 MHz)."""
import ctypes, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
from roaringbitmap_amd import Engine
from roaringbitmap_amd._lib import lib
torch.cuda.set_device(0)
e = Engine(0)
a, b = e.synth(0, 0xC2A0), e.synth(0, 0xC2B0)
for _ in range(5):
    e.pairwise("and", a, b)
e.sync()
times = []
for rnd in range(3):
    e.profile(20)
    for _ in range(20):
        e.pairwise("and", a, b)
    k, ph = e.profile_read()
    e.profile(0)
    times.append(ph[1] / max(k, 1))
tag = os.environ.get("RBG_LIB", "default")
print(f"lib={os.path.basename(tag)} RBG_PW_CU={os.environ.get('RBG_PW_CU', 'default')} C2 AND compute kernel ms per launch (3 x 20 launches): "
      + " ".join(f"{t:.4f}" for t in times), flush=True)
if "probe" in tag:
    buf = (ctypes.c_uint64 * 20)()
    path = "gpurun_out/xcd_probe.bin"
    if os.path.exists(path):
        os.remove(path)
    for rep in range(3):
        os.environ.pop("RBG_WAVE_DUMP", None)
        lib().rbg_debug_stamps(buf, 1)  # clear
        e.pairwise("and", a, b)
        e.sync()
        os.environ["RBG_WAVE_DUMP"] = path
        lib().rbg_debug_stamps(buf, 0)
        os.environ.pop("RBG_WAVE_DUMP")
    raw = np.fromfile(path, dtype=np.uint32).reshape(3, 16384, 3, 4)
    for rep in range(3):
        w = raw[rep]
        live = w[:, 2, 2] == 1
        r0 = w[live, 0, 0].astype(np.uint64) | (w[live, 0, 1].astype(np.uint64) << np.uint64(32))
        r1 = w[live, 0, 2].astype(np.uint64) | (w[live, 0, 3].astype(np.uint64) << np.uint64(32))
        m0 = w[live, 1, 0].astype(np.uint64) | (w[live, 1, 1].astype(np.uint64) << np.uint64(32))
        m1 = w[live, 1, 2].astype(np.uint64) | (w[live, 1, 3].astype(np.uint64) << np.uint64(32))
        xcc, ntask = w[live, 2, 0] & 0xF, w[live, 2, 1]
        base = r0.min()
        end_us = (r1 - base).astype(np.float64) / 100.0
        life_us = (r1 - r0).astype(np.float64) / 100.0
        print(f"launch {rep}: {live.sum()} waves, last wave end {end_us.max():.1f} us after the first start, "
              f"starts spread {float((r0.max() - base)) / 100.0:.1f} us; wave end p10 / p50 / p90 / p99 "
              + " / ".join(f"{np.percentile(end_us, q):.1f}" for q in (10, 50, 90, 99)) + " us; tasks per wave "
              f"min {int(ntask.min())} max {int(ntask.max())}", flush=True)
        for x in range(8):
            m = xcc == x
            if not m.any():
                continue
            mhz = float((m1[m] - m0[m]).sum()) / float((r1[m] - r0[m]).sum()) * 100.0
            print(f"  xcc {x}: waves {m.sum():5d} tasks {int(ntask[m].sum()):6d}  wave end mean {end_us[m].mean():6.1f} "
                  f"max {end_us[m].max():6.1f} us  life mean {life_us[m].mean():6.1f} us  shader clock {mhz:7.1f} MHz",
                  flush=True)
