"""Experiment: the C2 AND step as op + serialization (two calls) against the pipelined form
(rbg_ctx_pairwise_serialized: K key ranges, each range's placement and payload copies on a second
stream while the next range computes), over K and the compute / copy grids (RBG_PIPE_PW_WG,
RBG_PIPE_COPY_WG: workgroups per CU).  Alternating rounds on one box; checks the bytes."""
import hashlib, os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from roaringbitmap_amd import Engine
torch.cuda.set_device(0)
N = int(os.environ.get("N", "60"))
e = Engine(0)
a, b = e.synth(0, 0xC2A0), e.synth(0, 0xC2B0)
e.pairwise("and", a, b)
ref = hashlib.sha256(e.fetch().serialize()).hexdigest()[:16]
CONFIGS = [c.split(":") for c in os.environ.get(
    "CONFIGS", "base,1:0:1,2:0:1,4:0:1,8:0:1,4:3:1,8:3:1,4:0:2,8:0:4,16:0:1,16:3:2").split(",")]


def step(cfg):
    if cfg[0] == "base":
        e.pairwise("and", a, b)
        e.serialize()
    else:
        e.pairwise_serialized("and", a, b)


def setenv(cfg):
    if cfg[0] == "base":
        return
    k, pw, cp = cfg
    os.environ["RBG_SER_PIPE"] = k
    if pw != "0":
        os.environ["RBG_PIPE_PW_WG"] = pw
    else:
        os.environ.pop("RBG_PIPE_PW_WG", None)
    os.environ["RBG_PIPE_COPY_WG"] = cp


for rnd in range(2):
    for cfg in CONFIGS:
        setenv(cfg)
        for _ in range(5):
            step(cfg)
        e.sync()
        sha = hashlib.sha256(e.fetch().serialize()).hexdigest()[:16]
        t0 = time.perf_counter()
        for _ in range(N):
            step(cfg)
        e.sync()
        dt = (time.perf_counter() - t0) / N
        print(f"round={rnd} cfg={':'.join(cfg)} ms_per_step={dt * 1e3:.4f} input_GBps={0.717459586 / dt:.1f} "
              f"sha_ok={sha == ref}", flush=True)
