#!/usr/bin/env python3
"""Benchmark: pairwise AND of two full 2^32-universe bitmaps (BASELINE.json configs[1], "C2").

One step = RoaringBitmap.and(x1, x2) over a device-resident C2 pair (65,536 mixed
array/bitmap/run containers each, generated on the GPU), ending at the device-resident
serialized result: key plan, container kernel, result placement and the
portable serialization (RB/RoaringArray.java:896-940) are all inside the step.

Multi-GPU (python -m torch.distributed.run ... bench.py --gpus N): one process per
GPU.  At N > 1 the headline is ONE C2 pair's RoaringBitmap.and split into key ranges over
the ranks (strong scaling): each rank computes its key range, the shard
layout is all-gathered on the device (RCCL), every rank writes its slice at its global
place (shard.DeviceShard.place) and rank 0 receives every slice at its place
(DeviceShard.gather, point-to-point RCCL): the step ends, like N = 1, with the whole
serialized bitmap on GPU 0, whose sha is checked against the whole-pair result
(extra.c2_strong; its ms_per_step_without_gather is the step with the slices left in
each rank's HBM).  barrier + synchronize bracket the timed loop and the max time over
ranks is used.  extra.c2_and_weak keeps the weak-scaling form (an independent pair per
rank).  At N = 1, extra.rank_slice_ms times on this GPU what rank r of N = 2 / 4 / 8
does per step, for C2 and C3 uniform.

Prints ONE JSON line (rank 0).  Extra fields:
  roofline     - dominant kernel (container compute) achieved algorithmic GB/s vs
                 the 8 TB/s HBM peak, timed with HIP events on the engine's stream
  cpu_baseline - the CPU oracle (C++ restatement of the reference, not the JVM: no JDK here) on
                 this host, legs for C1-C5 (BASELINE.md §2 protocol: 5 warmup + 5 measured
                 iterations, median; ParallelAggregation legs on cores - 1 workers)
  extra        - per-phase times, container mix, result size, C3 (whole sharded op with the
                 result assembled on GPU 0), C4, C5, runOptimize, decode

`python bench.py --gpus N` without a launcher re-runs itself under torch.distributed.run with N
ranks; `--only W` runs one workload alone (per-workload rocprofv3 --pmc passes).
"""
import argparse
import hashlib
import json
import math
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)
# the one-GPU headline step as rbg_ctx_pairwise_serialized (RBG_BENCH_PIPE=1; default: the op, then the
# serialization -- measured faster than 2-16 pipelined key ranges)
PIPELINED = os.environ.get("RBG_BENCH_PIPE", "0") != "0"
PIPE_K = int(os.environ.get("RBG_SER_PIPE", "4"))  # key ranges when RBG_BENCH_PIPE=1
# the dense-range pairwise compute kernel: one 16-wave workgroup per CU
PW_KERNEL = "k_pair_cu"
METRIC = "wide-OR/pairwise-AND input GB/s + % of HBM peak at 1/2/4/8 MI355X"
EXTRA_STEPS, EXTRA_WARMUP = 20, 3  # floor of every extra's timed steps, and its warmups (independent of --steps)
SETTLE_S = float(os.environ.get("RBG_BENCH_SETTLE_S", "0.25"))  # device settle before the headline's warmups


def _pmc_traffic(key="k_pair_wave"):
    """Per-launch HBM bytes of a kernel from a committed rocprofv3 --pmc pass of that workload
    alone (profiles/pmc_traffic.json, written by scripts/summarize_prof.py)."""
    p = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    if not os.path.exists(p):
        return None
    try:
        with open(p) as f:
            return json.load(f).get(key, {}).get("hbm_bytes_per_launch")
    except Exception:
        return None


def _cpu_info():
    model = None
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    try:
        avail = len(os.sched_getaffinity(0))
    except AttributeError:
        avail = os.cpu_count()
    return {"nproc": os.cpu_count(), "affinity": avail, "model": model}


def c3_wide_or(eng, kind, n, rank, world, dist, steps, warmup, cdev, op="or", slices=None):
    """C3 wide OR (or AND) of n synthetic bitmaps, key-range sharded over the ranks.

    Each rank generates and reduces only its key slice (equal input bytes).  One step is the
    whole sharded op with its result assembled on rank 0's GPU as the portable bitmap:
    the slice's FastAggregation.or, the RCCL all-gather of the shard layout (containers,
    payload bytes, has_run), every rank writing its descriptors / global offsets / payload
    (rbg_ctx_fetch_shard_device) and rank 0 receiving each slice straight into its place
    (point-to-point RCCL).  At one GPU the same step writes the whole bitmap in place.
    Strong scaling: the 10,000-bitmap job is fixed.
    """
    import torch
    from roaringbitmap_amd import shard
    from roaringbitmap_amd.engine import synth_key_bytes
    seed = 0xC3000000
    # equal algorithmic input bytes per rank, for uniform and clustered alike
    ranges = shard.key_ranges(synth_key_bytes(kind, seed, n), world) if world > 1 else [(0, 65536)]
    lo, hi = ranges[rank]
    b = eng.synth(kind, seed, n, lo, hi)
    st = eng.batch_stats(b)
    in_bytes = st["payload_bytes"] + 4 * st["containers"]
    dev = torch.device("cuda", torch.cuda.current_device())
    comm = dev if cdev == "cuda" else torch.device("cpu")
    fill = shard.engine_fill(eng)

    def step():
        eng.wide(op, b, lo, hi)
        if dist is None:  # one GPU: the device serialization is the whole bitmap, no host round trip
            eng.serialize()
            return None, None
        rs = eng.result_stats()
        lay = shard.exchange_layout(rs["containers"], rs["payload_bytes"], rs["has_run"], device=comm)
        return shard.assemble(fill, lay, rank, fill_device=dev, comm_device=comm, sync=eng.sync), lay

    for _ in range(warmup):
        out, lay = step()
    torch.cuda.synchronize()
    rs = eng.result_stats()
    out_bytes = rs["payload_bytes"] + 4 * rs["containers"]
    total_bytes = lay.nbytes if lay is not None else shard.header_size(rs["containers"], rs["has_run"]) + \
        rs["payload_bytes"]
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        out, lay = step()
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    wall = time.perf_counter() - t0
    eng.profile(steps)
    for _ in range(steps):
        eng.wide(op, b, lo, hi)
    k, ph = eng.profile_read()
    rd_bytes = eng.profile_bytes() / max(k, 1)  # workShyAnd: what the early-exit chains read per launch
    eng.profile(0)
    kern_ms = ph[1] / max(k, 1)
    t = torch.tensor([wall, float(in_bytes), float(out_bytes)], dtype=torch.float64, device=comm)
    if dist is not None:
        tm = t.clone()
        dist.all_reduce(tm[:1], op=dist.ReduceOp.MAX)
        dist.all_reduce(t[1:], op=dist.ReduceOp.SUM)
        t[0] = tm[0]
    wall, tin, tout = float(t[0]), float(t[1]), float(t[2])
    if slices is not None:  # one GPU: rank r of N's share of this job (rank_slices)
        kb = synth_key_bytes(kind, seed, n)
        slices.update(rank_slices(eng, lambda lo_, hi_: eng.wide(op, b, lo_, hi_),
                                  lambda nr: shard.key_ranges(kb, nr), steps, warmup))
    eng.release(b)
    ms = wall / steps * 1e3
    ach = (in_bytes + out_bytes) / (kern_ms / 1e3) / 1e9
    tkey = f"k_wide<OR>_{'uniform' if kind == 1 else 'clustered'}"
    return {"workload": f"C3 {'uniform' if kind == 1 else 'clustered'}: FastAggregation.{op} of {n} synthetic bitmaps, "
                        f"key-range sharded over {world} GPU(s), result assembled on GPU 0",
            **({"input_GBps": round(tin / (wall / steps) / 1e9, 1)} if op == "or" else {}),
            "ms_per_step": round(ms, 4), "input_bytes": int(tin), "output_bytes": int(tout),
            "result_serialized_bytes": int(total_bytes), "containers_in": st["containers"], "rank0_keys": [lo, hi],
            "roofline_rank0": ({"kernel": "k_wide<OR>", "achieved_GBps": round(ach, 1),
                                "frac": round(ach / HBM_PEAK_GBS, 4), "kernel_ms": round(kern_ms, 4),
                                "traffic": _pmc_traffic(tkey),
                                # the bytes the counters saw (the algorithmic input counts 4 B descriptors
                                # that the key-major packed kernel never reads)
                                **({"counter_GBps": round(_pmc_traffic(tkey) / (kern_ms / 1e3) / 1e9, 1),
                                    "counter_frac": round(_pmc_traffic(tkey) / (kern_ms / 1e3) / 1e9 / HBM_PEAK_GBS,
                                                          4)} if _pmc_traffic(tkey) and world == 1 else {})}
                               if op == "or" else
                               {"kernel": "k_wide<AND_SHY>", "kernel_ms": round(kern_ms, 4),
                                # per key the chain stops at an empty intersection: the bytes it read
                                # (payload + 4 B per container, counted by the kernel in the profiled
                                # pass) are the algorithmic input of this launch, not input_bytes
                                "bytes_read_per_launch": int(rd_bytes),
                                "achieved_GBps": round((rd_bytes + out_bytes) / (kern_ms / 1e3) / 1e9, 1),
                                "frac": round((rd_bytes + out_bytes) / (kern_ms / 1e3) / 1e9 / HBM_PEAK_GBS, 4)})}


def rank_slices(eng, run_range, ranges_of, steps, warmup):
    """SURVEY §8(e) projected on one GPU: for N = 2, 4, 8 ranks, what rank r of a key-sharded op does per
    step -- its key range's op (run_range(lo, hi)), the result layout into a device tensor
    (rbg_ctx_result_layout_device) and its slice written at its global place from the global layout
    (rbg_ctx_fetch_shard_device_dyn) -- timed rank by rank on this GPU (wall clock, >= `steps` steps after
    `warmup`), with the compute kernel's own share from the engine's events.  The global layout is the
    one the all-gather would deliver (every range run once first).  Left out: the layout all-gather
    (3 int64 per rank) and rank 0's receive of the other slices (xGMI), which one GPU cannot time.
    -> {N: {"max_rank_ms", "per_rank_ms", "per_rank_compute_ms", "ranges"}}"""
    import torch
    from roaringbitmap_amd import shard
    dev = torch.device("cuda", torch.cuda.current_device())
    out = torch.empty(shard.MAX_SERIALIZED, dtype=torch.uint8, device=dev)
    runb = torch.empty(shard.KEYS, dtype=torch.uint8, device=dev)
    lay_local = torch.zeros(3, dtype=torch.int64, device=dev)
    rows = {}
    for n in (2, 4, 8):
        ranges = ranges_of(n)
        lay = torch.zeros(3 * n, dtype=torch.int64, device=dev)
        torch.cuda.synchronize(dev)  # the allocations' fills before any engine-stream write
        for r, (lo, hi) in enumerate(ranges):
            run_range(lo, hi)
            eng.result_layout_device(lay[3 * r: 3 * r + 3])
        eng.sync()
        per, comp = [], []
        for r, (lo, hi) in enumerate(ranges):
            def step():
                run_range(lo, hi)
                eng.result_layout_device(lay_local)
                eng.fetch_shard_device_dyn(lay, r, n, out, runb)
            for _ in range(warmup):
                step()
            eng.sync()
            t0 = time.perf_counter()
            for _ in range(steps):
                step()
            eng.sync()
            per.append(round((time.perf_counter() - t0) / steps * 1e3, 4))
            eng.profile(steps)
            for _ in range(steps):
                run_range(lo, hi)
            k, ph = eng.profile_read()
            eng.profile(0)
            comp.append(round(ph[1] / max(k, 1), 4))
        rows[str(n)] = {"max_rank_ms": max(per), "per_rank_ms": per, "per_rank_compute_ms": comp,
                        "ranges": [list(x) for x in ranges]}
    return rows


def c3_uniform_decoded(eng, n, steps, warmup):
    """FastAggregation.or over C3 uniform bitmaps that arrive as serialized bytes (what the Java class or an
    ImmutableRoaringBitmap buffer uploads) against the same bitmaps generated on the device: the wide OR +
    serialization step, input GB/s per layout -- the synthetic packed batch, the decoded batch with its
    array payloads packed as in the portable format (rbg_ctx_load_packed, the wide ops' load) and the
    decoded batch with 16 B slots (rbg_ctx_load).  n bitmaps over all 65,536 keys (host memory bounds n)."""
    sb = eng.synth(1, 0xC3000000, n)
    st = eng.batch_stats(sb)
    in_bytes = st["payload_bytes"] + 4 * st["containers"]
    bufs = [x.serialize() for x in eng.batch_fetch_range(sb)]
    t0 = time.perf_counter()
    pk = eng.load(bufs, packed=True)
    load_s = time.perf_counter() - t0
    pd = eng.load(bufs)
    del bufs
    out = {"workload": f"FastAggregation.or + serialize of {n} C3 uniform bitmaps (all 65,536 keys), device batch "
                       f"generated vs decoded from the serialized bytes", "input_bytes": int(in_bytes),
           "load_packed_s_pcie_included": round(load_s, 3)}
    sha = None
    for name, b in (("synthetic", sb), ("decoded_packed", pk), ("decoded_slots", pd)):
        for _ in range(warmup):
            eng.wide("or", b)
            eng.serialize()
        eng.sync()
        t0 = time.perf_counter()
        for _ in range(steps):
            eng.wide("or", b)
            eng.serialize()
        eng.sync()
        dt = (time.perf_counter() - t0) / steps
        eng.profile(steps)
        for _ in range(steps):
            eng.wide("or", b)
        k, ph = eng.profile_read()
        eng.profile(0)
        h = hashlib.sha256(eng.fetch().serialize()).hexdigest()[:16]
        sha = sha or h
        out[name] = {"ms_per_step": round(dt * 1e3, 4), "input_GBps": round(in_bytes / dt / 1e9, 1),
                     "kernel_ms": round(ph[1] / max(k, 1), 4), "result_sha16": h, "same_result": h == sha}
        eng.release(b)
    out["decoded_packed_vs_synthetic"] = round(out["decoded_packed"]["input_GBps"] / out["synthetic"]["input_GBps"], 4)
    out["decoded_slots_vs_synthetic"] = round(out["decoded_slots"]["input_GBps"] / out["synthetic"]["input_GBps"], 4)
    return out


def c2_weak(rank, world, dist, steps, warmup, cdev):
    """The weak-scaling form of the headline: every rank ANDs its own C2 pair (seeds offset by the
    rank) with the serialization, no data-path collective; max time over ranks."""
    import torch
    from roaringbitmap_amd import Engine
    e = Engine(torch.cuda.current_device())
    try:
        a = e.synth(0, 0xC2A0 + 0x10000 * rank)
        b = e.synth(0, 0xC2B0 + 0x10000 * rank)
        sa, sb = e.batch_stats(a), e.batch_stats(b)
        in_bytes = sa["payload_bytes"] + sb["payload_bytes"] + 4 * (sa["containers"] + sb["containers"])
        for _ in range(warmup):
            e.pairwise("and", a, b)
            e.serialize()
        e.sync()
        if dist is not None:
            dist.barrier()
        t0 = time.perf_counter()
        for _ in range(steps):
            e.pairwise("and", a, b)
            e.serialize()
        e.sync()
        if dist is not None:
            dist.barrier()
        t = torch.tensor([time.perf_counter() - t0, float(in_bytes)], dtype=torch.float64, device=cdev)
        if dist is not None:
            tm = t.clone()
            dist.all_reduce(tm[:1], op=dist.ReduceOp.MAX)
            dist.all_reduce(t[1:], op=dist.ReduceOp.SUM)
            t[0] = tm[0]
        e.release(a)
        e.release(b)
    finally:
        e.close()
    step = float(t[0]) / steps
    return {"workload": f"C2 RoaringBitmap.and + serialization, an independent pair per GPU ({world} GPUs)",
            "input_GBps": round(float(t[1]) / step / 1e9, 1), "ms_per_step": round(step * 1e3, 4), "scaling": "weak"}


def c2_two_streams(eng, a, b, in_bytes, steps, warmup):
    """The headline op (RoaringBitmap.and + serialization) as a stream of independent calls on two
    engine contexts, alternating: each context has its own HIP stream and device state."""
    import torch
    from roaringbitmap_amd import Engine
    e2 = Engine(torch.cuda.current_device())
    try:
        a2 = e2.synth(0, 0xC2A0 + 0x10000 * int(os.environ.get("RANK", "0")))
        b2 = e2.synth(0, 0xC2B0 + 0x10000 * int(os.environ.get("RANK", "0")))
        ctx = [(eng, a, b), (e2, a2, b2)]
        for i in range(warmup * 2):
            e, x, y = ctx[i % 2]
            e.pairwise("and", x, y)
            e.serialize()
        eng.sync()
        e2.sync()
        t0 = time.perf_counter()
        for i in range(2 * steps):
            e, x, y = ctx[i % 2]
            e.pairwise("and", x, y)
            e.serialize()
        eng.sync()
        e2.sync()
        dt = (time.perf_counter() - t0) / (2 * steps)
        e2.release(a2)
        e2.release(b2)
    finally:
        e2.close()
    return {"workload": "C2 RoaringBitmap.and + serialization, independent calls alternating on two engine contexts "
                        "(two HIP streams)", "ms_per_op": round(dt * 1e3, 4),
            "input_GBps": round(in_bytes / dt / 1e9, 1)}


def c4_batch_and_card(eng, n_pairs, rank, world, dist, steps, warmup, cdev):
    """C4: batched andCardinality of n_pairs small sparse pairs per rank (weak scaling)."""
    import torch
    b = eng.synth(3, 0xC4 + 0x10000 * rank, n_pairs)
    matched, allb = eng.pair_bytes(b)
    for _ in range(warmup):
        eng.batch_and_card(b)
    eng.sync()
    if dist is not None:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(steps):
        eng.batch_and_card(b)
    eng.sync()
    if dist is not None:
        dist.barrier()
    wall = time.perf_counter() - t0
    t = torch.tensor([wall, float(n_pairs), float(matched)], dtype=torch.float64, device=cdev)
    if dist is not None:
        tm = t.clone()
        dist.all_reduce(tm[:1], op=dist.ReduceOp.MAX)
        dist.all_reduce(t[1:], op=dist.ReduceOp.SUM)
        t[0] = tm[0]
    step = float(t[0]) / steps
    eng.release(b)
    return {"workload": f"C4: batched RoaringBitmap.andCardinality of {n_pairs} small sparse pairs per GPU",
            "pairs_per_s": round(float(t[1]) / step, 1), "ms_per_step": round(step * 1e3, 4),
            "input_GBps": round(float(t[2]) / step / 1e9, 1), "input_bytes_per_rank": matched,
            "all_bytes_per_rank": allb}


def decode_c2(eng, a, steps):
    """Upload + device decode of one serialized C2 operand (Engine.load: pinned staging, one H2D
    copy, header parse, key sort, slot placement, payload copy); wall time per load."""
    x = eng.batch_fetch(a).serialize()
    for _ in range(EXTRA_WARMUP):
        eng.release(eng.load([x]))
    t0 = time.perf_counter()
    for _ in range(steps):
        b = eng.load([x])
        eng.release(b)
    dt = (time.perf_counter() - t0) / steps
    return {"workload": "Engine.load of one serialized C2 operand (65,536 containers), PCIe included",
            "ms_per_load": round(dt * 1e3, 4), "serialized_MB": round(len(x) / 1e6, 2),
            "GBps": round(len(x) / dt / 1e9, 2)}


def c2_oneshot(eng, a, b, steps):
    """The drop-in path a JNI caller takes (rbg_pairwise, RB/RoaringBitmap.java:377 with
    serialize / deserialize at the boundary, :3017-3019 / :1805-1811): the two serialized C2
    operands from host memory to the serialized result in host memory, PCIe included, timed at
    the C ABI (ctypes calls on the bytes, rbg_free of the result: no Python-side copy).  Split,
    through the same calls of a session context: the upload + device decode of both operands
    (rbg_ctx_load_separate), the op with its serialization, and the download (rbg_ctx_fetch)."""
    import ctypes
    from roaringbitmap_amd import _lib
    from roaringbitmap_amd._lib import check
    L = _lib.lib()
    xa = eng.batch_fetch(a).serialize()
    xb = eng.batch_fetch(b).serialize()
    out = _lib.rbg_buffer()

    def one():
        check(L.rbg_pairwise(0, xa, len(xa), xb, len(xb), ctypes.byref(out)))
        n = out.len
        L.rbg_free(ctypes.byref(out))
        return n

    n_out = one()  # warm the one-shot context (staging and result buffers)
    for _ in range(EXTRA_WARMUP - 1):
        one()
    t0 = time.perf_counter()
    for _ in range(steps):
        one()
    per_call = (time.perf_counter() - t0) / steps
    arr, lens = _lib.buf_array([xa, xb])
    ids = (ctypes.c_int32 * 2)()

    def split():
        t1 = time.perf_counter()
        check(L.rbg_ctx_load_separate(eng._ctx, arr, lens, 2, ids))
        t2 = time.perf_counter()
        check(L.rbg_ctx_pairwise(eng._ctx, 0, ids[0], 0, ids[1], 0))
        check(L.rbg_ctx_serialize(eng._ctx))
        check(L.rbg_ctx_sync(eng._ctx))
        t3 = time.perf_counter()
        check(L.rbg_ctx_fetch(eng._ctx, ctypes.byref(out)))
        t4 = time.perf_counter()
        L.rbg_free(ctypes.byref(out))
        check(L.rbg_ctx_release(eng._ctx, ids[0]))
        check(L.rbg_ctx_release(eng._ctx, ids[1]))
        return t2 - t1, t3 - t2, t4 - t3

    split()  # warm the session's staging buffers at the pair's size
    tt = [0.0, 0.0, 0.0]
    for _ in range(steps):
        for i, x in enumerate(split()):
            tt[i] += x
    n = float(steps)
    return {"workload": "rbg_pairwise(AND) from host bytes to host bytes on the C2 pair (PCIe included), "
                        "timed at the C ABI",
            "ms_per_call": round(per_call * 1e3, 3), "input_MB": round((len(xa) + len(xb)) / 1e6, 1),
            "output_MB": round(n_out / 1e6, 1),
            "split_ms": {"upload_decode_both": round(tt[0] / n * 1e3, 3), "op_serialize": round(tt[1] / n * 1e3, 3),
                         "download": round(tt[2] / n * 1e3, 3)},
            "pcie_inclusive_input_GBps": round((len(xa) + len(xb)) / per_call / 1e9, 2)}


def pq_or_queue(eng, rows, steps):
    """FastAggregation.priorityqueue_or (RB/FastAggregation.java:737-781) over the 32 bitmaps of a
    synthetic bit-sliced index of `rows` rows (C5's generator: ebM as full run containers, 31
    slices of bitmaps), device-resident: the size-ordered queue runs on the device, one launch per
    queue step (a batch without run containers skips the queue -- its bytes are
    naive_or's -- so this input keeps the runs).  Latency-bound (a chain of dependent loads per
    key and a serial plan per step): time per queue step, no roofline."""
    b = eng.synth(4, 0xC5000000, rows)
    try:
        st = eng.batch_stats(b)
        n = st["bitmaps"]
        for _ in range(EXTRA_WARMUP):
            eng.wide("priorityqueue_or", b)
        eng.sync()
        t0 = time.perf_counter()
        for _ in range(steps):
            eng.wide("priorityqueue_or", b)
            eng.sync()
        ms = (time.perf_counter() - t0) / steps * 1e3
        rs = eng.result_stats()
        for _ in range(EXTRA_WARMUP):
            eng.wide("or", b)
        eng.sync()
        t0 = time.perf_counter()
        for _ in range(steps):
            eng.wide("or", b)
            eng.sync()
        naive_ms = (time.perf_counter() - t0) / steps * 1e3
    finally:
        eng.release(b)
    return {"workload": f"FastAggregation.priorityqueue_or of the {n} bitmaps of a {rows}-row synthetic BSI "
                        f"({st['containers']} containers, {st['run']} runs; one GPU)",
            "ms_per_op": round(ms, 3), "queue_steps": n - 1, "us_per_step": round(ms * 1e3 / max(n - 1, 1), 2),
            "result_containers": rs["containers"], "naive_or_ms_same_input": round(naive_ms, 4)}


def run_optimize_c2(eng, a, sa, steps):
    """RoaringBitmap.runOptimize of one C2 operand on the device (plan, scan, write into a new
    batch); wall time per call with the new batch's allocation (pooled) included.  The new batch's
    statistics stay on the device (no host read-back inside the loop); one sync ends the loop."""
    o, _ = eng.run_optimize(a)
    so = eng.batch_stats(o)
    eng.release(o)
    for _ in range(EXTRA_WARMUP - 1):
        o, _ = eng.run_optimize(a, answers=False)
        eng.release(o)
    eng.sync()
    t0 = time.perf_counter()
    for _ in range(steps):
        o, _ = eng.run_optimize(a, answers=False)
        eng.release(o)
    eng.sync()
    dt = (time.perf_counter() - t0) / steps
    return {"workload": "RoaringBitmap.runOptimize of one C2 operand (65,536 containers)",
            "ms_per_call": round(dt * 1e3, 4), "input_GBps": round(sa["payload_bytes"] / dt / 1e9, 1),
            "types_before": [sa["array"], sa["bitmap"], sa["run"]],
            "types_after": [so["array"], so["bitmap"], so["run"]]}


def ornot_c2(eng, a, b, sa, sb, steps):
    """RoaringBitmap.orNot(x1, x2, 2^32) on the C2 pair (every key holds both operands: c1.or(c2.not(0,
    65536)) per key) + the device serialization, as the headline step; the orNot launches' own device time
    from the engine's phase events (k_ornot_scan + k_plan_ornot + k_ornot)."""
    end = 1 << 32
    eng.ornot(a, b, end)
    rs = eng.result_stats()
    for _ in range(EXTRA_WARMUP):
        eng.ornot(a, b, end)
        eng.serialize()
    eng.sync()
    t0 = time.perf_counter()
    for _ in range(steps):
        eng.ornot(a, b, end)
        eng.serialize()
    eng.sync()
    dt = (time.perf_counter() - t0) / steps
    eng.profile(steps)
    for _ in range(steps):
        eng.ornot(a, b, end)
    n, ph = eng.profile_read()
    eng.profile(0)
    k_ms = ph[1] / max(n, 1)
    in_b = sa["payload_bytes"] + sb["payload_bytes"] + 4 * (sa["containers"] + sb["containers"])
    out_b = rs["payload_bytes"] + 4 * rs["containers"]
    return {"workload": "RoaringBitmap.orNot(x1, x2, 2^32) on the C2 pair + serialize (device-resident)",
            "ms_per_step": round(dt * 1e3, 4), "input_GBps": round(in_b / dt / 1e9, 1),
            "result_containers": rs["containers"], "result_payload_bytes": rs["payload_bytes"],
            "roofline": {"kernel": "k_ornot_scan + k_plan_ornot + k_ornot", "kernel_ms": round(k_ms, 4),
                         "bytes": int(in_b + out_b),
                         "achieved_GBps": round((in_b + out_b) / (k_ms / 1e3) / 1e9, 1) if k_ms > 0 else None,
                         "frac": round((in_b + out_b) / (k_ms / 1e3) / 1e9 / HBM_PEAK_GBS, 4) if k_ms > 0 else None}}


def c5_bsi(eng, rows, rank, world, dist, steps, warmup, cdev):
    """C5: RoaringBitmapSliceIndex.compare(RANGE) + sum over `rows` rows (31 slices),
    rows sharded by key range across the ranks (strong scaling); one step = the fused
    compare + sum pass + the (sum, count) all-reduce."""
    import torch
    nkeys = (rows + 65535) // 65536
    lo_k, hi_k = (nkeys * rank) // world, (nkeys * (rank + 1)) // world
    b = eng.synth(4, 0xC5, rows, lo_k, hi_k)
    st = eng.batch_stats(b)
    mn, mx = eng.batch_minmax(b)
    mm = torch.tensor([mn, -mx], dtype=torch.int64, device=cdev)
    if dist is not None:
        dist.all_reduce(mm, op=dist.ReduceOp.MIN)  # the BSI's min / max are global
    mn, mx = int(mm[0]), -int(mm[1])
    lo, hi = 1 << 29, 1 << 30
    # sum(found) stays on the device: (sum, count) copied into a device tensor on the engine
    # stream and all-reduced from there (RCCL); no host read inside the step
    ext = torch.cuda.ExternalStream(eng.stream_ptr)
    sums = torch.zeros(2, dtype=torch.int64, device=torch.device("cuda", torch.cuda.current_device()))

    eng.bsi_sums_target(sums)  # (sum, count) written into `sums` by the kernel that sums

    def step():
        ext.wait_stream(torch.cuda.current_stream())  # the last step's all-reduce has read `sums`
        eng.bsi(b, "RANGE", 31, lo, hi, mn, mx, want_sum=True)
        if dist is not None:
            torch.cuda.current_stream().wait_stream(ext)
            if cdev == "cuda":
                dist.all_reduce(sums)
            else:  # gloo rehearsal: the collective runs on host memory
                t = sums.cpu()
                dist.all_reduce(t)
                sums.copy_(t)

    for _ in range(warmup):
        step()
    torch.cuda.synchronize()
    eng.sync()
    if dist is not None:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    eng.sync()
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    wall = time.perf_counter() - t0
    eng.bsi_sums_target(None)
    sc = (int(sums[0]), int(sums[1]))
    ein = st["payload_bytes"] + 4 * st["containers"]
    t = torch.tensor([wall, float(ein)], dtype=torch.float64, device=cdev)
    if dist is not None:
        tm = t.clone()
        dist.all_reduce(tm[:1], op=dist.ReduceOp.MAX)
        dist.all_reduce(t[1:], op=dist.ReduceOp.SUM)
        t[0] = tm[0]
    step_s = float(t[0]) / steps
    eng.release(b)
    # compare + sum read ebM and every slice once (k_bsi_reg holds a key's slices in registers)
    return {"workload": f"C5: RoaringBitmapSliceIndex.compare(RANGE, 2^29, 2^30) + sum over {rows} rows x 31 slices, "
                        f"key-range sharded over {world} GPU(s)",
            "rows_per_s": round(rows / step_s, 1), "ms_per_step": round(step_s * 1e3, 4),
            "index_bytes": int(t[1]), "index_GBps": round(float(t[1]) / step_s / 1e9, 1),
            "frac_of_peak_1pass": round(float(t[1]) / step_s / 1e9 / HBM_PEAK_GBS, 4),
            "traffic_k_bsi_reg": _pmc_traffic("k_bsi_reg"),
            "sum_count": list(sc), "min_max": [mn, mx]}


def _median_of(fn, target_s):
    """BASELINE.md §2 protocol (the JMH settings of jmh/build.gradle.kts:53-58): 5 warmup + 5
    measured iterations, median.  One iteration runs fn(reps) with reps sized so that it takes
    about target_s; returns (seconds per single run, reps)."""
    t1 = max(fn(1), 1e-6)
    reps = max(1, int(round(target_s / t1)))
    for _ in range(5):
        fn(reps)
    times = sorted(fn(reps) for _ in range(5))
    return times[2] / reps, reps


def cpu_baselines(eng, a, b, in_bytes, budget_s):
    """CPU legs on this host (rank 0, N=1), one per BASELINE.json config, with the BASELINE.md §2
    protocol (5 warmup + 5 measured iterations, median).  The reference JVM path is probed for
    (`java` on PATH); this image has none, so every leg is the oracle's C++ restatement of the
    reference: FastAggregation / RoaringBitmap semantics on one thread, and ParallelAggregation's
    key-parallel semantics (RB/ParallelAggregation.java:171-173) on cores - 1 workers, the
    ForkJoin common pool's default parallelism.  Each leg runs on a bounded sample of its
    workload (stated per leg)."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import shutil

    import numpy as np

    import _oracle as O  # CPU baseline leg only
    info = _cpu_info()
    java = shutil.which("java")
    threads = max(1, (info["affinity"] or 1) - 1)
    n_legs = 13
    target = budget_s / (n_legs * 11.0)  # 11 iterations per leg (calibration + 5 + 5)
    legs = {}

    def leg(name, fn, nbytes, thr, what, **kw):
        sec, reps = _median_of(fn, target)
        legs[name] = {"GBps": round(nbytes / sec / 1e9, 3), "ms": round(sec * 1e3, 3), "threads": thr,
                      "reps_per_iter": reps, "what": what, **kw}

    def algo_bytes(bufs):
        n = p = 0
        for x in bufs:
            st = O.stats(x)
            n += st["array"] + st["bitmap"] + st["run"]
            p += st["payload"]
        return p + 4 * n

    # C1: census1881 (200 bitmaps, bitmapOf + runOptimize as RealDataBenchmarkState), FastAggregation.or
    # and the pairwise and / andCardinality loops k = 0..198 of the jmh realdata benchmarks
    z = np.load(os.path.join(ROOT, "tests", "golden", "realdata", "census1881.npz"))
    vals, offs = z["values"], z["offsets"]
    c1 = [O.from_values(vals[offs[i]:offs[i + 1]], True) for i in range(len(offs) - 1)]
    c1_bytes = algo_bytes(c1)
    pairs = [x for k in range(len(c1) - 1) for x in (c1[k], c1[k + 1])]
    leg("c1_census_or_1t", lambda r: O.time_wide("or", c1, r), c1_bytes, 1,
        "FastAggregation.or of the 200 census1881 bitmaps (runOptimize'd)")
    leg("c1_census_and_1t", lambda r: O.time_pairs("and", pairs, 1, r), algo_bytes(pairs), 1,
        "RoaringBitmap.and(b[k], b[k+1]).getCardinality(), k = 0..198 (census1881)")
    leg("c1_census_andcard_1t", lambda r: O.time_pairs("and_card", pairs, 1, r), algo_bytes(pairs), 1,
        "RoaringBitmap.andCardinality(b[k], b[k+1]), k = 0..198 (census1881)")
    # C2: the headline pair itself
    xa = eng.batch_fetch(a).serialize()
    xb = eng.batch_fetch(b).serialize()
    leg("c2_and_1t", lambda r: O.time_pairwise("and", xa, xb, r), in_bytes, 1,
        "RoaringBitmap.and(x1, x2) on the full C2 pair")
    leg("c2_and_mt", lambda r: O.time_and_parallel(xa, xb, threads, r), in_bytes, threads,
        f"key-parallel RoaringBitmap.and over {threads} key ranges, full C2 pair")
    # C3: all 10,000 bitmaps restricted to a key sample (uniform: 128 keys; clustered: 512 keys) on one
    # thread; ParallelAggregation.or over the whole clustered job (1.3 GB) and the uniform sample (the
    # whole uniform job is 22 GB)
    for kind, name, keys in ((1, "uniform", 128), (2, "clustered", 512)):
        sb = eng.synth(kind, 0xC3000000, 10000, 0, keys)
        st = eng.batch_stats(sb)
        sbytes = st["payload_bytes"] + 4 * st["containers"]
        bufs = [x.serialize() for x in eng.batch_fetch_range(sb)]
        eng.release(sb)
        leg(f"c3_{name}_or_1t_sample", lambda r: O.time_wide("or", bufs, r), sbytes, 1,
            f"FastAggregation.or of 10,000 C3 {name} bitmaps, keys [0, {keys})")
        if kind == 1:
            leg(f"c3_{name}_or_mt_sample", lambda r: O.time_wide_parallel("or", bufs, threads, r), sbytes, threads,
                f"ParallelAggregation.or (key groups over {threads} workers), same sample")
        del bufs
    sb = eng.synth(2, 0xC3000000, 10000)
    st = eng.batch_stats(sb)
    sbytes = st["payload_bytes"] + 4 * st["containers"]
    bufs = [x.serialize() for x in eng.batch_fetch_range(sb)]
    eng.release(sb)
    leg("c3_clustered_or_mt", lambda r: O.time_wide_parallel("or", bufs, threads, r), sbytes, threads,
        f"ParallelAggregation.or (key groups over {threads} workers) of the whole C3 clustered job "
        f"(10,000 bitmaps, {sbytes / 1e9:.2f} GB)")
    del bufs
    # C4: the first 65,536 of the million pairs (same generator, seed 0xC4)
    n4 = 65536
    sb = eng.synth(3, 0xC4, n4)
    matched, _ = eng.pair_bytes(sb)
    bufs = [x.serialize() for x in eng.batch_fetch_range(sb)]
    eng.release(sb)
    leg("c4_andcard_1t", lambda r: O.time_pairs("and_card", bufs, 1, r), matched, 1,
        f"loop of RoaringBitmap.andCardinality over {n4} C4 pairs (seed 0xC4)", pairs_per_s=None)
    legs["c4_andcard_1t"]["pairs_per_s"] = round(n4 / (legs["c4_andcard_1t"]["ms"] / 1e3), 1)
    leg("c4_andcard_mt", lambda r: O.time_pairs("and_card", bufs, threads, r), matched, threads,
        f"the same loop split over {threads} workers")
    legs["c4_andcard_mt"]["pairs_per_s"] = round(n4 / (legs["c4_andcard_mt"]["ms"] / 1e3), 1)
    del bufs
    # C5: the 10^9-row column's first 16 keys (1,048,576 rows), ebM + 31 slices, on one thread; the
    # whole column key-parallel
    sb = eng.synth(4, 0xC5, 16 * 65536, 0, 16)
    st = eng.batch_stats(sb)
    sbytes = st["payload_bytes"] + 4 * st["containers"]
    bufs = [x.serialize() for x in eng.batch_fetch_range(sb)]
    eng.release(sb)
    lo, hi = 1 << 29, 1 << 30
    leg("c5_bsi_range_sum_1t_sample", lambda r: O.time_bsi_range_sum(bufs[0], bufs[1:], lo, hi, r)[0], sbytes, 1,
        "RoaringBitmapSliceIndex.compare(RANGE, 2^29, 2^30) + sum, rows [0, 2^20) (16 keys x 31 slices)")
    legs["c5_bsi_range_sum_1t_sample"]["rows_per_s"] = round(
        16 * 65536 / (legs["c5_bsi_range_sum_1t_sample"]["ms"] / 1e3), 1)
    del bufs
    rows5 = 10 ** 9
    sb = eng.synth(4, 0xC5, rows5)
    st = eng.batch_stats(sb)
    sbytes = st["payload_bytes"] + 4 * st["containers"]
    bufs = [x.serialize() for x in eng.batch_fetch_range(sb)]
    eng.release(sb)
    leg("c5_bsi_range_sum_mt", lambda r: O.time_bsi_range_sum_parallel(bufs[0], bufs[1:], lo, hi, threads, r)[0],
        sbytes, threads, f"the same query over all {rows5} rows ({st['containers']} containers), key ranges over "
                         f"{threads} workers (per-key sums added before sum's int cast)")
    legs["c5_bsi_range_sum_mt"]["rows_per_s"] = round(rows5 / (legs["c5_bsi_range_sum_mt"]["ms"] / 1e3), 1)
    legs["c5_bsi_range_sum_mt"]["sum_count"] = list(O.time_bsi_range_sum_parallel(bufs[0], bufs[1:], lo, hi,
                                                                                  threads, 1)[1])
    del bufs
    best = legs["c2_and_mt"]
    return {"value": best["GBps"], "unit": "GB/s", "cores": best["threads"], "kind": "port",
            "sample": f"full C2 pair (same bytes as the GPU step): key-parallel RoaringBitmap.and on {best['threads']} "
                      f"threads (cores - 1, the ForkJoin common-pool default) of the C++ restatement oracle/rbcpu, "
                      f"median of 5 after 5 warmup iterations -- C++ restatement, not the reference JVM "
                      f"(java on this host: {java})",
            "java": java, "protocol": "5 warmup + 5 measured iterations, median (BASELINE.md §2)",
            "host": info, "legs": legs}


def _relaunch(args):
    """`bench.py --gpus N` without a launcher: run N ranks under torch.distributed.run as a
    child process (nothing has touched the GPU yet) and exit with its status."""
    import socket
    import subprocess
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY=os.environ.get("HSA_ENABLE_IPC_MODE_LEGACY", "0"))
    sys.exit(subprocess.call(cmd, env=env))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    # 200 timed steps: the loop's fixed cost (the closing stream sync and barrier, ~0.3 ms) is then 1.5 us of
    # a 0.32 ms step instead of 15 us at 20 steps
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--cpu-seconds", type=float, default=24.0, help="bounded CPU-baseline budget (all legs)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--c3-n", type=int, default=10000, help="bitmaps of the C3 wide-OR workloads (0 = skip)")
    ap.add_argument("--c4-pairs", type=int, default=1000000, help="pairs of the C4 workload per GPU (0 = skip)")
    ap.add_argument("--c5-rows", type=int, default=1000000000, help="rows of the C5 BSI workload (0 = skip)")
    ap.add_argument("--only", default="", help="profiling: run one workload alone (c2, c2card, c3u, c3c, c3u_and, c3c_and, c4, c5, runopt, ornot)")
    ap.add_argument("--backend", default="nccl", help="torch.distributed backend (nccl = RCCL; gloo to rehearse "
                                                       "several ranks on one GPU)")
    args = ap.parse_args()

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        _relaunch(args)
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus and rank == 0:
        print(f"bench: WORLD_SIZE={world} overrides --gpus {args.gpus}", file=sys.stderr)

    import torch
    ndev = torch.cuda.device_count()
    local = local % max(ndev, 1)  # rehearsal: several ranks may share one GPU (gloo)
    torch.cuda.set_device(local)
    dist = None
    cdev = "cuda"
    if world > 1:
        import torch.distributed as dist
        if args.backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(args.backend)
            cdev = "cpu"

    from roaringbitmap_amd import Engine

    eng = Engine(local)
    if args.only:
        _only(eng, args, rank, world, dist, cdev)
        if dist is not None:
            dist.destroy_process_group()
        return
    a = eng.synth(0, 0xC2A0)  # ONE pair: at N > 1 every rank holds it and computes its key range
    b = eng.synth(0, 0xC2B0)
    sa, sb = eng.batch_stats(a), eng.batch_stats(b)
    # algorithmic bytes: AND reads the descriptors of both operands and the
    # payload of matched pairs (every key matches here); writes the result payload + 4 B/container
    in_bytes = sa["payload_bytes"] + sb["payload_bytes"] + 4 * (sa["containers"] + sb["containers"])
    eng.pairwise("and", a, b)
    rs = eng.result_stats()
    out_bytes = rs["payload_bytes"] + 4 * rs["containers"]
    rs["sha16"] = hashlib.sha256(eng.fetch().serialize()).hexdigest()[:16]  # of the serialized result

    stream = torch.cuda.ExternalStream(eng.stream_ptr)
    strong = world > 1
    if strong:
        from roaringbitmap_amd import shard
        key_lo, key_hi = (65536 * rank) // world, (65536 * (rank + 1)) // world
        dshard = shard.DeviceShard(eng, rank, world, torch.device("cuda", local),
                                   torch.device("cuda", local) if cdev == "cuda" else "cpu")

        def c2_step():  # this rank's key range of ONE pair -> its slice at its global place -> one bitmap on GPU 0
            eng.pairwise("and", a, b, key_lo=key_lo, key_hi=key_hi)
            dshard.place()
            dshard.gather()  # rank 0 receives every slice at its place: the step ends, like N = 1, with one bitmap
    elif PIPELINED:
        def c2_step():  # RoaringBitmap.and(x1, x2) + serialize as one pipeline (rbg_ctx_pairwise_serialized):
            eng.pairwise_serialized("and", a, b)  # key range r placed and copied while range r + 1 computes
    else:
        def c2_step():  # RoaringBitmap.and(x1, x2) -> the device-resident serialized result
            eng.pairwise("and", a, b)
            eng.serialize()

    # Device settle before the warmups: ~0.25 s of the whole-pair op on this GPU, so that the timed steps run
    # at the clocks a sustained load holds.  With the driver's 5 warmups (1.6 ms) the first timed steps still
    # ran the compute kernel ~4 % slower (0.2205 against 0.2089 ms, --steps 20 on one box, round 6,
    # profiles/r06/experiments/bench_settle.txt).  Setup only, and local: no collective (each rank's clock
    # decides how many it runs), so at N > 1 the ranks cannot fall out of step; the W warmups and the K timed
    # steps that follow are unchanged.
    t_settle = time.perf_counter()
    while time.perf_counter() - t_settle < SETTLE_S:
        for _ in range(16):
            eng.pairwise("and", a, b)
            eng.serialize()
        eng.sync()
    for _ in range(args.warmup):
        c2_step()
    eng.sync()

    def barrier():
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize()

    barrier()
    ev0 = torch.cuda.Event(enable_timing=True)
    ev1 = torch.cuda.Event(enable_timing=True)
    # the compute kernel's device time over the timed region itself: the engine records two HIP events per
    # op on its own stream (the stream the kernel runs on), around the compute launch -- four per op (every
    # phase) added 8-9 us to each step (scripts/c2_events.py); the pipelined form keeps the phase events
    eng.profile(args.steps, compute_only=not PIPELINED)
    t0 = time.perf_counter()
    ev0.record(stream)
    for _ in range(args.steps):
        c2_step()
    ev1.record(stream)
    eng.sync()
    barrier()
    wall = time.perf_counter() - t0
    gpu_ms = ev0.elapsed_time(ev1)
    n_live, ph_live = eng.profile_read()
    eng.profile(0)
    ph_live = [x / max(n_live, 1) for x in ph_live]

    strong_info = None
    if strong:  # the step without its gather (slices left in each rank's HBM), and the gathered bitmap's sha
        ks_g = max(EXTRA_STEPS, args.steps // 4)
        barrier()
        tg = time.perf_counter()
        for _ in range(ks_g):
            eng.pairwise("and", a, b, key_lo=key_lo, key_hi=key_hi)
            dshard.place()
        eng.sync()
        barrier()
        ng_ms = (time.perf_counter() - tg) / ks_g * 1e3
        out = dshard.gather()
        got = hashlib.sha256(bytes(out.cpu().numpy().tobytes())).hexdigest()[:16] if rank == 0 else None
        lay = dshard.layout()
        strong_info = {"workload": f"C2 RoaringBitmap.and of ONE pair, key-range sharded over {world} GPUs; the step "
                                   f"ends with the whole serialized bitmap on GPU 0 (slices placed on the device, the "
                                   f"layout all-gathered, every slice received by rank 0 at its place)",
                       "rank0_keys": [key_lo, key_hi], "ms_per_step_without_gather": round(ng_ms, 4),
                       "result_serialized_bytes": int(lay.nbytes), "result_sha16": got,
                       "sha_equals_whole_pair_result": (got == rs["sha16"]) if rank == 0 else None,
                       "layout_exchange": "device all-gather (RCCL)" if cdev == "cuda" else "gloo (host)"}

    # the serialization's own device time (events around it, on the engine's stream)
    ser_ms = 0.0
    for _ in range(args.steps):
        eng.pairwise("and", a, b)
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        eng.serialize()
        e1.record(stream)
        eng.sync()
        ser_ms += e0.elapsed_time(e1)
    ser_ms /= args.steps

    # per-phase device time of the op before serialization (separate pass: HIP events between
    # phases, on the engine's stream)
    eng.profile(args.steps)
    for _ in range(args.steps):
        eng.pairwise("and", a, b)
    n_ops, ph = eng.profile_read()
    eng.profile(0)
    ph_avg = [x / max(n_ops, 1) for x in ph]

    # the headline's cross-rank reduction first: the extras below cannot lose it
    t = torch.tensor([wall, float(in_bytes)], dtype=torch.float64, device=cdev)
    if dist is not None:
        tmax = t.clone()
        dist.all_reduce(tmax[:1], op=dist.ReduceOp.MAX)
        wall_max = float(tmax[0])
    else:
        wall_max = wall
    total_in = float(in_bytes)  # one pair, whatever the number of GPUs (strong scaling)

    extra = {}

    def run_extra(name, fn):
        # One GPU: an extra that raises is reported in its entry instead of ending the run
        # without the headline line.  Several ranks: it propagates -- a rank that stopped
        # inside an extra's collectives or point-to-point assembly would leave the others
        # blocked there; failing fast lets torch.distributed.run end the whole group.
        if world > 1:
            extra[name] = fn()
            return
        try:
            extra[name] = fn()
        except Exception as e:  # noqa: BLE001
            print(f"bench: extra {name} failed: {e!r}", file=sys.stderr)
            extra[name] = {"error": repr(e)}

    # RoaringBitmap.andCardinality on the same pair: the same input bytes,
    # no result containers
    for _ in range(args.warmup):
        eng.and_cardinality(a, b)
    eng.sync()
    t0c = time.perf_counter()
    for _ in range(args.steps):
        eng.and_cardinality(a, b)
    eng.sync()
    card_wall = (time.perf_counter() - t0c) / args.steps
    eng.profile(args.steps)
    for _ in range(args.steps):
        eng.and_cardinality(a, b)
    kc, phc = eng.profile_read()
    eng.profile(0)
    card_kern = phc[1] / max(kc, 1)
    extra["c2_and_cardinality"] = {
        "workload": "RoaringBitmap.andCardinality on the C2 pair (device-resident)",
        "ms_per_step": round(card_wall * 1e3, 4), "input_GBps": round(in_bytes / card_wall / 1e9, 1),
        "roofline": {"kernel": f"{PW_KERNEL}<AND, card>", "kernel_ms": round(card_kern, 4),
                     "achieved_GBps": round(in_bytes / (card_kern / 1e3) / 1e9, 1),
                     "frac": round(in_bytes / (card_kern / 1e3) / 1e9 / HBM_PEAK_GBS, 4),
                     "traffic": _pmc_traffic("k_pair_wave_card")}}
    ks = max(EXTRA_STEPS, args.steps // 4)  # every extra: >= 20 timed steps after EXTRA_WARMUP warmups
    # a stream of independent C2 ANDs issued alternately on two engine contexts (two HIP streams):
    # one op's serialization overlaps the next op's compute (throughput of concurrent calls, as a
    # server would issue them; the headline above is one call after another)
    run_extra("c2_and_two_streams", lambda: c2_two_streams(eng, a, b, in_bytes, args.steps, args.warmup))
    if strong:  # the weak-scaling form beside the key-sharded headline
        extra["c2_strong"] = strong_info
        run_extra("c2_and_weak", lambda: c2_weak(rank, world, dist, ks, EXTRA_WARMUP, cdev))
    # one GPU: what rank r of N = 2 / 4 / 8 does per step, for C2 (equal key ranges, as the strong headline)
    # and C3 uniform (equal input bytes): the fixed costs that cap a speed-up before an 8-GPU node exists
    slices = {"c3_uniform_or": {}} if world == 1 else None
    if world == 1:
        run_extra("rank_slice_ms", lambda: {
            "what": rank_slices.__doc__.split("->")[0].strip(),
            "c2_and": rank_slices(eng, lambda lo_, hi_: eng.pairwise("and", a, b, key_lo=lo_, key_hi=hi_),
                                  lambda nr: [((65536 * r) // nr, (65536 * (r + 1)) // nr) for r in range(nr)],
                                  ks, EXTRA_WARMUP),
            "c2_and_n1_ms_per_step": round(wall_max / args.steps * 1e3, 4),
            "c3_uniform_or": slices["c3_uniform_or"]})
    if args.c3_n > 0:
        for kind, name in ((1, "c3_uniform_or"), (2, "c3_clustered_or")):
            run_extra(name, lambda kind=kind: c3_wide_or(eng, kind, args.c3_n, rank, world, dist, ks, EXTRA_WARMUP, cdev,
                                                         slices=slices["c3_uniform_or"] if slices and kind == 1
                                                         else None))
        if world == 1:  # the same op over bitmaps decoded from their serialized bytes (packed vs 16 B slots)
            run_extra("c3_uniform_or_decoded", lambda: c3_uniform_decoded(eng, min(args.c3_n, 2000), ks,
                                                                          EXTRA_WARMUP))
        # FastAggregation.and (N > 10: workShyAnd): per key the chain stops once the
        # intersection is empty, so it reads far less than the algorithmic input bytes
        for kind, name in ((1, "c3_uniform_and"), (2, "c3_clustered_and")):
            run_extra(name, lambda kind=kind: c3_wide_or(eng, kind, args.c3_n, rank, world, dist, ks, EXTRA_WARMUP,
                                                         cdev, op="and"))
    if args.c4_pairs > 0:
        run_extra("c4_batch_and_card", lambda: c4_batch_and_card(eng, args.c4_pairs, rank, world, dist, ks,
                                                                  EXTRA_WARMUP, cdev))
    if args.c5_rows > 0:
        run_extra("c5_bsi_range_sum", lambda: c5_bsi(eng, args.c5_rows, rank, world, dist, ks, EXTRA_WARMUP, cdev))

    if args.c3_n > 0 or args.c4_pairs > 0 or args.c5_rows > 0:
        run_extra("run_optimize_c2", lambda: run_optimize_c2(eng, a, sa, ks))
        if not strong:
            run_extra("ornot_c2", lambda: ornot_c2(eng, a, b, sa, sb, ks))
        run_extra("decode_c2", lambda: decode_c2(eng, a, ks))
        if rank == 0:
            run_extra("c2_and_oneshot", lambda: c2_oneshot(eng, a, b, ks))
            run_extra("pq_or_bsi_slices", lambda: pq_or_queue(eng, 10 ** 8, ks))

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baselines(eng, a, b, in_bytes, args.cpu_seconds)

    if rank == 0:
        step_s = wall_max / args.steps
        # compute phase of the timed steps (pipelined: the span of the K range launches on the engine
        # stream, each launch 1/K of the bytes, so bytes / span = bytes per launch / mean launch time)
        compute_s = (ph_live[1] if ph_live[1] > 0 else ph_avg[1]) / 1e3
        achieved = (in_bytes + out_bytes) / compute_s / 1e9 if compute_s > 0 else 0.0
        line = {
            "metric": METRIC,
            "value": round(total_in / (wall_max / args.steps) / 1e9, 2),
            "unit": "GB/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(step_s * 1e3, 4),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "u64",
            "data": "synthetic",
            "config": {"workload": "C2: RoaringBitmap.and(x1, x2), two full 2^32-universe bitmaps of 65536 "
                                   "mixed array/bitmap/run containers each (configs[1])",
                       "per_rank": "the pair's key range [65536 r / N, 65536 (r + 1) / N); slices placed in each "
                                   "rank's HBM" if strong else "the whole pair",
                       "parallelism": f"key-range sharding over {world} GPU(s)"},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": _pmc_traffic(),
                         "kernel": f"{PW_KERNEL}<AND> (container compute)",
                         "bytes_per_launch": int((in_bytes + out_bytes) / (PIPE_K if PIPELINED and not strong else 1)),
                         "launches_per_step": PIPE_K if PIPELINED and not strong else 1,
                         "measured": "HIP events on the engine stream around the compute launches of the timed steps",
                         "standalone_kernel_ms": round(ph_avg[1], 4)},
            "cpu_baseline": cpu,
            "extra": {
                "input_bytes_per_step": int(in_bytes), "output_bytes_per_step": int(out_bytes),
                "gpu_event_ms_per_step": round(gpu_ms / args.steps, 4),
                "phase_ms": {"plan": round(ph_avg[0], 4), "compute": round(ph_avg[1], 4),
                             "place": round(ph_avg[2], 4), "serialize": round(ser_ms, 4)},
                "step_form": (f"pipelined: rbg_ctx_pairwise_serialized, {PIPE_K} key ranges" if PIPELINED and not strong
                              else "rbg_ctx_pairwise + rbg_ctx_serialize"),
                "timed_phase_ms": {"compute_span": round(ph_live[1], 4)},
                "elements_per_s": round((sa["cardinality"] + sb["cardinality"]) / step_s, 1),
                "operand_mix": {k: [sa[k], sb[k]] for k in ["array", "bitmap", "run"]},
                "result": rs,
                "input_frac_of_peak_per_gpu": round(total_in / step_s / 1e9 / world / HBM_PEAK_GBS, 4),
                **extra,
            },
        }
        print(json.dumps(line), flush=True)
    if dist is not None:
        dist.destroy_process_group()


def _only(eng, args, rank, world, dist, cdev):
    """One workload alone (for per-workload rocprofv3 --pmc passes): prints a short JSON line."""
    w = args.only
    steps = args.steps
    if w in ("c2", "c2card"):
        a = eng.synth(0, 0xC2A0 + 0x10000 * rank)
        b = eng.synth(0, 0xC2B0 + 0x10000 * rank)
        for _ in range(args.warmup + steps):
            if w == "c2":  # the headline step: the op and its serialization
                eng.pairwise("and", a, b)
                eng.serialize()
            else:
                eng.and_cardinality(a, b)
        eng.sync()
        res = {"only": w}
    elif w in ("c3u", "c3c"):
        res = {"only": w, **c3_wide_or(eng, 1 if w == "c3u" else 2, args.c3_n, rank, world, dist, steps,
                                       args.warmup, cdev)}
    elif w in ("c3u_and", "c3c_and"):
        res = {"only": w, **c3_wide_or(eng, 1 if w == "c3u_and" else 2, args.c3_n, rank, world, dist, steps,
                                       args.warmup, cdev, op="and")}
    elif w == "c4":
        res = {"only": w, **c4_batch_and_card(eng, args.c4_pairs, rank, world, dist, steps, args.warmup, cdev)}
    elif w == "c5":
        res = {"only": w, **c5_bsi(eng, args.c5_rows, rank, world, dist, steps, args.warmup, cdev)}
    elif w == "runopt":
        a = eng.synth(0, 0xC2A0 + 0x10000 * rank)
        res = {"only": w, **run_optimize_c2(eng, a, eng.batch_stats(a), steps)}
    elif w == "ornot":
        a = eng.synth(0, 0xC2A0 + 0x10000 * rank)
        b = eng.synth(0, 0xC2B0 + 0x10000 * rank)
        res = {"only": w, **ornot_c2(eng, a, b, eng.batch_stats(a), eng.batch_stats(b), steps)}
    else:
        raise SystemExit(f"unknown workload {w}")
    if rank == 0:
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
