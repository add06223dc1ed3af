"""Multi-process key sharding through the HIP engine on the one GPU of the box.

Two ranks (gloo: RCCL refuses two ranks on one device) each generate and reduce their own
key slice of a C3 batch with the engine, then `shard.assemble` builds the global portable
bitmap on rank 0: rank 0 writes its slice in place, rank 1's descriptors, global offsets,
run bytes and payload are received straight into their places.  The result must be
byte-identical to the unsharded engine result (which tests/test_gpu_shard.py and
tests/test_gpu_fullsize.py pin to the oracle).  bench.py's own multi-rank path is
rehearsed the same way (`--gpus 2 --backend gloo`).
"""
import json
import os
import socket
import subprocess
import sys
import tempfile

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, outdir, kind, op):
    import torch
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from roaringbitmap_amd import Engine, shard
        from roaringbitmap_amd.engine import synth_key_bytes
        n, seed = 200, 0xC3000000
        e = Engine(0)
        ranges = shard.key_ranges(synth_key_bytes(kind, seed, n), world)
        lo, hi = ranges[rank]
        b = e.synth(kind, seed, n, lo, hi)
        e.wide(op, b, lo, hi)
        rs = e.result_stats()
        lay = shard.exchange_layout(rs["containers"], rs["payload_bytes"], rs["has_run"], device="cpu")
        out = shard.assemble(shard.engine_fill(e), lay, rank, fill_device=torch.device("cuda", 0),
                             comm_device="cpu", sync=e.sync)
        if rank == 0:
            full = e.synth(kind, seed, n)
            e.wide(op, full)
            ref = e.fetch().serialize()
            with open(os.path.join(outdir, "res.bin"), "wb") as f:
                f.write(bytes(out.numpy().tobytes()))
            with open(os.path.join(outdir, "ref.bin"), "wb") as f:
                f.write(ref)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("kind,op", [(1, "or"), (2, "or"), (2, "xor"), (1, "workshy_and")])
def test_two_rank_engine_assembly(gpu, kind, op):
    import torch.multiprocessing as mp
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_worker, args=(2, _free_port(), d, kind, op), nprocs=2, join=True)
        res = open(os.path.join(d, "res.bin"), "rb").read()
        ref = open(os.path.join(d, "ref.bin"), "rb").read()
    assert res == ref


def _pair_worker(rank, world, port, outdir, op):
    import numpy as np
    import torch
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from roaringbitmap_amd import Engine, shard
        e = Engine(0)
        # a mixed pair over ~200 keys with run containers on both sides (RB/RoaringBitmap.java:382-399)
        rng = np.random.default_rng(11)
        import roaringbitmap_amd as rb
        va = np.concatenate([rng.integers(0, 200 << 16, 300000), np.arange(5 << 16, 9 << 16)])
        vb = np.concatenate([rng.integers(0, 200 << 16, 300000), np.arange(7 << 16, (7 << 16) + 40000)])
        xa = rb.RoaringBitmap.from_values(va, run_optimize=True).serialize()
        xb = rb.RoaringBitmap.from_values(vb, run_optimize=True).serialize()
        a, b = e.load([xa]), e.load([xb])
        lo, hi = [(0, 77), (77, 65536)][rank]
        e.pairwise(op, a, b, key_lo=lo, key_hi=hi)
        rs = e.result_stats()
        lay = shard.exchange_layout(rs["containers"], rs["payload_bytes"], rs["has_run"], device="cpu")
        out = shard.assemble(shard.engine_fill(e), lay, rank, fill_device=torch.device("cuda", 0),
                             comm_device="cpu", sync=e.sync)
        if rank == 0:
            e.pairwise(op, a, b)
            ref = e.fetch().serialize()
            with open(os.path.join(outdir, "res.bin"), "wb") as f:
                f.write(bytes(out.numpy().tobytes()))
            with open(os.path.join(outdir, "ref.bin"), "wb") as f:
                f.write(ref)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("op", ["and", "or", "xor", "andnot"])
def test_two_rank_pairwise_assembly(gpu, op):
    """A pairwise op split into two key ranges over two processes, assembled on rank 0, equals
    the unsharded result byte for byte."""
    import torch.multiprocessing as mp
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_pair_worker, args=(2, _free_port(), d, op), nprocs=2, join=True)
        res = open(os.path.join(d, "res.bin"), "rb").read()
        ref = open(os.path.join(d, "ref.bin"), "rb").read()
    assert res == ref


def _dyn_worker(rank, world, port, outdir, op):
    import numpy as np
    import torch
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import roaringbitmap_amd as rb
        from roaringbitmap_amd import Engine, shard
        e = Engine(0)
        rng = np.random.default_rng(12)
        va = np.concatenate([rng.integers(0, 300 << 16, 400000), np.arange(5 << 16, 9 << 16)])
        vb = np.concatenate([rng.integers(0, 300 << 16, 400000), np.arange(7 << 16, (7 << 16) + 40000)])
        a = e.load([rb.RoaringBitmap.from_values(va, run_optimize=True).serialize()])
        b = e.load([rb.RoaringBitmap.from_values(vb, run_optimize=True).serialize()])
        lo, hi = [(0, 100), (100, 65536)][rank]
        ds = shard.DeviceShard(e, rank, world, torch.device("cuda", 0), "cpu")
        for _ in range(2):  # a repeated step reuses the buffers
            e.pairwise(op, a, b, key_lo=lo, key_hi=hi)
            ds.place()
        out = ds.gather()
        if rank == 0:
            e.pairwise(op, a, b)
            ref = e.fetch().serialize()
            with open(os.path.join(outdir, "res.bin"), "wb") as f:
                f.write(bytes(out.cpu().numpy().tobytes()))
            with open(os.path.join(outdir, "ref.bin"), "wb") as f:
                f.write(ref)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("op", ["and", "or"])
def test_two_rank_device_layout(gpu, op):
    """shard.DeviceShard (the bench's N > 1 headline step): the layout all-gathered from device
    tensors, each rank's slice placed at its global offsets in its own buffer, gathered on rank 0:
    equal to the unsharded result byte for byte."""
    import torch.multiprocessing as mp
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_dyn_worker, args=(2, _free_port(), d, op), nprocs=2, join=True)
        res = open(os.path.join(d, "res.bin"), "rb").read()
        ref = open(os.path.join(d, "ref.bin"), "rb").read()
    assert res == ref


def _bench(gpus):
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(gpus), "--backend", "gloo", "--steps", "2",
           "--warmup", "1", "--c3-n", "64", "--c4-pairs", "2000", "--c5-rows", "2000000", "--no-cpu-baseline"]
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=300, cwd=ROOT)
    assert p.returncode == 0, p.stderr[-3000:]
    return json.loads([ln for ln in p.stdout.splitlines() if ln.startswith("{")][-1])


def test_bench_two_ranks_rehearsal(gpu):
    one, two = _bench(1), _bench(2)
    assert one["n_gpus"] == 1 and two["n_gpus"] == 2
    # the N > 1 headline is the key-sharded C2 AND (strong scaling): its slices, gathered on GPU 0,
    # are the same bytes as the one-GPU headline's result (same pair)
    assert one["scaling"] == two["scaling"] == "strong"
    assert two["extra"]["c2_strong"]["result_sha16"] == one["extra"]["result"]["sha16"]
    assert two["extra"]["c2_strong"]["sha_equals_whole_pair_result"] is True
    assert two["extra"]["c2_and_weak"]["scaling"] == "weak"
    for w in ("c3_uniform_or", "c3_clustered_or", "c3_uniform_and"):
        assert two["extra"][w]["result_serialized_bytes"] == one["extra"][w]["result_serialized_bytes"], w
        assert two["extra"][w]["output_bytes"] == one["extra"][w]["output_bytes"], w
    assert two["extra"]["c5_bsi_range_sum"]["sum_count"] == one["extra"]["c5_bsi_range_sum"]["sum_count"]


def _rccl_worker(rank, world, port, outdir, op):
    import numpy as np
    import torch
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    # RCCL ("nccl" on ROCm) before any other GPU call of this process
    dist.init_process_group("nccl", rank=rank, world_size=world, device_id=torch.device("cuda", 0))
    try:
        import roaringbitmap_amd as rb
        from roaringbitmap_amd import Engine, shard
        e = Engine(0)
        rng = np.random.default_rng(13)
        va = np.concatenate([rng.integers(0, 300 << 16, 400000), np.arange(5 << 16, 9 << 16)])
        vb = np.concatenate([rng.integers(0, 300 << 16, 400000), np.arange(7 << 16, (7 << 16) + 40000)])
        a = e.load([rb.RoaringBitmap.from_values(va, run_optimize=True).serialize()])
        b = e.load([rb.RoaringBitmap.from_values(vb, run_optimize=True).serialize()])
        dev = torch.device("cuda", 0)
        ds = shard.DeviceShard(e, rank, world, dev, dev, collective=True)
        for _ in range(3):  # repeated steps reuse the buffers; every step waits on RCCL's stream
            e.pairwise(op, a, b)
            ds.place()
        lay_local = ds.lay_local.cpu().tolist()
        lay_all = ds.lay_all.cpu().tolist()
        out = ds.gather()
        e.pairwise(op, a, b)
        ref = e.fetch().serialize()
        with open(os.path.join(outdir, "res.bin"), "wb") as f:
            f.write(bytes(out.cpu().numpy().tobytes()))
        with open(os.path.join(outdir, "ref.bin"), "wb") as f:
            f.write(ref)
        with open(os.path.join(outdir, "lay.json"), "w") as f:
            json.dump({"local": lay_local, "all": lay_all, "backend": dist.get_backend()}, f)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("op", ["and", "or"])
def test_rccl_device_layout_world1(gpu, op):
    """The RCCL branch of shard.DeviceShard.place() on the one GPU of the box: a world-size-1 "nccl"
    process group, the layout all-gathered with all_gather_into_tensor on device memory, ordered
    against the engine stream by wait_stream both ways, then placed by rbg_ctx_fetch_shard_device_dyn:
    the gathered bitmap equals the engine's whole-pair result byte for byte."""
    import torch.multiprocessing as mp
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_rccl_worker, args=(1, _free_port(), d, op), nprocs=1, join=True)
        res = open(os.path.join(d, "res.bin"), "rb").read()
        ref = open(os.path.join(d, "ref.bin"), "rb").read()
        lay = json.load(open(os.path.join(d, "lay.json")))
    assert lay["backend"] == "nccl"
    assert lay["all"] == lay["local"] and lay["local"][0] > 0
    assert res == ref
