"""Key-range sharding host logic (roaringbitmap_amd/shard.py), on CPU.

SURVEY.md §8(e): per-key independence makes every FastAggregation op shard by key
range. The concatenation of per-shard results must be byte-identical to the
unsharded result. The world-size-2 tests run the real collectives over gloo on
127.0.0.1. The per-shard compute there is the CPU oracle applied to the inputs
restricted to the shard's keys; it stands in for the GPU engine, which
tests/test_gpu_shard.py exercises. Only the exchange and the assembly are under
test here.
"""
import os
import socket
import tempfile

import numpy as np
import pytest
import torch.multiprocessing as mp

import _gen
import _oracle as O
from _fmt import decode, encode
from roaringbitmap_amd import shard


def restrict(buf, lo, hi):
    """The containers of a serialized bitmap whose keys fall in [lo, hi)."""
    return encode([(k, kind, vals) for k, kind, _, vals, _ in decode(buf) if lo <= k < hi])


def _inputs(seed, n, nkeys=24, spread=65536):
    rng = np.random.default_rng(seed)
    keys = np.sort(rng.choice(spread, size=nkeys, replace=False))
    return [_gen.bitmap(rng, keys, p_present=0.8) for _ in range(n)]


def test_key_ranges_cover_and_balance():
    kb = np.zeros(65536, dtype=np.uint64)
    kb[100:200] = 1000
    kb[5000] = 50000
    for world in (1, 2, 3, 4, 8):
        rs = shard.key_ranges(kb, world)
        assert rs[0][0] == 0 and rs[-1][1] == 65536
        assert all(a[1] == b[0] for a, b in zip(rs, rs[1:]))
        assert all(lo <= hi for lo, hi in rs)
    uni = shard.key_ranges(np.ones(65536), 8)
    assert [hi - lo for lo, hi in uni] == [8192] * 8


@pytest.mark.parametrize("world", [1, 2, 3, 5])
@pytest.mark.parametrize("op", ["or", "xor", "workshy_and"])
def test_concat_of_key_shards_is_byte_identical(world, op):
    bufs = _inputs(11 + world, 14)
    full = O.wide(op, bufs)
    kb = np.zeros(65536)
    for b in bufs:
        for k, _, card, _, _ in decode(b):
            kb[k] += 4 + 2 * card
    parts = [O.wide(op, [restrict(b, lo, hi) for b in bufs]) for lo, hi in shard.key_ranges(kb, world)]
    assert shard.concat_serialized(parts) == full


def test_concat_header_variants():
    """run flags across shard boundaries; size < 4 with runs omits offsets (RB/RoaringArray.java:927-933)"""
    full = np.arange(65536, dtype=np.uint16)
    for n in range(1, 7):
        bm = encode([(k * 3, _fmt_kind(k), full[: 50 + k]) for k in range(n)])
        for cut in range(0, 3 * n + 1, 2):
            assert shard.concat_serialized([restrict(bm, 0, cut), restrict(bm, cut, 65536)]) == bm
    assert shard.concat_serialized([]) == encode([])


def _fmt_kind(k):
    from _fmt import A, R
    return R if k % 2 else A


@pytest.mark.parametrize("n_keys", [1, 3, 5, 40])
def test_assemble_single_process(n_keys):
    """assemble() at world 1 (no process group): the global bitmap of one shard, including
    the run-flag packing and the size < 4 layout without offsets."""
    bufs = _inputs(5 + n_keys, 6, nkeys=n_keys)
    for op in ("or", "xor"):
        part = O.wide(op, bufs)
        lay = shard.GlobalLayout([shard.shard_stats(part)])
        out = shard.assemble(shard.serialized_fill(part), lay, 0, fill_device="cpu", comm_device="cpu")
        assert bytes(out.numpy().tobytes()) == part


def test_parse_layout_golden():
    gold = os.path.join(os.path.dirname(__file__), "golden", "testdata")
    for name in ("bitmapwithruns.bin", "bitmapwithoutruns.bin"):
        b = open(os.path.join(gold, name), "rb").read()
        keys, _, runs, sizes, payload = shard.parse_layout(b)
        assert len(payload) == int(sizes.sum())
        assert shard.concat_serialized([b]) == O.roundtrip(b)[1]


# ---- world size 2 over gloo ---------------------------------------------------
def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, outdir):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        bufs = _inputs(77, 13)
        kb = np.zeros(65536)
        for b in bufs:
            for k, _, card, _, _ in decode(b):
                kb[k] += 4 + 2 * card
        lo, hi = shard.key_ranges(kb, world)[rank]
        mine = [restrict(b, lo, hi) for b in bufs]
        res = {}
        for op in ("or", "xor", "workshy_and"):
            res[op] = shard.sharded_wide(op, lambda start, op=op: O.wide(op, mine), len(bufs))
            local, lay = shard.sharded_wide(op, lambda start, op=op: O.wide(op, mine), len(bufs), gather=False)
            res[op + "_layout"] = lay
        # naive_and start over the whole universe: all-reduce of per-input container counts
        counts = np.array([len(decode(b)) for b in mine], dtype=np.int64)
        res["start"] = shard.global_start("naive_and", counts)
        res["card_or"] = shard.sharded_wide_card(O.wide_card("or", mine) if any(len(decode(b)) for b in mine) else 0)
        # device-style assembly on rank 0: slices received straight into their global place
        for op in ("or", "xor", "workshy_and"):
            part = O.wide(op, mine)
            lay = shard.exchange_layout(*shard.shard_stats(part))
            out = shard.assemble(shard.serialized_fill(part), lay, rank, fill_device="cpu", comm_device="cpu")
            if rank == 0:
                res[op + "_assembled"] = bytes(out.numpy().tobytes())
        if rank == 0:
            np.save(os.path.join(outdir, "res.npy"), np.array([res], dtype=object), allow_pickle=True)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_world_gloo_sharded_wide(world):
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_worker, args=(world, _free_port(), d), nprocs=world, join=True)
        res = np.load(os.path.join(d, "res.npy"), allow_pickle=True)[0]  # written by this test's own worker
    bufs = _inputs(77, 13)
    for op in ("or", "xor", "workshy_and"):
        assert res[op] == O.wide(op, bufs), op
        assert res[op + "_assembled"] == O.wide(op, bufs), op
        full = decode(O.wide(op, bufs))
        n_total, has_run, first, base = res[op + "_layout"]
        assert n_total == len(full) and first == 0 and base == 0
        assert has_run == any(c[1] == 2 for c in full)
    counts = np.array([len(decode(b)) for b in bufs])
    assert res["start"] == int(np.argmin(counts))
    assert res["card_or"] == O.wide_card("or", bufs)
