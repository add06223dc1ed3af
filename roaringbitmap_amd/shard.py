"""Key-range sharded wide aggregation across GPUs.

Every FastAggregation op is independent per high-16 key: the result container of
key k depends only on the inputs' containers of key k (RB/FastAggregation.java:
395-412, RB/RoaringBitmap.java:2405-2448, RB/ParallelAggregation.java:171-173).
So [0, 65536) is split into one contiguous key range per rank, with equal input
bytes rather than equal key counts (clustered inputs are skewed). Each rank (one
process per GPU) reduces its own key slice with the engine. The only exchanges
are small ones:

* an all-gather of every shard's (containers, payload bytes, has_run). That is
  all that is needed to place each shard inside the global portable layout: the
  cookie and run-flag choice, the container count and the payload offsets
  (RB/RoaringArray.java:896-940);
* for naive_and (N <= 10), an all-reduce of per-input container counts. It picks
  the input with the fewest containers over the whole universe
  (RB/FastAggregation.java:333-339), which no single key slice can see;
* for andCardinality / orCardinality, an all-reduce of the int64 partial sums,
  wrapped to a Java int at the end.

`concat_serialized` builds the global bitmap from the shard results. On a
distributed run, `gather_bytes` brings every shard to every rank first.

The collectives run over torch.distributed ("nccl" = RCCL over xGMI on ROCm; the
CPU tests use "gloo"). The per-shard compute is passed in as a callable;
`engine_shard` is the product binding to the HIP engine.
"""
import numpy as np

KEYS = 65536
NAIVE_AND_OPS = ("naive_and", "and_iter")


def key_ranges(key_bytes, world):
    """Contiguous key ranges [(lo, hi)] * world with about equal input bytes.

    An exclusive scan of the per-key bytes. Ranges may be empty
    when one key outweighs a whole share.
    """
    kb = np.asarray(key_bytes, dtype=np.float64)
    if kb.shape != (KEYS,):
        raise ValueError("key_bytes must have 65536 entries")
    cum = np.cumsum(kb)
    total = cum[-1]
    bounds = [0]
    for r in range(1, world):
        b = int(np.searchsorted(cum, total * r / world, side="left")) + 1 if total > 0 else (KEYS * r) // world
        bounds.append(min(max(b, bounds[-1]), KEYS))
    bounds.append(KEYS)
    return [(bounds[r], bounds[r + 1]) for r in range(world)]


# ---------------------------------------------------------------------------
# portable format (RB/RoaringArray.java:896-940) on the host
# ---------------------------------------------------------------------------
SERIAL_COOKIE_NO_RUN = 12346
SERIAL_COOKIE = 12347


def header_size(n, has_run):
    """RB/RoaringArray.java:781-790"""
    if has_run:
        return 4 + (n + 7) // 8 + (4 * n if n < 4 else 8 * n)
    return 8 + 8 * n


def parse_layout(buf):
    """-> (keys u16[n], card_minus_1 u16[n], is_run bool[n], sizes int64[n], payload bytes) of one bitmap."""
    b = memoryview(bytes(buf))
    cookie = int.from_bytes(b[0:4], "little")
    if (cookie & 0xFFFF) == SERIAL_COOKIE:
        n = (cookie >> 16) + 1
        nb = (n + 7) // 8
        flags = np.unpackbits(np.frombuffer(b[4:4 + nb], dtype=np.uint8), bitorder="little")[:n].astype(bool)
        pos = 4 + nb
    elif cookie == SERIAL_COOKIE_NO_RUN:
        n = int.from_bytes(b[4:8], "little")
        flags = np.zeros(n, dtype=bool)
        pos = 8
    else:
        raise ValueError("not a portable roaring bitmap")
    desc = np.frombuffer(b[pos:pos + 4 * n], dtype="<u2").reshape(n, 2)
    keys, cm1 = desc[:, 0].copy(), desc[:, 1].copy()
    hdr = header_size(n, bool(flags.any()))
    sizes = np.zeros(n, dtype=np.int64)
    p = hdr
    for i in range(n):  # payload sizes (getArraySizeInBytes), walking run counts
        if flags[i]:
            nr = int.from_bytes(b[p:p + 2], "little")
            sizes[i] = 2 + 4 * nr
        elif int(cm1[i]) + 1 > 4096:
            sizes[i] = 8192
        else:
            sizes[i] = 2 * (int(cm1[i]) + 1)
        p += int(sizes[i])
    return keys, cm1, flags, sizes, bytes(b[hdr:p])


def concat_serialized(parts):
    """One portable bitmap from shard results whose keys are disjoint and ascending across parts."""
    lay = [parse_layout(p) for p in parts]
    keys = np.concatenate([x[0] for x in lay]) if lay else np.zeros(0, np.uint16)
    cm1 = np.concatenate([x[1] for x in lay]) if lay else np.zeros(0, np.uint16)
    runs = np.concatenate([x[2] for x in lay]) if lay else np.zeros(0, bool)
    sizes = np.concatenate([x[3] for x in lay]) if lay else np.zeros(0, np.int64)
    if len(keys) > 1 and not np.all(keys[1:] > keys[:-1]):
        raise ValueError("shard key ranges overlap or are out of order")
    n = len(keys)
    has_run = bool(runs.any())
    out = bytearray()
    if has_run:
        out += (SERIAL_COOKIE | ((n - 1) << 16)).to_bytes(4, "little")
        out += np.packbits(runs.astype(np.uint8), bitorder="little").tobytes()
    else:
        out += SERIAL_COOKIE_NO_RUN.to_bytes(4, "little") + n.to_bytes(4, "little")
    d = np.empty((n, 2), dtype="<u2")
    d[:, 0], d[:, 1] = keys, cm1
    out += d.tobytes()
    if not has_run or n >= 4:
        offs = header_size(n, has_run) + np.concatenate([[0], np.cumsum(sizes)[:-1]]) if n else np.zeros(0)
        out += np.asarray(offs, dtype="<u4").tobytes()
    for x in lay:
        out += x[4]
    return bytes(out)


# ---------------------------------------------------------------------------
# collectives
# ---------------------------------------------------------------------------
def _dist():
    import torch.distributed as dist
    return dist


def global_layout(n_containers, payload_bytes, has_run, group=None, device="cpu"):
    """All-gather of every shard's (containers, payload bytes, has_run).

    Returns (total containers, has_run, first container index of this rank,
    payload byte offset of this rank within the global payload region).
    """
    import torch
    dist = _dist()
    world = dist.get_world_size(group)
    mine = torch.tensor([int(n_containers), int(payload_bytes), int(has_run)], dtype=torch.int64, device=device)
    allv = [torch.zeros_like(mine) for _ in range(world)]
    dist.all_gather(allv, mine, group=group)
    a = torch.stack(allv).cpu().numpy()
    r = dist.get_rank(group)
    return int(a[:, 0].sum()), bool(a[:, 2].any()), int(a[:r, 0].sum()), int(a[:r, 1].sum())


def gather_bytes(data, group=None, device="cpu"):
    """All-gather of one variable-length byte string per rank (sizes first, then padded bytes)."""
    import torch
    dist = _dist()
    world = dist.get_world_size(group)
    n = torch.tensor([len(data)], dtype=torch.int64, device=device)
    sizes = [torch.zeros_like(n) for _ in range(world)]
    dist.all_gather(sizes, n, group=group)
    sizes = [int(s.item()) for s in sizes]
    m = max(sizes) if sizes else 0
    buf = torch.zeros(max(m, 1), dtype=torch.uint8, device=device)
    if data:
        buf[:len(data)] = torch.frombuffer(bytearray(data), dtype=torch.uint8).to(device)
    outs = [torch.zeros_like(buf) for _ in range(world)]
    dist.all_gather(outs, buf, group=group)
    return [bytes(o[:s].cpu().numpy().tobytes()) for o, s in zip(outs, sizes)]


def global_start(op, counts, group=None, device="cpu"):
    """naive_and's start input over the whole universe: the fewest containers, first on ties."""
    import torch
    dist = _dist()
    if op not in NAIVE_AND_OPS and op != "and":
        return -1
    t = torch.as_tensor(np.asarray(counts, dtype=np.int64), device=device).clone()
    dist.all_reduce(t, group=group)
    if op == "and_iter":
        return 0
    return int(np.argmin(t.cpu().numpy())) if t.numel() else -1


def sharded_wide(op, shard_fn, n_inputs, counts=None, group=None, device="cpu", gather=True):
    """This rank's part of a key-sharded FastAggregation op.

    shard_fn(start_bm) -> serialized result of this rank's key slice. start_bm is
    the naive_and start input (-1 = not a naive_and chain).
    counts: containers per input bitmap in this rank's slice (naive_and only).
    Returns the global serialized bitmap when gather is true, else this rank's
    (shard bytes, global layout).
    """
    start = -1
    naive = op in NAIVE_AND_OPS or (op == "and" and n_inputs <= 10)
    if naive and counts is not None:
        start = global_start("and_iter" if op == "and_iter" else "naive_and", counts, group, device)
    local = shard_fn(start)
    if not gather:
        keys, _, runs, sizes, _ = parse_layout(local)
        return local, global_layout(len(keys), int(sizes.sum()), bool(runs.any()), group, device)
    return concat_serialized(gather_bytes(local, group, device))


def sharded_wide_card(partial, group=None, device="cpu"):
    """andCardinality / orCardinality over key shards: int64 all-reduce, then Java int wrap."""
    import torch
    dist = _dist()
    t = torch.tensor([int(partial)], dtype=torch.int64, device=device)
    dist.all_reduce(t, group=group)
    return int(np.int64(t.item()).astype(np.int32))


def engine_shard(engine, op, batch, key_lo, key_hi, ids=None):
    """Product shard function: the HIP engine reduces [key_lo, key_hi) of a device-resident batch."""
    def fn(start_bm):
        if start_bm >= 0:
            engine.wide_start(op, batch, key_lo, key_hi, start_bm, ids)
        else:
            engine.wide(op, batch, key_lo, key_hi, ids)
        return engine.fetch().serialize()
    return fn
