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

The result is assembled on rank 0's device (`assemble`): every rank writes its slice's
descriptors, global offset-table entries, run bytes and payload (`engine_fill`, i.e.
rbg_ctx_fetch_shard_device) and rank 0 receives each slice straight into its place in
the global bitmap over point-to-point RCCL. `concat_serialized` / `gather_bytes` are the
host-bytes form of the same assembly.

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


# ---------------------------------------------------------------------------
# device-resident result assembly
# ---------------------------------------------------------------------------
class GlobalLayout:
    """Where every shard's slice goes in the global portable bitmap (RB/RoaringArray.java:896-940).

    per_rank: int64 [world, 3] = (containers, payload bytes, has_run) of every rank's key slice,
    in key-range order.
    """

    def __init__(self, per_rank):
        a = np.asarray(per_rank, dtype=np.int64).reshape(-1, 3)
        self.n = a[:, 0].copy()
        self.pay = a[:, 1].copy()
        self.total = int(self.n.sum())
        self.has_run = bool(a[:, 2].any())
        self.first = np.concatenate([[0], np.cumsum(self.n)[:-1]]).astype(np.int64)
        self.base = np.concatenate([[0], np.cumsum(self.pay)[:-1]]).astype(np.int64)
        self.header = header_size(self.total, self.has_run)
        self.flag_bytes = (self.total + 7) // 8 if self.has_run else 0
        self.desc_base = 4 + self.flag_bytes if self.has_run else 8
        self.offsets = (not self.has_run) or self.total >= 4
        self.off_base = self.desc_base + 4 * self.total
        self.nbytes = self.header + int(self.pay.sum())

    def cookie(self) -> bytes:
        if self.has_run:
            return (SERIAL_COOKIE | ((self.total - 1) << 16)).to_bytes(4, "little")
        return SERIAL_COOKIE_NO_RUN.to_bytes(4, "little") + self.total.to_bytes(4, "little")


def exchange_layout(n_containers, payload_bytes, has_run, group=None, device="cpu"):
    """All-gather of (containers, payload bytes, has_run) -> GlobalLayout (single process: world 1)."""
    import torch
    mine = [int(n_containers), int(payload_bytes), int(bool(has_run))]
    dist = _dist()
    if not (dist.is_available() and dist.is_initialized()):
        return GlobalLayout([mine])
    t = torch.tensor(mine, dtype=torch.int64, device=device)
    allv = [torch.zeros_like(t) for _ in range(dist.get_world_size(group))]
    dist.all_gather(allv, t, group=group)
    return GlobalLayout(torch.stack(allv).cpu().numpy())


def _pack_flags(runb):
    """One byte per container (1 = run) -> the run-flag bitset (bit i%8 of byte i/8)."""
    import torch
    n = runb.numel()
    pad = torch.zeros(((n + 7) // 8) * 8, dtype=torch.int32, device=runb.device)
    pad[:n] = runb.to(torch.int32)
    w = torch.tensor([1, 2, 4, 8, 16, 32, 64, 128], dtype=torch.int32, device=runb.device)
    return (pad.view(-1, 8) * w).sum(dim=1).to(torch.uint8)


def assemble(fill, lay, rank=0, group=None, fill_device="cuda", comm_device="cuda", sync=None):
    """Assemble the global portable bitmap on rank 0 from every rank's key slice.

    fill(total, has_run, payload_base, desc, offsets, runflags, payload) writes this rank's
    slice into the given uint8 tensors (on fill_device): its descriptors, its entries of the
    global offset table, one run byte per container and its payload (Engine.fetch_shard_device
    for the HIP engine).  sync() (optional) waits for the fill.  Rank 0 owns the output buffer;
    its own slice is written in place and every other slice is received straight into its
    place (point-to-point over RCCL/xGMI, or gloo on the CPU) -- no all-gather of bulk data.
    Returns the uint8 tensor of the global bitmap on rank 0, None elsewhere.
    """
    import torch
    r = rank
    n, pay = int(lay.n[r]), int(lay.pay[r])

    def views(buf, runb, rr):
        nr, f, b = int(lay.n[rr]), int(lay.first[rr]), int(lay.base[rr])
        d = buf[lay.desc_base + 4 * f: lay.desc_base + 4 * (f + nr)]
        o = buf[lay.off_base + 4 * f: lay.off_base + 4 * (f + nr)] if lay.offsets else None
        rb_ = runb[f: f + nr] if runb is not None else None
        p = buf[lay.header + b: lay.header + b + int(lay.pay[rr])]
        return d, o, rb_, p

    def local(dev):
        d = torch.empty(4 * n, dtype=torch.uint8, device=dev)
        o = torch.empty(4 * n, dtype=torch.uint8, device=dev) if lay.offsets else None
        rb_ = torch.empty(n, dtype=torch.uint8, device=dev) if lay.has_run else None
        p = torch.empty(pay, dtype=torch.uint8, device=dev)
        return d, o, rb_, p

    def do_fill(parts):
        if n:
            fill(lay.total, lay.has_run, int(lay.base[r]), *parts)
            if sync is not None:
                sync()

    world = len(lay.n)
    if r == 0:
        out = torch.empty(lay.nbytes, dtype=torch.uint8, device=comm_device)
        # every byte is written: rank 0's slice by its fill, the others' by their receives
        # (a zero fill here would run on torch's stream, unordered with the engine's writes)
        runb = torch.empty(lay.total, dtype=torch.uint8, device=comm_device) if lay.has_run else None
        mine = views(out, runb, 0)
        if torch.device(fill_device) == torch.device(comm_device):
            do_fill(mine)
        else:
            tmp = local(fill_device)
            do_fill(tmp)
            for dst, src in zip(mine, tmp):
                if dst is not None:
                    dst.copy_(src)
        ops = []
        if world > 1:
            dist = _dist()
            for rr in range(1, world):
                if not int(lay.n[rr]):
                    continue
                src = rr if group is None else dist.get_global_rank(group, rr)
                ops += [(t, src) for t in views(out, runb, rr) if t is not None and t.numel()]
        reqs = _p2p([(dist.irecv, t, peer) for t, peer in ops], group) if ops else []
        out[:len(lay.cookie())] = torch.tensor(list(lay.cookie()), dtype=torch.uint8, device=comm_device)
        for q in reqs:
            q.wait()
        if lay.has_run and lay.total:
            out[4:4 + lay.flag_bytes] = _pack_flags(runb)
        return out
    parts = local(fill_device)
    do_fill(parts)
    if n:
        dist = _dist()
        dst = 0 if group is None else dist.get_global_rank(group, 0)
        sends = [t if torch.device(fill_device) == torch.device(comm_device) else t.to(comm_device)
                 for t in parts if t is not None and t.numel()]
        for q in _p2p([(dist.isend, t, dst) for t in sends], group):
            q.wait()
    return None


def _p2p(ops, group):
    """Point-to-point ops; grouped (one ncclGroup, all peers' transfers concurrent over their
    own xGMI links) on RCCL, posted in order on gloo."""
    dist = _dist()
    if dist.get_backend(group) == "nccl":
        return dist.batch_isend_irecv([dist.P2POp(fn, t, peer, group) for fn, t, peer in ops])
    kw = {} if group is None else {"group": group}
    return [fn(t, peer, **kw) for fn, t, peer in ops]


def engine_fill(engine):
    """fill() of assemble() for the HIP engine's pending result (Engine.fetch_shard_device)."""
    def fill(total, has_run, payload_base, desc, offsets, runflags, payload):
        engine.fetch_shard_device(total, has_run, payload_base, desc, offsets, runflags, payload)
    return fill


def serialized_fill(buf):
    """fill() of assemble() from a shard result held as serialized bytes (CPU stand-in for tests)."""
    import torch
    keys, cm1, runs, sizes, payload = parse_layout(buf)

    def fill(total, has_run, payload_base, desc, offsets, runflags, pay):
        d = np.empty((len(keys), 2), dtype="<u2")
        d[:, 0], d[:, 1] = keys, cm1
        desc.copy_(torch.frombuffer(bytearray(d.tobytes()), dtype=torch.uint8))
        if offsets is not None:
            o = header_size(total, has_run) + payload_base + np.concatenate([[0], np.cumsum(sizes)[:-1]])
            offsets.copy_(torch.frombuffer(bytearray(np.asarray(o, dtype="<u4").tobytes()), dtype=torch.uint8))
        if runflags is not None:
            runflags.copy_(torch.from_numpy(runs.astype(np.uint8)))
        if len(payload):
            pay.copy_(torch.frombuffer(bytearray(payload), dtype=torch.uint8))
    return fill


def shard_stats(buf):
    """(containers, payload bytes, has_run) of a serialized shard result."""
    keys, _, runs, sizes, _ = parse_layout(buf)
    return len(keys), int(sizes.sum()), bool(runs.any())


def engine_shard(engine, op, batch, key_lo, key_hi, ids=None):
    """Product shard function: the HIP engine reduces [key_lo, key_hi) of a device-resident batch."""
    def fn(start_bm):
        if start_bm >= 0:
            engine.wide_start(op, batch, key_lo, key_hi, start_bm, ids)
        else:
            engine.wide(op, batch, key_lo, key_hi, ids)
        return engine.fetch().serialize()
    return fn


# ---------------------------------------------------------------------------
# device-resident layout exchange: no host synchronisation inside a sharded step
# ---------------------------------------------------------------------------
MAX_SERIALIZED = 8 + 8 * KEYS + 8194 * KEYS  # bounds any global bitmap (header + payload)


class DeviceShard:
    """One rank's part of a key-sharded op whose result stays in HBM (SURVEY §8(e) steps 1-2,
    all on the device): after the engine's op on this rank's key range, `place()` writes the
    result's (containers, payload bytes, has_run) into a device tensor on the engine stream
    (rbg_ctx_result_layout_device), all-gathers it (RCCL on device memory; gloo through the
    host), and writes this rank's descriptors, offset-table entries, run bytes and payload at
    their global places in `out`, this rank's buffer laid out as the whole global bitmap
    (rbg_ctx_fetch_shard_device_dyn).  No host round trip: the step is a chain of stream
    dependencies.  `gather()` then assembles the global bitmap on rank 0 (point-to-point)."""

    def __init__(self, engine, rank, world, device, comm_device, group=None, collective=None):
        """collective: exchange the layout through the process group (default: when world > 1;
        True at world 1 runs the all-gather path, stream waits included, on one rank)."""
        import torch
        self.eng, self.rank, self.world, self.group = engine, rank, world, group
        self.collective = world > 1 if collective is None else bool(collective)
        self.dev, self.comm = torch.device(device), torch.device(comm_device)
        self.lay_local = torch.zeros(3, dtype=torch.int64, device=self.dev)
        self.lay_all = torch.zeros(3 * world, dtype=torch.int64, device=self.dev)
        self.out = torch.empty(MAX_SERIALIZED, dtype=torch.uint8, device=self.dev)
        self.runb = torch.empty(KEYS, dtype=torch.uint8, device=self.dev)
        self.ext = torch.cuda.ExternalStream(engine.stream_ptr, device=self.dev)
        torch.cuda.synchronize(self.dev)  # the zero fills (torch's stream) before any engine-stream write

    def place(self):
        import torch
        self.eng.result_layout_device(self.lay_local)
        if self.collective:
            dist = _dist()
            cur = torch.cuda.current_stream(self.dev)
            cur.wait_stream(self.ext)  # the layout is written
            if self.comm.type == "cuda":
                dist.all_gather_into_tensor(self.lay_all, self.lay_local, group=self.group)
            else:  # gloo rehearsal: the collective runs on host memory
                parts = [torch.zeros(3, dtype=torch.int64) for _ in range(self.world)]
                dist.all_gather(parts, self.lay_local.cpu(), group=self.group)
                self.lay_all.copy_(torch.cat(parts))
            self.ext.wait_stream(cur)  # the gathered layout is in place
            lay = self.lay_all
        else:
            lay = self.lay_local
        self.eng.fetch_shard_device_dyn(lay, self.rank, self.world, self.out, self.runb)

    def layout(self):
        """the last step's GlobalLayout (synchronises)"""
        self.eng.sync()
        a = (self.lay_all if self.collective else self.lay_local).cpu().numpy()
        return GlobalLayout(a.reshape(-1, 3))

    def gather(self):
        """Rank 0 receives every other rank's slice into its `out` (each rank's buffer has the
        global layout, so every slice travels to the same place) and packs the run flags.
        Returns the global bitmap (a uint8 tensor view) on rank 0, None elsewhere."""
        import torch
        lay = self.layout()
        r = self.rank

        def views(rr):
            nr, f, b = int(lay.n[rr]), int(lay.first[rr]), int(lay.base[rr])
            v = [self.out[lay.desc_base + 4 * f: lay.desc_base + 4 * (f + nr)]]
            if lay.offsets:
                v.append(self.out[lay.off_base + 4 * f: lay.off_base + 4 * (f + nr)])
            if lay.has_run:
                v.append(self.runb[f: f + nr])
            v.append(self.out[lay.header + b: lay.header + b + int(lay.pay[rr])])
            return [t for t in v if t.numel()]

        on_dev = self.comm.type == "cuda"
        if self.world > 1:
            dist = _dist()
            peer = (lambda x: x) if self.group is None else (lambda x: dist.get_global_rank(self.group, x))
            if r == 0:
                recv = [(t, rr) for rr in range(1, self.world) if int(lay.n[rr]) for t in views(rr)]
                bufs = [(t if on_dev else torch.empty(t.numel(), dtype=torch.uint8), t, rr) for t, rr in recv]
                for q in _p2p([(dist.irecv, b, peer(rr)) for b, _, rr in bufs], self.group) if bufs else []:
                    q.wait()
                if not on_dev:
                    for b, t, _ in bufs:
                        t.copy_(b)
            elif int(lay.n[r]):
                sends = [t if on_dev else t.cpu() for t in views(r)]
                for q in _p2p([(dist.isend, t, peer(0)) for t in sends], self.group):
                    q.wait()
        if r != 0:
            return None
        if lay.has_run and lay.total:
            self.out[4:4 + lay.flag_bytes] = _pack_flags(self.runb[:lay.total])
        torch.cuda.synchronize(self.dev)
        return self.out[:lay.nbytes]
