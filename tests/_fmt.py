"""Independent encoder/decoder of the portable Roaring format, for building test
inputs with explicit container types (RB/RoaringArray.java:896-940).  Test-only."""
import struct

import numpy as np

A, B, R = 0, 1, 2


def runs_of(vals):
    vals = np.asarray(vals, dtype=np.int64)
    if vals.size == 0:
        return []
    brk = np.nonzero(np.diff(vals) != 1)[0]
    starts = np.concatenate([[0], brk + 1])
    ends = np.concatenate([brk, [vals.size - 1]])
    return [(int(vals[s]), int(vals[e] - vals[s])) for s, e in zip(starts, ends)]


def encode(containers):
    """containers: list of (key, kind, sorted unique uint16 values)."""
    containers = sorted(containers, key=lambda c: c[0])
    size = len(containers)
    has_run = any(k == R for _, k, _ in containers)
    payloads = []
    for key, kind, vals in containers:
        vals = np.asarray(vals, dtype=np.uint16)
        if kind == A:
            payloads.append(vals.astype("<u2").tobytes())
        elif kind == B:
            w = np.zeros(1024, dtype=np.uint64)
            np.bitwise_or.at(w, vals.astype(np.int64) >> 6, np.uint64(1) << (vals.astype(np.uint64) & np.uint64(63)))
            payloads.append(w.astype("<u8").tobytes())
        else:
            rs = runs_of(vals)
            payloads.append(struct.pack("<H", len(rs)) + b"".join(struct.pack("<HH", s, l) for s, l in rs))
    out = bytearray()
    if has_run:
        out += struct.pack("<I", 12347 | ((size - 1) << 16))
        fl = bytearray((size + 7) // 8)
        for i, (_, k, _) in enumerate(containers):
            if k == R:
                fl[i // 8] |= 1 << (i % 8)
        out += fl
        header = 4 + len(fl) + (4 * size if size < 4 else 8 * size)
    else:
        out += struct.pack("<II", 12346, size)
        header = 8 + 8 * size
    for key, kind, vals in containers:
        out += struct.pack("<HH", key, len(vals) - 1)
    if not has_run or size >= 4:
        off = header
        for p in payloads:
            out += struct.pack("<I", off)
            off += len(p)
    for p in payloads:
        out += p
    return bytes(out)


def decode(buf):
    """-> list of (key, kind, card, values ndarray)"""
    cookie = struct.unpack_from("<I", buf, 0)[0]
    pos = 4
    has_run = (cookie & 0xFFFF) == 12347
    if has_run:
        size = (cookie >> 16) + 1
        fl = buf[pos:pos + (size + 7) // 8]
        pos += (size + 7) // 8
    else:
        assert cookie == 12346
        size = struct.unpack_from("<I", buf, pos)[0]
        pos += 4
        fl = b""
    desc = [struct.unpack_from("<HH", buf, pos + 4 * i) for i in range(size)]
    pos += 4 * size
    if not has_run or size >= 4:
        pos += 4 * size
    out = []
    for i, (key, c1) in enumerate(desc):
        card = c1 + 1
        is_run = has_run and (fl[i // 8] >> (i % 8)) & 1
        if is_run:
            nr = struct.unpack_from("<H", buf, pos)[0]
            pr = np.frombuffer(buf, dtype="<u2", count=2 * nr, offset=pos + 2).astype(np.int64)
            pos += 2 + 4 * nr
            vals = np.concatenate([np.arange(s, s + l + 1) for s, l in zip(pr[0::2], pr[1::2])]) if nr else np.zeros(0)
            out.append((key, R, card, vals.astype(np.uint16), nr))
        elif card > 4096:
            w = np.frombuffer(buf, dtype="<u8", count=1024, offset=pos)
            pos += 8192
            bits = np.unpackbits(w.view(np.uint8), bitorder="little")
            out.append((key, B, card, np.nonzero(bits)[0].astype(np.uint16), 0))
        else:
            vals = np.frombuffer(buf, dtype="<u2", count=card, offset=pos).copy()
            pos += 2 * card
            out.append((key, A, card, vals, 0))
    return out


def kinds(buf):
    return [c[1] for c in decode(buf)]


def container_table(buf):
    """Fast container table of a serialized bitmap (numpy over the descriptors and the
    offset table): -> (keys, kinds, cards, payload offsets, payload lengths)."""
    cookie = struct.unpack_from("<I", buf, 0)[0]
    has_run = (cookie & 0xFFFF) == 12347
    if has_run:
        size = (cookie >> 16) + 1
        fl = np.frombuffer(buf, dtype=np.uint8, count=(size + 7) // 8, offset=4)
        pos = 4 + (size + 7) // 8
        is_run = ((fl[np.arange(size) // 8] >> (np.arange(size) % 8)) & 1).astype(bool)
    else:
        size = struct.unpack_from("<I", buf, 4)[0]
        pos = 8
        is_run = np.zeros(size, dtype=bool)
    d = np.frombuffer(buf, dtype="<u2", count=2 * size, offset=pos).reshape(-1, 2).astype(np.int64)
    keys, cards = d[:, 0], d[:, 1] + 1
    pos += 4 * size
    kinds = np.where(is_run, R, np.where(cards > 4096, B, A))
    if not has_run or size >= 4:
        offs = np.frombuffer(buf, dtype="<u4", count=size, offset=pos).astype(np.int64)
    else:  # walk (size < 4)
        offs, p = [], pos
        for i in range(size):
            offs.append(p)
            p += 2 + 4 * struct.unpack_from("<H", buf, p)[0] if kinds[i] == R else (8192 if kinds[i] == B else 2 * cards[i])
        offs = np.array(offs, dtype=np.int64)
    lens = np.where(kinds == B, 8192, 2 * cards)
    for i in np.nonzero(kinds == R)[0]:
        lens[i] = 2 + 4 * struct.unpack_from("<H", buf, int(offs[i]))[0]
    return keys, kinds, cards, offs, lens


def sub_bitmap(buf, keep_keys):
    """The serialized bitmap holding only the containers of `buf` whose key is in keep_keys
    (payload bytes copied verbatim; header per RB/RoaringArray.java:896-940)."""
    keys, kinds, cards, offs, lens = container_table(buf)
    sel = np.nonzero(np.isin(keys, np.asarray(list(keep_keys), dtype=np.int64)))[0]
    size = len(sel)
    has_run = bool(np.any(kinds[sel] == R))
    out = bytearray()
    if has_run:
        out += struct.pack("<I", 12347 | ((size - 1) << 16))
        fl = bytearray((size + 7) // 8)
        for j, i in enumerate(sel):
            if kinds[i] == R:
                fl[j // 8] |= 1 << (j % 8)
        out += fl
        header = 4 + len(fl) + (4 * size if size < 4 else 8 * size)
    else:
        out += struct.pack("<II", 12346, size)
        header = 8 + 8 * size
    for i in sel:
        out += struct.pack("<HH", int(keys[i]), int(cards[i] - 1))
    if not has_run or size >= 4:
        off = header
        for i in sel:
            out += struct.pack("<I", off)
            off += int(lens[i])
    for i in sel:
        out += buf[int(offs[i]):int(offs[i] + lens[i])]
    return bytes(out)
