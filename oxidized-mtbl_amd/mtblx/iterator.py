"""Seek-based iteration: ReaderIntoIter (src/reader.rs:219-405) built by new / new_from /
new_get_prefix / new_get_range, with next() and the mid-iteration seek() (:302-335).

The device does the seeking and decoding (include/mtblx.h "seek-based iteration"):

    index_iter.seek(key) + block_at_index / Reader::block   mtblx_index_seek_batch
    bi.seek(key) / seek_to_first + the block's records        mtblx_block_seek_batch
    landed index entry -> index position (directory entry)    mtblx_entry_offsets
    blocks after the sought one                               mtblx_decode_blocks (only those
                                                              the iteration reaches)
    ReaderIntoIter's stop rules (Get / GetPrefix / GetRange)  mtblx_key_filter

The host keeps the iterator's state exactly as the reference does: `first`, `valid`, the
index position, and `block_offset` -- set to 0 by the constructors and never updated by
next() (:244-246, :269-271, :362-366), so seek() re-seeks whatever block the iterator holds
when the landed index entry's block offset equals it, with that iterator's key capacity
(src/block.rs:106-112, :132).

Two surfaces:
  * `bulk(reader, kind, key, key2)` -> reader.Scan: the whole iteration (iter_from /
    iter_prefix / iter_range) with the records on the device, decoding the sought block's
    tail plus the following blocks in growing chunks until the stop rule or the end.
  * `ReaderIntoIter`: the stateful iterator (next() -> (key, value) | None, seek(key)), host
    records, for callers that interleave seeks and nexts.

One documented approximation: the index seek runs on a fresh index iterator.  The reference
re-seeks its live index iterator, which differs only when the INDEX block's restart entries
are corrupt (BlockIter::seek's early return keeps the old position); such index blocks fail
the checksum at open unless verification is off.
"""
from __future__ import annotations

import bisect
import ctypes as C

import numpy as np
import torch

from . import _lib, codec

ITER, GET, PREFIX, RANGE = 0, 1, 2, 3
KINDS = {"iter": ITER, "from": ITER, "get": GET, "prefix": PREFIX, "range": RANGE}


def _dev_bytes(b: bytes, dev) -> torch.Tensor:
    return torch.frombuffer(bytearray(b or b"\0"), dtype=torch.uint8).to(dev)


# ------------------------------------------------------------------ device primitives
def index_seek(r, key: bytes) -> _lib.IndexSeek:
    """index_iter.seek(key) -> landed entry, its block offset and Reader::block framing."""
    dev = r.file.device
    kb = _dev_bytes(key, dev)
    ke = torch.tensor([len(key)], dtype=torch.int64, device=dev)
    out = torch.zeros(C.sizeof(_lib.IndexSeek), dtype=torch.uint8, device=dev)
    rc = _lib.lib().mtblx_index_seek_batch(C.c_void_p(r.file.data_ptr()), r.len, r.version, 1 if r.verify else 0,
                                           r.index_off, r.index_len, C.c_void_p(kb.data_ptr()),
                                           C.c_void_p(ke.data_ptr()), 1, C.c_void_p(out.data_ptr()),
                                           C.c_void_p(codec._stream_handle(None)))
    if rc != 0:
        raise RuntimeError(f"mtblx_index_seek_batch failed: {rc}")
    return _lib.IndexSeek.from_buffer_copy(out.cpu().numpy().tobytes())


class Emitted:
    """Records one BlockIter yields from its position on (mtblx_block_seek_batch), device."""

    def __init__(self, q: _lib.BlockSeek, keys, vals, key_end, val_end, kcaps):
        self.status, self.end, self.entry = int(q.status), int(q.end), int(q.entry)
        self.nrec, self.kcap_end = int(q.nrec), int(q.kcap)
        self.has_val, self.last_voff, self.last_vlen = bool(q.has_val), int(q.last_voff), int(q.last_vlen)
        self.keys, self.vals, self.key_end, self.val_end, self.kcaps = keys, vals, key_end, val_end, kcaps

    def host_records(self):
        ke = self.key_end.cpu().numpy()
        ve = self.val_end.cpu().numpy()
        k = self.keys.cpu().numpy().tobytes()
        v = self.vals.cpu().numpy().tobytes()
        out, pk, pv = [], 0, 0
        for i in range(self.nrec):
            out.append((k[pk: ke[i]], v[pv: ve[i]]))
            pk, pv = int(ke[i]), int(ve[i])
        return out


def block_seek(content, key: bytes | None, kcap: int = 0, max_records: int = 1 << 62,
               small_caps: bool = False) -> Emitted:
    """BlockIter::seek(key) (key None: seek_to_first) on content = (tensor, off, len) with the
    given key capacity, then the records it yields until get() is None.  small_caps: start
    from small output buffers and size them exactly from the first pass's counts (blocks of
    GiBs)."""
    data, off, ln = content
    dev = data.device
    kb = _dev_bytes(key or b"", dev)
    ke = torch.tensor([len(key or b"")], dtype=torch.int64, device=dev)
    q = _lib.BlockSeek(data_off=off, data_len=ln, kcap=kcap, max_records=max_records, first=1 if key is None else 0)
    rec_cap = min(max_records, ln // 3 + 1)
    keys_cap, vals_cap = 2 * ln + 64, ln + 16
    if small_caps:
        rec_cap, keys_cap, vals_cap = min(rec_cap, 1 << 16), min(keys_cap, 1 << 20), min(vals_cap, 1 << 20)
    for _ in range(3):
        qt = torch.frombuffer(bytearray(bytes(q)), dtype=torch.uint8).to(dev)
        okeys = torch.empty(max(keys_cap, 1), dtype=torch.uint8, device=dev)
        ovals = torch.empty(max(vals_cap, 1), dtype=torch.uint8, device=dev)
        oke = torch.empty(max(rec_cap, 1), dtype=torch.int64, device=dev)
        ove = torch.empty(max(rec_cap, 1), dtype=torch.int64, device=dev)
        okc = torch.empty(max(rec_cap, 1), dtype=torch.int64, device=dev)
        rc = _lib.lib().mtblx_block_seek_batch(C.c_void_p(data.data_ptr()), C.c_void_p(kb.data_ptr()),
                                               C.c_void_p(ke.data_ptr()), 1, C.c_void_p(qt.data_ptr()),
                                               C.c_void_p(okeys.data_ptr()), keys_cap, C.c_void_p(ovals.data_ptr()),
                                               vals_cap, C.c_void_p(oke.data_ptr()), C.c_void_p(ove.data_ptr()),
                                               C.c_void_p(okc.data_ptr()), rec_cap,
                                               C.c_void_p(codec._stream_handle(None)))
        if rc != 0:
            raise RuntimeError(f"mtblx_block_seek_batch failed: {rc}")
        res = _lib.BlockSeek.from_buffer_copy(qt.cpu().numpy().tobytes())
        if res.end != _lib.EMIT_OVERFLOW:
            n = int(res.nrec)
            return Emitted(res, okeys[: int(res.key_bytes)], ovals[: int(res.val_bytes)], oke[:n], ove[:n], okc[:n])
        rec_cap, keys_cap, vals_cap = int(res.nrec), int(res.key_bytes), int(res.val_bytes)
    raise RuntimeError("mtblx_block_seek_batch: output sizes did not converge")


def key_filter(keys: torch.Tensor, key_end: torch.Tensor, n: int, typ: int, k: bytes) -> int:
    """index of the first record the stop rule of `typ` rejects, or n"""
    if n == 0 or typ == ITER:
        return n
    dev = keys.device
    kt = _dev_bytes(k, dev)
    ff = torch.full((1,), n, dtype=torch.int64, device=dev)
    kk = keys if keys.numel() else torch.zeros(1, dtype=torch.uint8, device=dev)
    rc = _lib.lib().mtblx_key_filter(C.c_void_p(kk.data_ptr()), C.c_void_p(key_end.data_ptr()), n, typ,
                                     C.c_void_p(kt.data_ptr()), len(k), C.c_void_p(ff.data_ptr()),
                                     C.c_void_p(codec._stream_handle(None)))
    if rc != 0:
        raise RuntimeError(f"mtblx_key_filter failed: {rc}")
    return int(ff.item())


def prefix_successor(p: bytes):
    """smallest key greater than every key starting with p (None: no such key)"""
    b = bytearray(p)
    while b and b[-1] == 0xFF:
        b.pop()
    if not b:
        return None
    b[-1] += 1
    return bytes(b)


# ------------------------------------------------------------------ bulk iteration
def bulk(r, kind: str, key: bytes, key2: bytes = b""):
    """ReaderIntoIter::new_from / new_get_prefix / new_get_range (src/reader.rs:256-300) run to
    the end -> reader.Scan with the records on the device."""
    from .reader import (END_ERR_NEXT, END_ERR_OPEN, END_LOOP, END_NONE, END_PANIC, MtblError, ReferencePanic, Scan)
    typ = KINDS[kind]
    k = key2 if typ == RANGE else key
    dev = r.file.device

    def empty(end, err="None"):
        z = torch.zeros(0, dtype=torch.uint8, device=dev)
        e = torch.zeros(0, dtype=torch.int64, device=dev)
        return Scan(end, err, 0, z, z, e, e)

    s = index_seek(r, key)
    if s.status == _lib.SEEK_PANIC:
        return empty(END_PANIC)
    if s.status == _lib.SEEK_LOOP:
        return empty(END_LOOP)
    if not s.valid:
        return empty(END_NONE)            # no index entry: bi is None, next() -> None
    e = r._ordinal(int(s.entry))
    try:
        content = r._seek_content(s)
    except MtblError as x:
        return empty(END_ERR_OPEN, x.args[0])
    except ReferencePanic:
        return empty(END_PANIC)
    head = block_seek(content, key)
    if head.status == _lib.SEEK_ERR:
        return empty(END_ERR_OPEN, "InvalidBlock")
    if head.status == _lib.SEEK_PANIC:
        return empty(END_PANIC)
    if head.status == _lib.SEEK_LOOP:
        return empty(END_LOOP)
    if head.status == _lib.SEEK_UNSUPPORTED:
        raise NotImplementedError("emitting seek: block >= 4 GiB or key > 64 KiB")
    parts = [(head.keys, head.vals, head.key_end, head.val_end, head.nrec)]
    end, err = END_NONE, "None"
    stop = key_filter(head.keys, head.key_end, head.nrec, typ, k)
    if stop < head.nrec:
        parts[0] = _cut_part(parts[0], stop)
    elif head.end == _lib.EMIT_PANIC:
        end = END_PANIC
    elif head.end == _lib.EMIT_LOOP:
        end = END_LOOP
    else:
        # the following blocks, in chunks: up to the index entry whose separator reaches the
        # stop key (well-formed files end there), doubling while the iteration goes on
        i0 = e + 1
        stop_key = None if typ == ITER else (k if typ in (GET, RANGE) else prefix_successor(k))
        grow = 1
        while True:
            if i0 >= r.nent:
                end = END_PANIC if r.index_status == _lib.ST_CORRUPT else END_LOOP if r.index_status == _lib.ST_LOOP \
                    else END_NONE
                break
            if stop_key is None:
                i1 = r.nent
            else:
                j = bisect.bisect_left(r._index_keys(), stop_key)
                i1 = min(r.nent, max(j + 1, i0 + grow))
            part, pend, perr, stopped = r._walk_range(i0, i1)
            n = part[4]
            cut = key_filter(part[0], part[2], n, typ, k)
            if cut < n:
                parts.append(_cut_part(part, cut))
                break
            parts.append(part)
            if stopped:
                end, err = pend, perr
                break
            grow = 2 * (i1 - i0)
            i0 = i1
    return _assemble(parts, end, err, dev)


def _cut_part(part, n):
    keys, vals, ke, ve, _ = part
    kl = int(ke[n - 1].item()) if n else 0
    vl = int(ve[n - 1].item()) if n else 0
    return keys[:kl], vals[:vl], ke[:n], ve[:n], n


def _assemble(parts, end, err, dev):
    from .reader import Scan
    parts = [p for p in parts if p[4] > 0]
    if not parts:
        z = torch.zeros(0, dtype=torch.uint8, device=dev)
        e = torch.zeros(0, dtype=torch.int64, device=dev)
        return Scan(end, err, 0, z, z, e, e)
    kb = vb = 0
    K, V, KE, VE = [], [], [], []
    for keys, vals, ke, ve, n in parts:
        K.append(keys)
        V.append(vals)
        KE.append(ke + kb)
        VE.append(ve + vb)
        kb += keys.numel()
        vb += vals.numel()
    nrec = sum(p[4] for p in parts)
    return Scan(end, err, nrec, torch.cat(K), torch.cat(V), torch.cat(KE), torch.cat(VE))


# ------------------------------------------------------------------ stateful iterator
class _Bi:
    """one BlockIter as the host iterator holds it: the records from its position on"""

    def __init__(self, content, recs, end, kcaps=None, kcap_end=0):
        self.content = content      # (tensor, off, len): re-seeks and key capacities
        self.recs = recs
        self.end = end              # EMIT_END / EMIT_PANIC / EMIT_LOOP after the last record
        self.kcaps = kcaps          # key capacity at each record (None: from seek_to_first, lazily)
        self.kcap_end = kcap_end
        self.pos = 0
        self.last_val = None        # value of the last entry a seek parsed (None: val is None)

    def kcap(self) -> int:
        """the key Vec's capacity now (parse_next_key's END leaves it unchanged)"""
        if not self.recs:
            return self.kcap_end
        if self.kcaps is None:   # records came from the bulk decoder: replay seek_to_first + next
            em = block_seek(self.content, None, 0, len(self.recs))
            self.kcaps = em.kcaps.cpu().numpy().tolist()
        return int(self.kcaps[min(self.pos, len(self.recs) - 1)])


class ReaderIntoIter:
    """src/reader.rs:219-405.  kind: "iter" (Reader::into_iter), "from", "get", "prefix",
    "range" (end key = key2, inclusive).  next() -> (key, value) or None; raises MtblError for
    Some(Err(e)) / Err at construction, ReferencePanic where the reference panics,
    ReferenceLoop where it never returns."""

    def __init__(self, r, kind: str = "iter", key: bytes = b"", key2: bytes = b""):
        from .reader import ReferenceLoop, ReferencePanic
        self.r = r
        self.type = KINDS[kind]
        self.k = bytes(key2 if kind == "range" else key)
        self.block_offset = 0
        self.first = True
        self.valid = True
        self.bi = None
        self.e = None                # index position (directory entry), None: index iterator invalid
        self._chunk = None           # prefetched blocks: (i0, [ _Bi | exception ])
        self._grow = 1
        if kind == "iter":           # new (:231-254): index seek_to_first, block_at_index, seek_to_first
            if r.nent == 0:
                if r.index_status == _lib.ST_CORRUPT:
                    raise ReferencePanic("index block: first entry")
                return
            self.e = 0
            self.bi = self._load(0)
            return
        key = bytes(key)
        s = index_seek(r, key)       # new_from (:256-279)
        if s.status == _lib.SEEK_PANIC:
            raise ReferencePanic("index seek")
        if s.status == _lib.SEEK_LOOP:
            raise ReferenceLoop("index seek")
        if not s.valid:
            return
        self.e = r._ordinal(int(s.entry))
        self.bi = self._seek_block(r._seek_content(s), key, 0)

    # the block of directory entry i as next() loads it (Reader::block + seek_to_first)
    def _load(self, i: int) -> _Bi:
        if self._chunk is None or not (self._chunk[0] <= i < self._chunk[0] + len(self._chunk[1])):
            n = min(self.r.nent - i, self._grow)
            self._grow = min(2 * self._grow, 256)
            self._chunk = (i, self.r._host_blocks(i, i + n))
        b = self._chunk[1][i - self._chunk[0]]
        if isinstance(b, Exception):
            raise b
        return _Bi(b[0], list(b[1]), b[2])

    def _seek_block(self, content, key: bytes, kcap: int) -> _Bi:
        from .reader import MtblError, ReferenceLoop, ReferencePanic
        em = block_seek(content, key, kcap)
        if em.status == _lib.SEEK_ERR:
            raise MtblError(6)
        if em.status == _lib.SEEK_PANIC:
            raise ReferencePanic("BlockIter::seek")
        if em.status == _lib.SEEK_LOOP:
            raise ReferenceLoop("BlockIter::seek")
        if em.status == _lib.SEEK_UNSUPPORTED:
            raise NotImplementedError("emitting seek: block >= 4 GiB or key > 64 KiB")
        bi = _Bi(content, em.host_records(), em.end, em.kcaps.cpu().numpy().tolist(), em.kcap_end)
        if em.has_val:   # BlockIter::val of the last parsed entry (Reader::get's Err quirk)
            d, o, _ = content
            bi.last_val = d[o + em.last_voff: o + em.last_voff + em.last_vlen].cpu().numpy().tobytes()
        return bi

    def __iter__(self):
        return self

    def __next__(self):
        rec = self.next()
        if rec is None:
            raise StopIteration
        return rec

    def next(self):
        from .reader import ReferenceLoop, ReferencePanic
        if not self.valid or self.bi is None:
            return None
        bi = self.bi
        if not self.first and bi.pos < len(bi.recs):
            bi.pos += 1                                   # bi.next()
        self.first = False
        if bi.pos == len(bi.recs) and bi.end == _lib.EMIT_PANIC:
            raise ReferencePanic("BlockIter::next / get")
        if bi.pos == len(bi.recs) and bi.end == _lib.EMIT_LOOP:
            raise ReferenceLoop("BlockIter::next")
        if bi.pos < len(bi.recs):
            rec = bi.recs[bi.pos]
        else:
            self.valid = False
            if self.e is None:
                return None
            if self.e + 1 >= self.r.nent:                 # index_iter.next() past the last entry
                st = self.r.index_status
                self.e = None
                if st == _lib.ST_CORRUPT:
                    raise ReferencePanic("index block: next entry")
                if st == _lib.ST_LOOP:
                    raise ReferenceLoop("index block: next entry")
                return None
            self.e += 1
            nb = self._load(self.e)                       # Some(Err(e)) raises; valid stays false
            self.bi = nb
            if nb.end == _lib.EMIT_PANIC and not nb.recs:
                raise ReferencePanic("BlockIter::seek_to_first / get")
            if not nb.recs:
                return None
            self.valid = True
            rec = nb.recs[0]
        k = rec[0]
        if self.type == GET and k != self.k:
            self.valid = False
        elif self.type == PREFIX and not k.startswith(self.k):
            self.valid = False
        elif self.type == RANGE and k > self.k:
            self.valid = False
        return rec if self.valid else None

    def seek(self, key: bytes) -> bool:
        """ReaderIntoIter::seek (:302-335): Ok(true), or raises (Err / panic / loop)."""
        from .reader import ReferenceLoop, ReferencePanic
        key = bytes(key)
        s = index_seek(self.r, key)
        if s.status == _lib.SEEK_PANIC:
            raise ReferencePanic("index seek")
        if s.status == _lib.SEEK_LOOP:
            raise ReferenceLoop("index seek")
        if not s.valid:
            self.valid = False
            self.e = None
            return True
        self.e = self.r._ordinal(int(s.entry))
        if self.block_offset != int(s.block_off):
            self.block_offset = int(s.block_off)          # updated before the load (:322)
            self.bi = self._seek_block(self.r._seek_content(s), key, 0)
        elif self.bi is not None:                         # the held block, whatever it is
            self.bi = self._seek_block(self.bi.content, key, self.bi.kcap())
        self.first = True
        self.valid = True
        return True
