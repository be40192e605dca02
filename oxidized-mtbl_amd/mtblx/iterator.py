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

ReaderIntoIter::seek (:302-335) re-seeks the LIVE index iterator (:303) and then seeks the
data block with the landed INDEX entry's key -- `key` is shadowed at :305 -- so seek(k) +
next() yields the first record >= the separator, not >= k.

The index iterator.  When the index block is *regular* (mtblx_entry_offsets: chains land on
the restart points, restart entries have shared == 0, no entry has shared > the previous key's
length), a seek from any index iterator state lands on the scan chain with the scan's own key
and the key-capacity assert cannot fire, so the index position is a directory entry and the
blocks after it come from the directory (batched decode).  Otherwise (a corrupt index, read
with verification off) the live index iterator is driven on the device exactly:
mtblx_block_seek_batch seeks the index block with the iterator's key capacity (an early return
keeps the old position) and emits the records next() visits from the landing, on the scan
chain or not; `_IxList` holds them, resuming the emission when it runs out.
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
        self.early, self.stop_off = bool(q.early), int(q.stop_off)
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


_BIG_BLOCK = 64 << 20   # past this, the values move with the whole grid whatever the caller asks


def block_seek(content, key: bytes | None, kcap: int = 0, max_records: int = 1 << 62,
               small_caps: bool = False, resume_off: int | None = None, values: bool = True) -> Emitted:
    """BlockIter::seek(key) (key None: seek_to_first) on content = (tensor, off, len) with the
    given key capacity, then the records it yields until get() is None.  resume_off: instead
    of seeking, an iterator holding key bytes `key` and capacity kcap calls next(), which
    parses the entry at resume_off.  small_caps: start from small output buffers and size them
    exactly from the first pass's counts, and move the value bytes with the whole grid
    (mtblx_block_seek_batch_ex + mtblx_copy_ranges) instead of the seeking wave (blocks of GiBs).
    values=False: the value bytes are not moved at all (the emission's key capacities only)."""
    defer = small_caps or not values or content[2] > _BIG_BLOCK
    data, off, ln = content
    dev = data.device
    kb = _dev_bytes(key or b"", dev)
    ke = torch.tensor([len(key or b"")], dtype=torch.int64, device=dev)
    first = 2 if resume_off is not None else (1 if key is None else 0)
    q = _lib.BlockSeek(data_off=off, data_len=ln, kcap=kcap, max_records=max_records, first=first,
                       resume_off=resume_off or 0)
    rec_cap = min(max_records, ln // 3 + 1)
    keys_cap, vals_cap = 2 * ln + 64, ln + 16
    if small_caps:
        rec_cap, keys_cap, vals_cap = min(rec_cap, 1 << 16), min(keys_cap, 1 << 20), min(vals_cap, 1 << 20)
    kbuf = None   # the iterator's key: 64 KiB of LDS, or (a longer key) a device buffer
    for _ in range(4):
        qt = torch.frombuffer(bytearray(bytes(q)), dtype=torch.uint8).to(dev)
        okeys = torch.empty(max(keys_cap, 1), dtype=torch.uint8, device=dev)
        ovals = torch.empty(max(vals_cap, 1), dtype=torch.uint8, device=dev)
        oke = torch.empty(max(rec_cap, 1), dtype=torch.int64, device=dev)
        ove = torch.empty(max(rec_cap, 1), dtype=torch.int64, device=dev)
        okc = torch.empty(max(rec_cap, 1), dtype=torch.int64, device=dev)
        vsrc = torch.empty(max(rec_cap, 1), dtype=torch.int64, device=dev) if defer else None
        args = [C.c_void_p(data.data_ptr()), C.c_void_p(kb.data_ptr()), C.c_void_p(ke.data_ptr()), 1,
                C.c_void_p(qt.data_ptr()), C.c_void_p(okeys.data_ptr()), keys_cap, C.c_void_p(ovals.data_ptr()),
                vals_cap, C.c_void_p(oke.data_ptr()), C.c_void_p(ove.data_ptr()), C.c_void_p(okc.data_ptr()), rec_cap]
        if defer:
            rc = _lib.lib().mtblx_block_seek_batch_ex(*args, C.c_void_p(kbuf.data_ptr() if kbuf is not None else 0),
                                                      kbuf.numel() if kbuf is not None else 0,
                                                      C.c_void_p(vsrc.data_ptr()), C.c_void_p(codec._stream_handle(None)))
        elif kbuf is None:
            rc = _lib.lib().mtblx_block_seek_batch(*args, C.c_void_p(codec._stream_handle(None)))
        else:
            rc = _lib.lib().mtblx_block_seek_batch_kbuf(*args, C.c_void_p(kbuf.data_ptr()), kbuf.numel(),
                                                        C.c_void_p(codec._stream_handle(None)))
        if rc != 0:
            raise RuntimeError(f"mtblx_block_seek_batch failed: {rc}")
        res = _lib.BlockSeek.from_buffer_copy(qt.cpu().numpy().tobytes())
        if res.status == _lib.SEEK_UNSUPPORTED and kbuf is None:
            # a key past 64 KiB: again with the key in device memory, sized for any key this
            # iterator can build (the held key plus every suffix in the block)
            kbuf = torch.empty(len(key or b"") + ln + 64, dtype=torch.uint8, device=dev)
            continue
        if res.end != _lib.EMIT_OVERFLOW:
            n = int(res.nrec)
            if defer and values and n:
                _copy_values(data, off, vsrc[:n], ove[:n], ovals)
            return Emitted(res, okeys[: int(res.key_bytes)], ovals[: int(res.val_bytes)], oke[:n], ove[:n], okc[:n])
        rec_cap, keys_cap, vals_cap = int(res.nrec), int(res.key_bytes), int(res.val_bytes)
    raise RuntimeError("mtblx_block_seek_batch: output sizes did not converge")


def _copy_values(data, off: int, vsrc, vend, ovals):
    """the emitted records' values, block content offsets vsrc -> ovals at their END offsets vend
    (mtblx_copy_ranges: every CU moves the GiBs)"""
    start = torch.cat([torch.zeros(1, dtype=torch.int64, device=vend.device), vend[:-1]])
    ln = vend - start
    chunks = (ln + 15) // 16
    base = torch.cumsum(chunks, 0) - chunks
    total = int(chunks.sum().item())
    src_off = (vsrc + off).contiguous()
    rc = _lib.lib().mtblx_copy_ranges(C.c_void_p(data.data_ptr()), C.c_void_p(src_off.data_ptr()),
                                      C.c_void_p(ovals.data_ptr()), C.c_void_p(start.data_ptr()),
                                      C.c_void_p(ln.data_ptr()), C.c_void_p(base.data_ptr()), int(vend.numel()),
                                      total, C.c_void_p(codec._stream_handle(None)))
    if rc != 0:
        raise RuntimeError(f"mtblx_copy_ranges failed: {rc}")


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


def _varint_decode64(v: bytes) -> int:
    """varint_decode64(val, &mut offset) of an index value (src/varint.rs:78-97, host C++)"""
    from .reader import ReferencePanic
    out = C.c_uint64(0)
    b = np.frombuffer(v or b"\0", np.uint8)
    if _lib.lib().mtblx_varint_decode64(b.ctypes.data_as(_lib.u8p), len(v), C.byref(out)) < 0:
        raise ReferencePanic("varint_decode64 of the index value")
    return int(out.value)


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
    if not r.index_regular():
        return _bulk_stateful(r, kind, key, key2)

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
        raise RuntimeError("emitting seek: key buffer too small")
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


def _bulk_stateful(r, kind: str, key: bytes, key2: bytes):
    """new_from / new_get_prefix / new_get_range run to the end on a corrupt (irregular) index:
    the stateful iterator below, which follows the live index iterator exactly; the records
    are uploaded as a Scan"""
    from .reader import END_ERR_NEXT, END_ERR_OPEN, END_LOOP, END_NONE, END_PANIC, MtblError, ReferenceLoop, \
        ReferencePanic
    recs, end, err = [], END_NONE, "None"
    try:
        it = ReaderIntoIter(r, kind, key, key2)
    except MtblError as x:
        it, end, err = None, END_ERR_OPEN, x.args[0]
    except ReferencePanic:
        it, end = None, END_PANIC
    except ReferenceLoop:
        it, end = None, END_LOOP
    if it is not None:
        it.bulk = True
        try:
            while True:
                rec = it.next()
                if rec is None:
                    break
                recs.append(rec)
        except MtblError as x:
            end, err = END_ERR_NEXT, x.args[0]
        except ReferencePanic:
            end = END_PANIC
        except ReferenceLoop:
            end = END_LOOP
    return _from_host(recs, end, err, r.file.device)


def _from_host(recs, end, err, dev):
    from .reader import Scan
    kb = b"".join(k for k, _ in recs)
    vb = b"".join(v for _, v in recs)
    ke = np.cumsum([len(k) for k, _ in recs], dtype=np.int64)
    ve = np.cumsum([len(v) for _, v in recs], dtype=np.int64)
    return Scan(end, err, len(recs), _dev_bytes(kb, dev)[: len(kb)], _dev_bytes(vb, dev)[: len(vb)],
                torch.from_numpy(ke).to(dev), torch.from_numpy(ve).to(dev))


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
            em = block_seek(self.content, None, 0, len(self.recs), values=False)
            self.kcaps = em.kcaps.cpu().numpy().tolist()
        return int(self.kcaps[min(self.pos, len(self.recs) - 1)])


class _IxList:
    """the live index iterator of an irregular index (src/reader.rs:223): the records its
    next() visits from its current position on, with the key capacity at each, as
    mtblx_block_seek_batch emitted them; `end` says what the next() after the last one does.
    ord0: directory entry of record 0 when the landing lies on the scan chain (the records
    then name the directory's blocks, which next() may load from the batched decode)"""

    EMIT = 256   # records per emission

    def __init__(self, em: "Emitted | None", ord0):
        if em is None:                     # BlockIter::init: invalid, key capacity 0
            self.recs, self.kcaps, self.end, self.stop_off, self.kcap_end = [], [], _lib.EMIT_END, 0, 0
        else:
            self.recs = em.host_records()
            self.kcaps = em.kcaps.cpu().numpy().tolist()
            self.end, self.stop_off, self.kcap_end = em.end, em.stop_off, em.kcap_end
        self.pos = 0
        self.ord0 = ord0

    def valid(self) -> bool:
        return self.pos < len(self.recs)

    def kcap(self) -> int:
        return int(self.kcaps[self.pos]) if self.valid() else int(self.kcap_end)

    def ordinal(self, r):
        """directory entry of the current record, or None (off the chain / past the directory)"""
        if self.ord0 is None:
            return None
        j = self.ord0 + self.pos
        return j if j < r.nent else None


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
        self.e = None                # regular index: index position (directory entry), None: invalid
        self.ix = None               # irregular index: the live index iterator (_IxList)
        self.bulk = False            # driven to the end by bulk(): a looping index never returns
        self._chunk = None           # prefetched blocks: (i0, [ _Bi | exception ])
        self._grow = 1
        self._vchunk = None          # irregular index: prefetched blocks of the current _IxList
        regular = kind == "iter" or r.index_regular()
        if kind == "iter":           # new (:231-254): index seek_to_first, block_at_index, seek_to_first
            if r.nent == 0:
                if r.index_status == _lib.ST_CORRUPT:
                    raise ReferencePanic("index block: first entry")
                if not r.index_regular():
                    self.ix = _IxList(None, None)
                return
            if not r.index_regular():   # the scan's own chain = the directory, with its key capacities
                self.ix = _IxList(block_seek(r.index_content(), None, 0, _IxList.EMIT), 0)
            else:
                self.e = 0
            self.bi = self._load(0)
            return
        key = bytes(key)
        if regular:
            s = index_seek(r, key)       # new_from (:256-279)
            if s.status == _lib.SEEK_PANIC:
                raise ReferencePanic("index seek")
            if s.status == _lib.SEEK_LOOP:
                raise ReferenceLoop("index seek")
            if not s.valid:
                return
            self.e = r._ordinal(int(s.entry))
            self.bi = self._seek_block(r._seek_content(s), key, 0)
            return
        self.ix = _IxList(None, None)    # a fresh index iterator, seeked
        self._ix_seek(key)
        if not self.ix.valid():
            return
        self.bi = self._seek_block(r._value_content(self.ix.recs[self.ix.pos][1]), key, 0)

    # ---------------------------------------------------------------- the index iterator
    def _ix_seek(self, key: bytes):
        """index_iter.seek(key) on the live iterator of an irregular index (src/block.rs:154-194)"""
        from .reader import ReferenceLoop, ReferencePanic
        em = block_seek(self.r.index_content(), key, self.ix.kcap(), _IxList.EMIT)
        if em.status == _lib.SEEK_PANIC:
            raise ReferencePanic("index seek")
        if em.status == _lib.SEEK_LOOP:
            raise ReferenceLoop("index seek")
        if em.status == _lib.SEEK_UNSUPPORTED:
            raise RuntimeError("emitting seek: key buffer too small")
        if em.early:                 # returned on a corrupt restart entry: the old position stays
            return
        self.ix = _IxList(em, self.r._chain_ordinal(em.entry) if em.nrec else None)
        self._vchunk = None

    def _ix_next(self) -> bool:
        """index_iter.next() (src/block.rs:196-202) on the live iterator"""
        from .reader import ReferenceLoop, ReferencePanic
        ix = self.ix
        if not ix.valid():
            return False
        if ix.pos + 1 < len(ix.recs):
            ix.pos += 1
            return True
        if ix.end == _lib.EMIT_END:
            ix.pos = len(ix.recs)
            return False
        if ix.end == _lib.EMIT_PANIC:
            raise ReferencePanic("index block: next entry")
        if ix.end == _lib.EMIT_LOOP:   # a zero-progress entry: next() parses it again, same record
            if self.bulk:
                raise ReferenceLoop("index block: next entry")
            return True
        # EMIT_MAX: the entry after the last record, parsed from that record's key / capacity
        k, _ = ix.recs[-1]
        em = block_seek(self.r.index_content(), k, int(ix.kcaps[-1]), _IxList.EMIT, resume_off=ix.stop_off)
        if em.status == _lib.SEEK_PANIC:
            raise ReferencePanic("index block: next entry")
        if em.status == _lib.SEEK_UNSUPPORTED:
            raise RuntimeError("emitting seek: key buffer too small")
        self.ix = _IxList(em, None if ix.ord0 is None else ix.ord0 + len(ix.recs))
        self._vchunk = None
        return self.ix.valid()

    def _ix_load(self) -> "_Bi":
        """block_at_index of the live index iterator's record (Reader::block + seek_to_first)"""
        ix = self.ix
        j = ix.ordinal(self.r)
        if j is not None:
            return self._load(j)
        if self._vchunk is None or not (self._vchunk[0] <= ix.pos < self._vchunk[0] + len(self._vchunk[1])):
            n = min(len(ix.recs) - ix.pos, self._grow)
            self._grow = min(2 * self._grow, 256)
            self._vchunk = (ix.pos, self.r._value_blocks([v for _, v in ix.recs[ix.pos: ix.pos + n]]))
        b = self._vchunk[1][ix.pos - self._vchunk[0]]
        if isinstance(b, Exception):
            raise b
        return _Bi(b[0], list(b[1]), b[2])

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
            raise RuntimeError("emitting seek: key buffer too small")
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
            if self.ix is not None:                       # irregular index: the live iterator
                if not self._ix_next():
                    return None
                nb = self._ix_load()                      # Some(Err(e)) raises; valid stays false
            else:
                if self.e is None:
                    return None
                if self.e + 1 >= self.r.nent:             # index_iter.next() past the last entry
                    st = self.r.index_status
                    self.e = None
                    if st == _lib.ST_CORRUPT:
                        raise ReferencePanic("index block: next entry")
                    if st == _lib.ST_LOOP:
                        raise ReferenceLoop("index block: next entry")
                    return None
                self.e += 1
                nb = self._load(self.e)                   # Some(Err(e)) raises; valid stays false
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
        """ReaderIntoIter::seek (:302-335): Ok(true), or raises (Err / panic / loop).  The data
        block is seeked with the landed index entry's key (`key` is shadowed at :305)."""
        from .reader import ReferenceLoop, ReferencePanic
        key = bytes(key)
        r = self.r
        if self.ix is not None:                           # irregular index: the live iterator
            self._ix_seek(key)
            if not self.ix.valid():
                self.valid = False
                return True
            ikey, ival = self.ix.recs[self.ix.pos]
            new_off = _varint_decode64(ival)
            content = lambda: r._value_content(ival)      # noqa: E731
        else:
            s = index_seek(r, key)
            if s.status == _lib.SEEK_PANIC:
                raise ReferencePanic("index seek")
            if s.status == _lib.SEEK_LOOP:
                raise ReferenceLoop("index seek")
            if not s.valid:
                self.valid = False
                self.e = None
                return True
            self.e = r._ordinal(int(s.entry))
            ikey = r._index_keys()[self.e]
            new_off = int(s.block_off)
            content = lambda: r._seek_content(s)          # noqa: E731
        if self.block_offset != new_off:
            self.block_offset = new_off                   # updated before the load (:322)
            self.bi = self._seek_block(content(), ikey, 0)
        elif self.bi is not None:                         # the held block, whatever it is
            self.bi = self._seek_block(self.bi.content, ikey, self.bi.kcap())
        self.first = True
        self.valid = True
        return True
