"""Reader / ReaderBuilder mirror over the device codec (reference src/reader.rs).

A whole .mtbl file is scanned on the GPU:

    ReaderBuilder::read   src/reader.rs:31-81   footer + index framing (host, a few bytes)
    index block           decoded on the device like any block (mtblx_decode_blocks)
    block_at_index        src/reader.rs:177-186 \\ all entries at once: mtblx_block_dir
    Reader::block framing src/reader.rs:139-157 /
    crc32c verify         src/reader.rs:159-164  mtblx_crc32c_blocks (framed), if verifying
    Block::init + scan    src/block.rs           mtblx_decode_blocks over the directory
    ReaderIntoIter::next  src/reader.rs:337-405  how the iteration ENDS is decided on the host
                                                 from the per-block statuses (below); the
                                                 records stay on the device

`Reader.iter()` returns a `Scan`: the records the reference iterator yields, in order, as a
prefix of the device output arrays, plus how the iteration ends (`end`: NONE / ERR_OPEN /
ERR_NEXT / PANIC / LOOP, the oracle's codes).  Errors the reference returns from
ReaderBuilder::read raise `MtblError` here.

Seek-based iteration -- iter_from / iter_prefix / iter_range (src/reader.rs:128-138) and the
stateful ReaderIntoIter with next() / seek() (:219-405) -- goes through the device index seek,
block_at_index and block seek, decoding only the blocks the iteration reaches (iterator.py).
get() is the device Reader::get (mtblx_get).
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass

import numpy as np
import torch

from . import _lib, codec

END_NONE, END_ERR_OPEN, END_ERR_NEXT, END_PANIC, END_LOOP = range(5)
ERR_NAMES = ["None", "InvalidMetadataSize", "InvalidIndexBlockOffset", "InvalidIndexLength",
             "InvalidFormatVersion", "InvalidCompressionAlgorithm", "InvalidBlock", "Io"]
METADATA_SIZE = 512


class MtblError(RuntimeError):
    """Err(Error::Mtbl(..)) of the reference (src/error.rs:44-52)."""

    def __init__(self, code: int):
        super().__init__(ERR_NAMES[code] if 0 <= code < len(ERR_NAMES) else str(code))
        self.code = code


class ReferencePanic(RuntimeError):
    """Where the reference panics (assert / unwrap / slice out of range)."""


class ReferenceLoop(RuntimeError):
    """Where the reference never returns (an entry that does not advance)."""


@dataclass
class Scan:
    end: int                 # END_*
    err: str                 # error name for END_ERR_*
    nrec: int                # records yielded
    keys: torch.Tensor       # device, key bytes of the yielded records (concatenated)
    vals: torch.Tensor
    key_end: torch.Tensor    # device int64 [nrec], global END offsets into keys
    val_end: torch.Tensor

    def records(self):
        ke = self.key_end.cpu().numpy()
        ve = self.val_end.cpu().numpy()
        k = self.keys.cpu().numpy().tobytes()
        v = self.vals.cpu().numpy().tobytes()
        out, pk, pv = [], 0, 0
        for i in range(self.nrec):
            out.append((k[pk: ke[i]], v[pv: ve[i]]))
            pk, pv = int(ke[i]), int(ve[i])
        return out


class ReaderBuilder:
    """src/reader.rs:15-30: verify_checksums defaults to true."""

    def __init__(self):
        self._verify = True

    def verify_checksums(self, verify: bool) -> "ReaderBuilder":
        self._verify = bool(verify)
        return self

    def read(self, data, device="cuda") -> "Reader":
        return Reader(data, self._verify, device)


class Reader:
    def __init__(self, data, verify_checksums: bool = True, device="cuda"):
        codec._require_device()
        if isinstance(data, torch.Tensor):
            self.file = data.to(device=device, dtype=torch.uint8).contiguous()
            host = None
        else:
            host = np.frombuffer(bytes(data), np.uint8) if not isinstance(data, np.ndarray) else \
                np.ascontiguousarray(data, np.uint8)
            self.file = torch.from_numpy(host.copy()).to(device) if host.size else \
                torch.zeros(1, dtype=torch.uint8, device=device)
        self.len = int(host.size) if host is not None else int(self.file.numel())
        self.verify = verify_checksums
        L = _lib.lib()
        # ReaderBuilder::read (src/reader.rs:31-81): footer, index framing + checksum (host)
        if self.len < METADATA_SIZE:
            raise MtblError(1)
        tail = host[self.len - METADATA_SIZE:] if host is not None else \
            self.file[self.len - METADATA_SIZE:].cpu().numpy()
        f = _lib.Footer()
        # mtblx_read_footer wants the whole file for its offset check; a 512-byte view plus
        # the length is enough: pass a buffer whose last 512 bytes are the footer
        buf = np.zeros(self.len, np.uint8) if host is None else host
        if host is None:
            buf[self.len - METADATA_SIZE:] = tail
        rc = L.mtblx_read_footer(buf.ctypes.data_as(_lib.u8p), self.len, C.byref(f))
        if rc != 0:
            raise MtblError(int(f.err))
        self.meta = list(f.meta)
        self.version = int(f.version)
        self.compression = int(self.meta[2])   # 0..5 (read_footer rejects others: InvalidCompressionAlgorithm)
        idx_off = int(self.meta[0])
        if host is None:   # index block bytes to the host (framing + checksum)
            hi = self.len - METADATA_SIZE
            buf[idx_off:hi] = self.file[idx_off:hi].cpu().numpy()
        coff, clen, panic = C.c_uint64(0), C.c_uint64(0), C.c_int(0)
        rc = L.mtblx_frame_block(buf.ctypes.data_as(_lib.u8p), self.len, self.version, idx_off,
                                 1 if verify_checksums else 0, C.byref(coff), C.byref(clen), C.byref(panic))
        if panic.value:
            raise ReferencePanic("index block framing / checksum (src/reader.rs:52-74)")
        if rc != 0:
            raise MtblError(3)
        self.index_off, self.index_len = int(coff.value), int(clen.value)
        # index block on the device
        self._ibatch = codec.DeviceBatch(self.file, torch.tensor([coff.value], dtype=torch.int64, device=device),
                                         torch.tensor([clen.value], dtype=torch.int32, device=device),
                                         int(clen.value))
        self.index = codec.decode_blocks(self._ibatch)
        torch.cuda.synchronize()
        ist = int(self.index.status[0].item())
        if ist == _lib.ST_INVALID_BLOCK:
            raise MtblError(6)   # Block::init(index) -> InvalidBlock (src/reader.rs:76)
        self.index_status = ist
        self.nent = int(self.index.totals_host()[0])
        self._dir = None
        self._dir3 = None
        self._scan = None
        self._eoffs = None
        self._ikeys = None

    # ------------------------------------------------------------------ directory
    def directory(self):
        """(blk_off int64, blk_len int32, dir_status int32, crc_bad uint8|None) on the device,
        one entry per index record."""
        if self._dir is None:
            off, ln, st = self._framing()
            self._dir = (off, ln, st, self._bad_range(0, self.nent))
        return self._dir

    def _bad_range(self, i0: int, i1: int):
        """Reader::block's checksum assert for directory entries [i0, i1) (device uint8), or
        None when not verifying"""
        if not self.verify or i1 <= i0:
            return None
        off, ln, _ = self._framing()
        batch = codec.DeviceBatch(self.file, off[i0:i1], ln[i0:i1], int(ln[i0:i1].max().item()))
        return codec.crc32c_blocks(batch, framed=True)[1]

    def _framing(self):
        """block_at_index + Reader::block framing of every index entry: (off, len, status)"""
        if self._dir3 is None:
            n = max(self.nent, 1)
            dev = self.file.device
            off = torch.zeros(n, dtype=torch.int64, device=dev)
            ln = torch.zeros(n, dtype=torch.int32, device=dev)
            st = torch.zeros(n, dtype=torch.int32, device=dev)
            L = _lib.lib()
            if self.nent:
                rc = L.mtblx_block_dir(C.c_void_p(self.file.data_ptr()), self.len, self.version,
                                       C.c_void_p(self.index.vals.data_ptr()), C.c_void_p(self.index.val_end.data_ptr()),
                                       0, self.nent, C.c_void_p(off.data_ptr()), C.c_void_p(ln.data_ptr()),
                                       C.c_void_p(st.data_ptr()), C.c_void_p(codec._stream_handle(None)))
                if rc != 0:
                    raise RuntimeError(f"mtblx_block_dir failed: {rc}")
            self._dir3 = (off[: self.nent], ln[: self.nent], st[: self.nent])
        return self._dir3

    # ------------------------------------------------------------------ iteration
    def _decode_all(self):
        off, ln, st, bad = self.directory()
        self.zerr = None
        if self.compression != 0 and self.nent:
            # Reader::block decompresses after the checksum (src/reader.rs:166-170): on the
            # host, as the north star keeps src/compression.rs there; then one device decode
            buf, uoff, uln, self.zerr = self._host_stage(off, ln, st)
            ml = int(uln.max()) if uln.size else 0
            self._dbatch = codec.DeviceBatch.from_host(buf, uoff, uln, device=self.file.device)
        else:
            ml = int(ln.max().item()) if self.nent else 0
            self._dbatch = codec.DeviceBatch(self.file, off, ln, ml)
        self.data = codec.decode_blocks(self._dbatch) if self.nent else None
        torch.cuda.synchronize()
        return off, ln, st, bad

    def _host_stage(self, off, ln, st):
        """Reader::block's decompression step (src/reader.rs:166-170 -> src/compression.rs:57-68)
        on the host for every block the directory frames, any CompressionType:
        mtblx_decompress_blocks (16 threads; codecs_host.cpp).  A decoder error is the crate's
        Err(Error::Io); Lz4 / Lz4hc are its Err "unsupported" (also Error::Io)."""
        L = _lib.lib()
        host = self.file.cpu().numpy()
        o = off.cpu().numpy().view(np.uint64).copy()
        n = ln.cpu().numpy().view(np.uint32).copy()
        ok = st.cpu().numpy() == _lib.DIR_OK
        n[~ok] = 0
        o[~ok] = 0
        nb = o.size
        dst = _lib.u8p()
        doff = np.zeros(max(nb, 1), np.uint64)
        dlen = np.zeros(max(nb, 1), np.uint64)
        zst = np.zeros(max(nb, 1), np.int32)
        L.mtblx_decompress_blocks(self.compression, host.ctypes.data, o.ctypes.data, n.ctypes.data, nb, 16,
                                  C.byref(dst), doff.ctypes.data, dlen.ctypes.data, zst.ctypes.data)
        total = int(doff[nb - 1]) + ((int(dlen[nb - 1]) + 15) & ~15) if nb else 0
        buf = np.empty(max(total, 16), np.uint8)
        C.memmove(buf.ctypes.data, dst, total)
        L.mtblx_free(dst)
        zerr = zst[:nb].copy()
        zerr[~ok] = 0
        if (dlen[:nb] > 0xFFFFFFFF).any():
            raise NotImplementedError("decompressed block >= 4 GiB")
        return buf, doff[:nb].copy(), dlen[:nb].astype(np.uint32), zerr

    def iter(self) -> Scan:
        """ReaderIntoIter (mode Iter) to the end: the records yielded and how it ends."""
        if self._scan is not None:
            return self._scan
        off, ln, st, bad = self._decode_all()
        n = self.nent
        dst = st.cpu().numpy() if n else np.zeros(0, np.int32)
        cbad = bad.cpu().numpy() if (bad is not None and n) else np.zeros(n, np.uint8)
        if n:
            h = self.data.to_host()
            bst, bnr = h.status, h.nrec.astype(np.int64)
        else:
            bst = bnr = np.zeros(0, np.int64)
        end, err, take_blocks, take_last = END_NONE, "None", 0, 0
        # ReaderIntoIter::new: block_at_index(first entry) -- errors here are Err at open
        i = 0
        if n == 0:
            end = END_PANIC if self.index_status in (_lib.ST_CORRUPT,) else END_NONE
        while i < n:
            # Reader::block for entry i
            if dst[i] != _lib.DIR_OK or cbad[i]:
                end = END_PANIC if dst[i] != _lib.DIR_UNSUPPORTED else END_PANIC
                break
            if self.zerr is not None and self.zerr[i]:   # decompress -> Err(Error::Io) (src/reader.rs:166)
                end, err = (END_ERR_OPEN if i == 0 else END_ERR_NEXT), "Io"
                break
            s = int(bst[i])
            if s == _lib.ST_INVALID_BLOCK:
                end, err = (END_ERR_OPEN if i == 0 else END_ERR_NEXT), "InvalidBlock"
                break
            if s == _lib.ST_UNSUPPORTED:
                raise NotImplementedError("block >= 4 GiB")
            # an empty block ends the iteration, except the first one (src/reader.rs:362-371)
            if s == _lib.ST_OK and bnr[i] == 0 and i > 0:
                break
            if s in (_lib.ST_CORRUPT, _lib.ST_LOOP):   # records before the panic / loop, then stop
                take_blocks, take_last = i, int(bnr[i])
                end = END_PANIC if s == _lib.ST_CORRUPT else END_LOOP
                i = -1
                break
            i += 1
        if i == n and n:
            take_blocks = n
            if self.index_status == _lib.ST_CORRUPT:
                end = END_PANIC          # the index iterator panics advancing past its last entry
            elif self.index_status == _lib.ST_LOOP:
                end = END_LOOP
        elif i >= 0:
            take_blocks = i
        nblk_full = take_blocks
        self._scan = self._cut(nblk_full, take_last, end, err)
        return self._scan

    def _cut(self, nblk_full: int, take_last: int, end: int, err: str) -> Scan:
        return self._cut_data(self.data, nblk_full, take_last, end, err)

    def _cut_data(self, d, nblk_full: int, take_last: int, end: int, err: str) -> Scan:
        dev = self.file.device
        if d is None or (nblk_full == 0 and take_last == 0):
            z = torch.zeros(0, dtype=torch.uint8, device=dev)
            e = torch.zeros(0, dtype=torch.int64, device=dev)
            return Scan(end, err, 0, z, z, e, e)
        nr = d.nrec[: d.nblk].to(torch.int64)
        # records of the first nblk_full blocks + take_last records of the next block
        nrec = int(nr[:nblk_full].sum().item()) + take_last
        nb_used = nblk_full + (1 if take_last else 0)
        counts = nr[:nb_used].clone()
        if take_last:
            counts[-1] = take_last
        kb = d.key_base[:nb_used]
        vb = d.val_base[:nb_used]
        # blocks are laid out in order from record 0, so the yielded records are records 0..nrec
        blk_of = torch.repeat_interleave(torch.arange(nb_used, device=dev), counts)
        m32 = 0xFFFFFFFF
        key_end = kb[blk_of] + (d.key_end[:nrec].to(torch.int64) & m32)
        val_end = vb[blk_of] + (d.val_end[:nrec].to(torch.int64) & m32)
        klen = int(key_end[-1].item()) if nrec else 0
        vlen = int(val_end[-1].item()) if nrec else 0
        return Scan(end, err, nrec, d.keys[:klen], d.vals[:vlen], key_end, val_end)

    # ------------------------------------------------------------------ point queries
    def get_batch(self, keys, stream=None):
        """Reader::get for every key at once on the device (mtblx_get, f2).
        -> (status int32 [nq] (GET_*), val_off int64 [nq], val_len int64 [nq]) device tensors;
        the value of a FOUND query q is file[val_off[q] : val_off[q] + val_len[q]]."""
        if self.compression != 0:
            raise NotImplementedError("mtblx_get reads raw blocks; compressed files use get()")
        dev = self.file.device
        ks = [bytes(k) for k in keys]
        nq = len(ks)
        blob = b"".join(ks) or b"\0"
        kb = torch.frombuffer(bytearray(blob), dtype=torch.uint8).to(dev)
        ke = torch.tensor(np.cumsum([len(k) for k in ks], dtype=np.int64) if nq else [0], dtype=torch.int64,
                          device=dev)
        n = max(nq, 1)
        st = torch.zeros(n, dtype=torch.int32, device=dev)
        vo = torch.zeros(n, dtype=torch.int64, device=dev)
        vl = torch.zeros(n, dtype=torch.int64, device=dev)
        rc = _lib.lib().mtblx_get(C.c_void_p(self.file.data_ptr()), self.len, self.version, 1 if self.verify else 0,
                                  self.index_off, self.index_len, C.c_void_p(kb.data_ptr()),
                                  C.c_void_p(ke.data_ptr()), nq, C.c_void_p(st.data_ptr()), C.c_void_p(vo.data_ptr()),
                                  C.c_void_p(vl.data_ptr()), C.c_void_p(codec._stream_handle(stream)))
        if rc != 0:
            raise RuntimeError(f"mtblx_get failed: {rc}")
        return st[:nq], vo[:nq], vl[:nq]

    def get(self, key: bytes):
        """Reader::get (src/reader.rs:111-122): the value of `key`, or None; raises where the
        reference panics / returns Err."""
        if self.compression != 0:   # values live in decompressed blocks: the seek-based iterator
            from . import iterator
            it = iterator.ReaderIntoIter(self, "get", bytes(key))
            held = it.bi
            try:
                rec = it.next()
            except MtblError:
                # next() returned Some(Err): Reader::get matches Some(_) and returns the OLD
                # block iterator's `val` (src/reader.rs:111-122, :376-379), or None
                return held.last_val if held is not None else None
            if rec is None:
                return None
            # Some((k, v)) with k != key is still Some(_): ReaderIntoGet over bi's val
            return rec[1] if rec[0] == bytes(key) else it.bi.recs[it.bi.pos][1]
        st, vo, vl = self.get_batch([key])
        s = int(st[0].item())
        if s == _lib.GET_FOUND:
            o, n = int(vo[0].item()), int(vl[0].item())
            return self.file[o: o + n].cpu().numpy().tobytes()
        if s == _lib.GET_NONE:
            return None
        if s == _lib.GET_ERR:
            raise MtblError(6)
        raise ReferencePanic("Reader::get" + (" never returns" if s == _lib.GET_LOOP else ""))

    def _sorted_keys(self):
        s = self.iter()
        return s, s.records()

    def get_prefix(self, prefix: bytes):
        """iter_prefix's records on the host"""
        return self.iter_prefix(prefix).records()

    def get_range(self, start: bytes, end: bytes):
        """iter_range's records on the host"""
        return self.iter_range(start, end).records()

    # ------------------------------------------------------------------ seek-based iteration
    def iter_from(self, key: bytes) -> Scan:
        """Reader::iter_from (src/reader.rs:128-130) run to the end, touching only the blocks
        from the sought one on."""
        from . import iterator
        return iterator.bulk(self, "from", bytes(key))

    def iter_prefix(self, prefix: bytes) -> Scan:
        """Reader::iter_prefix (src/reader.rs:132-134)"""
        from . import iterator
        return iterator.bulk(self, "prefix", bytes(prefix))

    def iter_range(self, start: bytes, end: bytes) -> Scan:
        """Reader::iter_range (src/reader.rs:136-138): start <= key <= end"""
        from . import iterator
        return iterator.bulk(self, "range", bytes(start), bytes(end))

    def into_iter(self, kind: str = "iter", key: bytes = b"", key2: bytes = b""):
        """the stateful ReaderIntoIter (next() / seek()), see iterator.ReaderIntoIter"""
        from . import iterator
        return iterator.ReaderIntoIter(self, kind, key, key2)

    def _index_keys(self):
        if self._ikeys is None:
            self._ikeys = [k for k, _ in self.index.to_host().records(0)] if self.nent else []
        return self._ikeys

    def _ordinal(self, entry: int) -> int:
        """index position of the entry an index seek landed on (mtblx_entry_offsets)"""
        if self._eoffs is None:
            dev = self.file.device
            offs = torch.zeros(max(self.nent, 1), dtype=torch.int64, device=dev)
            cnt = torch.zeros(1, dtype=torch.int64, device=dev)
            rc = _lib.lib().mtblx_entry_offsets(C.c_void_p(self.file.data_ptr() + self.index_off), self.index_len,
                                                C.c_void_p(offs.data_ptr()), self.nent, C.c_void_p(cnt.data_ptr()),
                                                C.c_void_p(codec._stream_handle(None)))
            if rc != 0:
                raise RuntimeError(f"mtblx_entry_offsets failed: {rc}")
            n = min(int(cnt.item()), self.nent)
            self._eoffs = offs[:n].cpu().numpy()
        i = int(np.searchsorted(self._eoffs, entry))
        if i < self._eoffs.size and int(self._eoffs[i]) == entry:
            return i
        raise NotImplementedError("index seek landed off the index block's scan chain (corrupt index)")

    def _seek_content(self, s):
        """Reader::block of an index seek's landed entry -> (tensor, off, len) of the content
        BlockIter reads (host-decompressed for compressed files); raises Err / panic."""
        if s.block_status == _lib.SEEK_PANIC:
            raise ReferencePanic("Reader::block")
        if self.compression == 0:
            if s.block_status == _lib.SEEK_ERR:
                raise MtblError(6)
            if s.block_status == _lib.SEEK_UNSUPPORTED:
                raise NotImplementedError("block >= 4 GiB")
            return self.file, int(s.data_off), int(s.data_len)
        # compressed: Block::init runs on the decompressed content (mtblx_block_seek_batch);
        # block_status's ERR / UNSUPPORTED judged the compressed bytes and do not apply
        raw = self.file[int(s.data_off): int(s.data_off) + int(s.data_len)].cpu().numpy()
        L = _lib.lib()
        out = _lib.u8p()
        n = C.c_uint64(0)
        src = raw if raw.size else np.zeros(1, np.uint8)
        if L.mtblx_decompress(self.compression, src.ctypes.data, raw.size, C.byref(out), C.byref(n)) != 0:
            raise MtblError(7)
        b = C.string_at(out, n.value)
        L.mtblx_free(out)
        t = torch.frombuffer(bytearray(b or b"\0"), dtype=torch.uint8).to(self.file.device)
        return t, 0, len(b)

    def _decode_range(self, i0: int, i1: int):
        """decode directory entries [i0, i1) -> (dir status, crc bad, decompress errors, decoded,
        (base tensor, content offsets, content lengths)) with host arrays"""
        off, ln, st = self._framing()
        n = i1 - i0
        dst = st[i0:i1].cpu().numpy()
        bad = self._bad_range(i0, i1)
        bad = bad.cpu().numpy() if bad is not None else np.zeros(n, np.uint8)
        if self.compression != 0:
            buf, uoff, uln, zerr = self._host_stage(off[i0:i1], ln[i0:i1], st[i0:i1])
            batch = codec.DeviceBatch.from_host(buf, uoff, uln, device=self.file.device)
            where = (batch.data, uoff.astype(np.int64), uln.astype(np.int64))
        else:
            zerr = np.zeros(n, np.int32)
            batch = codec.DeviceBatch(self.file, off[i0:i1], ln[i0:i1], int(ln[i0:i1].max().item()))
            where = (self.file, off[i0:i1].cpu().numpy(), ln[i0:i1].cpu().numpy().view(np.uint32).astype(np.int64))
        data = codec.decode_blocks(batch)
        return dst, bad, zerr, data, where

    def _walk_range(self, i0: int, i1: int):
        """ReaderIntoIter::next over directory entries [i0, i1), each block loaded by next()
        (an empty block ends the iteration, src/reader.rs:362-371) -> ((keys, vals, key_end,
        val_end, nrec) on the device, end, err, stopped)"""
        dst, bad, zerr, data, _ = self._decode_range(i0, i1)
        n = i1 - i0
        bst = data.status[:n].cpu().numpy()
        bnr = data.nrec[:n].cpu().numpy().astype(np.int64)
        end, err, full, last, stopped = END_NONE, "None", n, 0, False
        for i in range(n):
            if dst[i] != _lib.DIR_OK or bad[i]:
                end, full, stopped = END_PANIC, i, True
                break
            if zerr[i]:
                end, err, full, stopped = END_ERR_NEXT, "Io", i, True
                break
            s = int(bst[i])
            if s == _lib.ST_INVALID_BLOCK:
                end, err, full, stopped = END_ERR_NEXT, "InvalidBlock", i, True
                break
            if s == _lib.ST_UNSUPPORTED:
                raise NotImplementedError("block >= 4 GiB")
            if s == _lib.ST_OK and bnr[i] == 0:
                full, stopped = i, True
                break
            if s in (_lib.ST_CORRUPT, _lib.ST_LOOP):
                end = END_PANIC if s == _lib.ST_CORRUPT else END_LOOP
                full, last, stopped = i, int(bnr[i]), True
                break
        sc = self._cut_data(data, full, last, end, err)
        return (sc.keys, sc.vals, sc.key_end, sc.val_end, sc.nrec), end, err, stopped

    def _host_blocks(self, i0: int, i1: int):
        """blocks [i0, i1) as next() loads them, for the stateful iterator: per block an
        exception to raise (Err / panic) or ((tensor, off, len), records, emit end)"""
        dst, bad, zerr, data, (base, boff, blen) = self._decode_range(i0, i1)
        h = data.to_host()
        out = []
        for i in range(i1 - i0):
            content = (base, int(boff[i]), int(blen[i]))
            if dst[i] != _lib.DIR_OK or bad[i]:
                out.append(ReferencePanic("Reader::block"))
                continue
            if zerr[i]:
                out.append(MtblError(7))
                continue
            s = int(h.status[i])
            if s == _lib.ST_INVALID_BLOCK:
                out.append(MtblError(6))
            elif s == _lib.ST_UNSUPPORTED:
                out.append(NotImplementedError("block >= 4 GiB"))
            else:
                end = {_lib.ST_CORRUPT: _lib.EMIT_PANIC, _lib.ST_LOOP: _lib.EMIT_LOOP}.get(s, _lib.EMIT_END)
                out.append((content, h.records(i), end))
        return out
