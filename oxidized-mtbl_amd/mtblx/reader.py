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
        self._regular = None
        self._ikeys = None
        self._irecs = None

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
        # u64 lengths: a content >= 4 GiB is not decoded by the batched call (u32 lengths) but by
        # the emitting block seek on its bytes in the uploaded buffer (_big_content)
        return buf, doff[:nb].copy(), dlen[:nb].copy(), zerr

    def iter(self) -> Scan:
        """ReaderIntoIter (mode Iter) to the end: the records yielded and how it ends."""
        if self._scan is not None:
            return self._scan
        from . import iterator
        n = self.nent
        end, err = END_NONE, "None"
        if n == 0:   # ReaderIntoIter::new with no index entry; a corrupt index panics at its first
            end = END_PANIC if self.index_status == _lib.ST_CORRUPT else END_NONE
            self._scan = iterator._assemble([], end, err, self.file.device)
            return self._scan
        parts, end, err, stopped = self._walk_blocks(0, n, first_exempt=True)
        if not stopped:
            if self.index_status == _lib.ST_CORRUPT:
                end = END_PANIC          # the index iterator panics advancing past its last entry
            elif self.index_status == _lib.ST_LOOP:
                end = END_LOOP
        self._scan = iterator._assemble(parts, end, err, self.file.device)
        return self._scan

    def _walk_blocks(self, i0: int, i1: int, first_exempt: bool):
        """ReaderIntoIter::next over directory entries [i0, i1) (src/reader.rs:337-405):
        Reader::block's framing / checksum / decompression, Block::init, the scan; an empty
        block loaded by next() ends the iteration (first_exempt: block i0 came from
        ReaderIntoIter::new, whose Err is an Err at open and whose emptiness does not end it).
        Blocks >= 4 GiB are decoded one by one (_big_block) and spliced in.
        -> (parts [(keys, vals, key_end, val_end, nrec)], end, err, stopped)"""
        dst, bad, zerr, data, (base, boff, blen) = self._decode_range(i0, i1)
        n = i1 - i0
        bst = data.status[:n].cpu().numpy()
        bnr = data.nrec[:n].cpu().numpy().astype(np.int64)
        parts, seg, take_last = [], 0, 0
        end, err, stopped = END_NONE, "None", False

        def errend(i):
            return END_ERR_OPEN if (first_exempt and i == 0) else END_ERR_NEXT

        i = 0
        while i < n:
            # content >= 4 GiB (u64 restart array): stored that big (DIR_UNSUPPORTED: framed,
            # checked and decompressed by _big_block), or decompressed that big (_big_content)
            big_dec = dst[i] == _lib.DIR_OK and not bad[i] and not zerr[i] and int(blen[i]) > 0xFFFFFFFF
            if dst[i] == _lib.DIR_UNSUPPORTED or big_dec:
                parts.append(self._slice(data, seg, i, 0))
                seg = i + 1
                kind, em = (self._big_content((base, int(boff[i]), int(blen[i]))) if big_dec
                            else self._big_block(i0 + i))
                if kind == "panic":
                    end, stopped = END_PANIC, True
                    break
                if kind == "loop":
                    end, stopped = END_LOOP, True
                    break
                if kind != "ok":
                    end, err, stopped = errend(i), kind, True
                    break
                if em.nrec == 0 and em.end == _lib.EMIT_END and not (first_exempt and i == 0):
                    stopped = True
                    break
                parts.append((em.keys, em.vals, em.key_end, em.val_end, em.nrec))
                if em.end in (_lib.EMIT_PANIC, _lib.EMIT_LOOP):
                    end, stopped = (END_PANIC if em.end == _lib.EMIT_PANIC else END_LOOP), True
                    break
                i += 1
                continue
            if dst[i] != _lib.DIR_OK or bad[i]:        # Reader::block panics (framing / checksum)
                end, stopped = END_PANIC, True
                break
            if zerr[i]:                                # decompress -> Err(Error::Io) (src/reader.rs:166)
                end, err, stopped = errend(i), "Io", True
                break
            st = int(bst[i])
            if st == _lib.ST_INVALID_BLOCK:
                end, err, stopped = errend(i), "InvalidBlock", True
                break
            if st == _lib.ST_UNSUPPORTED:     # the batch carries u32 lengths: cannot happen
                raise RuntimeError("batched decode: block >= 4 GiB")
            if st == _lib.ST_OK and bnr[i] == 0 and not (first_exempt and i == 0):
                stopped = True                         # an empty block ends the iteration (:362-371)
                break
            if st in (_lib.ST_CORRUPT, _lib.ST_LOOP):  # the records before the panic / loop, then stop
                take_last = int(bnr[i])
                end, stopped = (END_PANIC if st == _lib.ST_CORRUPT else END_LOOP), True
                break
            i += 1
        parts.append(self._slice(data, seg, i, take_last))
        return parts, end, err, stopped

    def _slice(self, d, i0: int, i1: int, take_last: int):
        """records of decoded blocks [i0, i1) plus the first take_last records of block i1
        -> (keys, vals, key_end, val_end, nrec) on the device, END offsets from the slice start"""
        dev = self.file.device
        nb_used = i1 - i0 + (1 if take_last else 0)
        z = torch.zeros(0, dtype=torch.uint8, device=dev)
        e = torch.zeros(0, dtype=torch.int64, device=dev)
        if d is None or nb_used <= 0:
            return z, z, e, e, 0
        counts = d.nrec[i0: i0 + nb_used].to(torch.int64).clone()
        if take_last:
            counts[-1] = take_last
        nrec = int(counts.sum().item())
        if nrec == 0:
            return z, z, e, e, 0
        r0 = int(d.rec_base[i0].item())
        kb = d.key_base[i0: i0 + nb_used]
        vb = d.val_base[i0: i0 + nb_used]
        k0, v0 = int(kb[0].item()), int(vb[0].item())
        blk_of = torch.repeat_interleave(torch.arange(nb_used, device=dev), counts)
        m32 = 0xFFFFFFFF
        key_end = kb[blk_of] - k0 + (d.key_end[r0: r0 + nrec].to(torch.int64) & m32)
        val_end = vb[blk_of] - v0 + (d.val_end[r0: r0 + nrec].to(torch.int64) & m32)
        klen = int(key_end[-1].item())
        vlen = int(val_end[-1].item())
        return d.keys[k0: k0 + klen], d.vals[v0: v0 + vlen], key_end, val_end, nrec

    def _big_frame(self, i: int):
        """Reader::block framing of directory entry i from its index value (host, a few bytes)
        -> (block offset, content start, content length, stored crc)"""
        return self._big_frame_value(self._index_records()[i][1])

    def _big_frame_value(self, v: bytes):
        L = _lib.lib()
        off = C.c_uint64(0)
        vb = np.frombuffer(v or b"\0", np.uint8)
        L.mtblx_varint_decode64(vb.ctypes.data_as(_lib.u8p), len(v), C.byref(off))
        off = int(off.value)
        head = self.file[off: off + 14].cpu().numpy()
        if self.version == 0:
            ll, size = 4, int.from_bytes(head[:4].tobytes(), "little")
        else:
            sz = C.c_uint64(0)
            ll = int(L.mtblx_varint_decode64(head.ctypes.data_as(_lib.u8p), head.size, C.byref(sz)))
            size = int(sz.value)
        stored = int.from_bytes(head[ll: ll + 4].tobytes(), "little")
        return off, off + ll + 4, size, stored

    def _crc_big(self, start: int, size: int) -> int:
        """CRC-32C of file[start, start + size) for size >= 4 GiB: the device CRC of <= 1 GiB
        pieces, joined on the host with crc(A || B) = x^(8|B|) * crc(A) ^ crc(B) (mod P)"""
        piece = 1 << 30
        offs = list(range(start, start + size, piece))
        lens = [min(piece, start + size - o) for o in offs]
        dev = self.file.device
        batch = codec.DeviceBatch(self.file, torch.tensor(offs, dtype=torch.int64, device=dev),
                                  torch.tensor(lens, dtype=torch.int32, device=dev), max(lens))
        crcs = codec.crc32c_blocks(batch)[0].cpu().numpy().view(np.uint32)
        c = int(crcs[0])
        for k in range(1, len(lens)):
            c = _gf2_mul(_x8n(lens[k]), c) ^ int(crcs[k])
        return c

    def _big_block(self, i: int):
        """Reader::block + Block::init + the scan for a block >= 4 GiB (u64 restart array,
        src/block.rs:25-42): decoded on the device by the emitting block seek (seek_to_first).
        -> ("ok", Emitted) | ("panic", None) | ("loop", None) | (error name, None)"""
        return self._big_block_value(self._index_records()[i][1])[:2]

    def _big_block_value(self, value: bytes):
        off, start, size, stored = self._big_frame_value(value)
        if start > self.len or size > self.len - start:
            return "panic", None, None
        if self.verify and self._crc_big(start, size) != stored:
            return "panic", None, None                 # assert_eq of the checksum (src/reader.rs:163)
        if self.compression == 0:
            content = (self.file, start, size)
        else:
            try:                                       # src/reader.rs:166-170 (host, any size)
                content = self._decompressed(start, size)
            except MtblError:
                return "Io", None, None
        return self._big_content(content) + (content,)

    def _big_content(self, content):
        """Block::init + the scan of a content >= 4 GiB (tensor, off, len) on the device"""
        from . import iterator
        em = iterator.block_seek(content, None, 0, small_caps=True)
        if em.status == _lib.SEEK_ERR:
            return "InvalidBlock", None
        if em.status == _lib.SEEK_PANIC:
            return "panic", None
        if em.status == _lib.SEEK_LOOP:
            return "loop", None
        if em.status == _lib.SEEK_UNSUPPORTED:
            raise RuntimeError("emitting seek: key buffer too small")
        return "ok", em

    # ------------------------------------------------------------------ point queries
    def _dec_table(self):
        """Every data block the directory frames, decompressed on the host (Reader::block's
        decompress step, src/reader.rs:166-170), on the device, with the table
        mtblx_get_decompressed takes: sorted by stored content start."""
        if getattr(self, "_dtab", None) is None:
            off, ln, st = self._framing()
            buf, doff, dlen, zerr = self._host_stage(off, ln, st)
            start = off.cpu().numpy().view(np.uint64)
            ok = st.cpu().numpy() == _lib.DIR_OK
            start, doff, dlen = start[ok], doff[ok], dlen[ok]
            zst = zerr[ok].astype(np.int32)
            order = np.argsort(start, kind="stable")
            dev = self.file.device
            t = lambda a, dt: torch.from_numpy(np.ascontiguousarray(a).view(dt)).to(dev)
            self._dtab = (t(start[order], np.int64), t(doff[order], np.int64), t(dlen[order], np.int64),
                          t(zst[order], np.int32), int(order.size), torch.from_numpy(buf).to(dev))
        return self._dtab

    def _dtab_add(self, starts, sizes):
        """decompress stored blocks [start, + size) the table lacks (a get_batch seek landed on
        them: MTBLX_GET_MISSING) and add them to the table"""
        ts, tdo, tdl, tst, n, dec = self._dec_table()
        L = _lib.lib()
        parts, base = [], int(dec.numel())
        s0, o0, l0, z0 = [], [], [], []
        for a, n_ in zip(starts, sizes):
            raw = self.file[int(a): int(a) + int(n_)].cpu().numpy()
            out = _lib.u8p()
            un = C.c_uint64(0)
            src = raw if raw.size else np.zeros(1, np.uint8)
            ok = L.mtblx_decompress(self.compression, src.ctypes.data, raw.size, C.byref(out), C.byref(un)) == 0
            b = np.empty(int(un.value) if ok else 0, np.uint8)
            if ok:
                C.memmove(b.ctypes.data, out, int(un.value))
                L.mtblx_free(out)
            s0.append(int(a)); o0.append(base); l0.append(b.size); z0.append(0 if ok else 1)
            parts.append(b)
            base += b.size
        dev = self.file.device
        start = np.concatenate([ts.cpu().numpy(), np.array(s0, np.int64)])
        doff = np.concatenate([tdo.cpu().numpy(), np.array(o0, np.int64)])
        dlen = np.concatenate([tdl.cpu().numpy(), np.array(l0, np.int64)])
        zst = np.concatenate([tst.cpu().numpy(), np.array(z0, np.int32)])
        order = np.argsort(start, kind="stable")
        t = lambda a_: torch.from_numpy(np.ascontiguousarray(a_)).to(dev)
        extra = torch.from_numpy(np.concatenate(parts) if parts else np.zeros(0, np.uint8)).to(dev)
        self._dtab = (t(start[order]), t(doff[order]), t(dlen[order]), t(zst[order]), int(order.size),
                      torch.cat([dec, extra]))

    @property
    def value_source(self):
        """the device bytes get_batch's val_off / val_len point into: the file, or for a
        compressed file its decompressed blocks"""
        return self.file if self.compression == 0 else self._dec_table()[5]

    def get_batch(self, keys, stream=None):
        """Reader::get for every key at once on the device (mtblx_get / mtblx_get_decompressed,
        f2).  -> (status int32 [nq] (GET_*), val_off int64 [nq], val_len int64 [nq]) device
        tensors; the value of a FOUND query q is value_source[val_off[q] : val_off[q] +
        val_len[q]] (the file itself unless it is compressed)."""
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
        if self.compression == 0:
            rc = _lib.lib().mtblx_get(C.c_void_p(self.file.data_ptr()), self.len, self.version, 1 if self.verify else 0,
                                      self.index_off, self.index_len, C.c_void_p(kb.data_ptr()),
                                      C.c_void_p(ke.data_ptr()), nq, C.c_void_p(st.data_ptr()),
                                      C.c_void_p(vo.data_ptr()), C.c_void_p(vl.data_ptr()),
                                      C.c_void_p(codec._stream_handle(stream)))
        else:
            # a lookup that reaches a stored block the table lacks (MTBLX_GET_MISSING: only a
            # corrupt index read with verification off leads there) gets that block decompressed
            # and added, and the batch runs again; every round adds a block, so this ends
            for _ in range(1 + 4096):
                ts, tdo, tdl, tst, ntab, dec = self._dec_table()
                rc = _lib.lib().mtblx_get_decompressed(
                    C.c_void_p(self.file.data_ptr()), self.len, self.version, 1 if self.verify else 0,
                    self.index_off, self.index_len, C.c_void_p(ts.data_ptr()), C.c_void_p(tdo.data_ptr()),
                    C.c_void_p(tdl.data_ptr()), C.c_void_p(tst.data_ptr()), ntab, C.c_void_p(dec.data_ptr()),
                    C.c_void_p(kb.data_ptr()), C.c_void_p(ke.data_ptr()), nq, C.c_void_p(st.data_ptr()),
                    C.c_void_p(vo.data_ptr()), C.c_void_p(vl.data_ptr()), C.c_void_p(codec._stream_handle(stream)))
                if rc != 0 or nq == 0:
                    break
                miss = (st[:nq] == _lib.GET_MISSING).cpu().numpy()
                if not miss.any():
                    break
                pairs = sorted(set(zip(vo[:nq].cpu().numpy()[miss].tolist(), vl[:nq].cpu().numpy()[miss].tolist())))
                self._dtab_add([a for a, _ in pairs], [b for _, b in pairs])
            else:
                raise RuntimeError("get_batch: missing blocks did not converge")
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

    def _index_records(self):
        """the index block's records (separator key, value) on the host, cached"""
        if self._irecs is None:
            self._irecs = self.index.to_host().records(0) if self.nent else []
        return self._irecs

    def _index_keys(self):
        if self._ikeys is None:
            self._ikeys = [k for k, _ in self._index_records()]
        return self._ikeys

    def _index_chain(self):
        """(entry offsets of the index scan chain, regular) from mtblx_entry_offsets: regular =
        a seek from any index iterator state lands on the chain and continues along the
        directory (include/mtblx.h); otherwise the iterators drive the live index iterator on
        the device (iterator._IxList)"""
        if self._eoffs is None:
            dev = self.file.device
            cap = max(self.index_len // 3 + 1, 1)          # an entry takes >= 3 bytes
            offs = torch.zeros(cap, dtype=torch.int64, device=dev)
            cnt = torch.zeros(1, dtype=torch.int64, device=dev)
            reg = torch.zeros(1, dtype=torch.int32, device=dev)
            rc = _lib.lib().mtblx_entry_offsets(C.c_void_p(self.file.data_ptr() + self.index_off), self.index_len,
                                                C.c_void_p(offs.data_ptr()), cap, C.c_void_p(cnt.data_ptr()),
                                                C.c_void_p(reg.data_ptr()), C.c_void_p(codec._stream_handle(None)))
            if rc != 0:
                raise RuntimeError(f"mtblx_entry_offsets failed: {rc}")
            n = min(int(cnt.item()), cap)
            self._eoffs = offs[:n].cpu().numpy()
            self._regular = bool(reg.item()) and self.index_status == _lib.ST_OK
        return self._eoffs, self._regular

    def index_regular(self) -> bool:
        return self._index_chain()[1]

    def _chain_ordinal(self, entry: int):
        """position on the index scan chain of the entry at `entry` (the index seek's landing),
        or None when it lies off the chain (a corrupt index)"""
        eoffs = self._index_chain()[0]
        i = int(np.searchsorted(eoffs, entry))
        if i < eoffs.size and int(eoffs[i]) == entry:
            return i
        return None

    def _ordinal(self, entry: int) -> int:
        """directory entry of a regular index's seek landing (always on the chain)"""
        i = self._chain_ordinal(entry)
        if i is None or i >= self.nent:
            raise RuntimeError("index seek landed off the directory of a regular index")
        return i

    def index_content(self):
        """the index block content on the device as (tensor, off, len)"""
        return self.file, self.index_off, self.index_len

    def _frame_values(self, values):
        """block_at_index + Reader::block framing (src/reader.rs:177-186, :139-157) of arbitrary
        index values (the live index iterator's records) on the device: (off, len, status)"""
        dev = self.file.device
        n = len(values)
        blob = b"".join(values) or b"\0"
        vals = torch.frombuffer(bytearray(blob), dtype=torch.uint8).to(dev)
        vend = torch.tensor(np.cumsum([len(v) for v in values], dtype=np.int64).astype(np.uint32).view(np.int32),
                            dtype=torch.int32, device=dev)
        off = torch.zeros(n, dtype=torch.int64, device=dev)
        ln = torch.zeros(n, dtype=torch.int32, device=dev)
        st = torch.zeros(n, dtype=torch.int32, device=dev)
        rc = _lib.lib().mtblx_block_dir(C.c_void_p(self.file.data_ptr()), self.len, self.version,
                                        C.c_void_p(vals.data_ptr()), C.c_void_p(vend.data_ptr()), 0, n,
                                        C.c_void_p(off.data_ptr()), C.c_void_p(ln.data_ptr()),
                                        C.c_void_p(st.data_ptr()), C.c_void_p(codec._stream_handle(None)))
        if rc != 0:
            raise RuntimeError(f"mtblx_block_dir failed: {rc}")
        return off, ln, st

    def _value_blocks(self, values):
        """the blocks of index values as next() loads them (see _host_blocks)"""
        off, ln, st = self._frame_values(values)
        return self._host_blocks_framed(off, ln, st, values)

    def _value_content(self, value: bytes):
        """Reader::block (src/reader.rs:139-175) at the offset an index value names -> the
        content (tensor, off, len) BlockIter reads; raises the reference's panics / Err"""
        off, ln, st = self._frame_values([value])
        s = int(st[0].item())
        if s == _lib.DIR_UNSUPPORTED:                   # stored content >= 4 GiB
            _, start, size, stored = self._big_frame_value(value)
            if self.verify and self._crc_big(start, size) != stored:
                raise ReferencePanic("Reader::block: checksum")
            if self.compression != 0:
                return self._decompressed(start, size)
            return self.file, start, size
        if s != _lib.DIR_OK:
            raise ReferencePanic("Reader::block: framing")
        if self.verify:
            batch = codec.DeviceBatch(self.file, off, ln, int(ln[0].item()))
            if int(codec.crc32c_blocks(batch, framed=True)[1][0].item()):
                raise ReferencePanic("Reader::block: checksum")
        o, n = int(off[0].item()), int(ln[0].item()) & 0xFFFFFFFF
        if self.compression == 0:
            return self.file, o, n
        return self._decompressed(o, n)

    def _seek_content(self, s):
        """Reader::block of an index seek's landed entry -> (tensor, off, len) of the content
        BlockIter reads (host-decompressed for compressed files); raises Err / panic."""
        if s.block_status == _lib.SEEK_PANIC:
            raise ReferencePanic("Reader::block")
        if self.compression == 0:
            if s.block_status == _lib.SEEK_ERR:
                raise MtblError(6)
            if s.block_status == _lib.SEEK_UNSUPPORTED:   # frame_block handles any size
                raise RuntimeError("index seek: unexpected block status")
            return self.file, int(s.data_off), int(s.data_len)
        # compressed: Block::init runs on the decompressed content (mtblx_block_seek_batch);
        # block_status's ERR / UNSUPPORTED judged the compressed bytes and do not apply
        return self._decompressed(int(s.data_off), int(s.data_len))

    def _decompressed(self, off: int, n: int):
        """src/compression.rs:57-68 on the host for one stored block -> content on the device"""
        raw = self.file[off: off + n].cpu().numpy()
        L = _lib.lib()
        out = _lib.u8p()
        un = C.c_uint64(0)
        src = raw if raw.size else np.zeros(1, np.uint8)
        if L.mtblx_decompress(self.compression, src.ctypes.data, raw.size, C.byref(out), C.byref(un)) != 0:
            raise MtblError(7)
        buf = np.empty(max(int(un.value), 1), np.uint8)   # no bytes object: blocks of GiBs
        C.memmove(buf.ctypes.data, out, int(un.value))
        L.mtblx_free(out)
        t = torch.from_numpy(buf).to(self.file.device)
        return t, 0, int(un.value)

    def _decode_range(self, i0: int, i1: int):
        """decode directory entries [i0, i1) -> (dir status, crc bad, decompress errors, decoded,
        (base tensor, content offsets, content lengths)) with host arrays"""
        off, ln, st = self._framing()
        bad = self._bad_range(i0, i1)
        return self._decode_framed(off[i0:i1], ln[i0:i1], st[i0:i1], bad)

    def _decode_framed(self, off, ln, st, bad="verify"):
        """decode framed blocks (off, len, dir status: device tensors); bad: the checksum
        assert per block (device uint8), None when not verifying, "verify" to compute it"""
        n = int(off.numel())
        dst = st.cpu().numpy()
        if isinstance(bad, str):
            bad = None
            if self.verify and n:
                okl = torch.where(st == _lib.DIR_OK, ln, torch.zeros_like(ln))
                batch = codec.DeviceBatch(self.file, off, okl, int(okl.max().item()))
                bad = codec.crc32c_blocks(batch, framed=True)[1]
        bad = bad.cpu().numpy() if bad is not None else np.zeros(n, np.uint8)
        if self.compression != 0:
            buf, uoff, uln, zerr = self._host_stage(off, ln, st)
            small = np.where(uln > 0xFFFFFFFF, 0, uln).astype(np.uint32)   # >= 4 GiB: _big_content
            batch = codec.DeviceBatch.from_host(buf, uoff, small, device=self.file.device)
            where = (batch.data, uoff.astype(np.int64), uln.astype(np.int64))
        else:
            zerr = np.zeros(n, np.int32)
            batch = codec.DeviceBatch(self.file, off, ln, int(ln.max().item()))
            where = (self.file, off.cpu().numpy(), ln.cpu().numpy().view(np.uint32).astype(np.int64))
        data = codec.decode_blocks(batch)
        return dst, bad, zerr, data, where

    def _walk_range(self, i0: int, i1: int):
        """ReaderIntoIter::next over directory entries [i0, i1), each block loaded by next()
        -> ((keys, vals, key_end, val_end, nrec) on the device, end, err, stopped)"""
        from . import iterator
        parts, end, err, stopped = self._walk_blocks(i0, i1, first_exempt=False)
        sc = iterator._assemble(parts, end, err, self.file.device)
        return (sc.keys, sc.vals, sc.key_end, sc.val_end, sc.nrec), end, err, stopped

    def _host_blocks(self, i0: int, i1: int):
        """blocks [i0, i1) as next() loads them, for the stateful iterator: per block an
        exception to raise (Err / panic) or ((tensor, off, len), records, emit end)"""
        off, ln, st = self._framing()
        recs = self._index_records()
        return self._host_blocks_framed(off[i0:i1], ln[i0:i1], st[i0:i1], [recs[i][1] for i in range(i0, i1)],
                                        self._bad_range(i0, i1))

    def _host_blocks_framed(self, off, ln, st, values, bad="verify"):
        dst, bad, zerr, data, (base, boff, blen) = self._decode_framed(off, ln, st, bad)
        h = data.to_host()
        out = []
        for i in range(len(values)):
            content = (base, int(boff[i]), int(blen[i]))
            big_dec = dst[i] == _lib.DIR_OK and not bad[i] and not zerr[i] and int(blen[i]) > 0xFFFFFFFF
            if dst[i] == _lib.DIR_UNSUPPORTED or big_dec:   # content >= 4 GiB
                if big_dec:
                    kind, em = self._big_content(content)
                else:
                    kind, em, content = self._big_block_value(values[i])
                if kind == "ok":
                    out.append((content, em.host_records(), em.end))
                elif kind in ("panic", "loop"):
                    out.append(ReferencePanic("Reader::block / BlockIter") if kind == "panic"
                               else ReferenceLoop("BlockIter::next"))
                else:
                    out.append(MtblError(7 if kind == "Io" else 6))
                continue
            if dst[i] != _lib.DIR_OK or bad[i]:
                out.append(ReferencePanic("Reader::block"))
                continue
            if zerr[i]:
                out.append(MtblError(7))
                continue
            s = int(h.status[i])
            if s == _lib.ST_INVALID_BLOCK:
                out.append(MtblError(6))
            elif s == _lib.ST_UNSUPPORTED:   # the batch carries u32 lengths: cannot happen
                out.append(RuntimeError("batched decode: block >= 4 GiB"))
            else:
                end = {_lib.ST_CORRUPT: _lib.EMIT_PANIC, _lib.ST_LOOP: _lib.EMIT_LOOP}.get(s, _lib.EMIT_END)
                out.append((content, h.records(i), end))
        return out


# GF(2) arithmetic of CRC-32C (reflected, x^0 = bit 31) for joining piece checksums
_POLY = 0x82F63B78


def _gf2_mul(a: int, b: int) -> int:
    p = 0
    for i in range(32):
        if a & (0x80000000 >> i):
            p ^= b
        b = (b >> 1) ^ _POLY if b & 1 else b >> 1
    return p


def _x8n(n: int) -> int:
    """x^(8 n) mod P"""
    r, sq, e = 0x80000000, 0x80000000 >> 8, n   # sq = x^8
    while e:
        if e & 1:
            r = _gf2_mul(sq, r)
        sq = _gf2_mul(sq, sq)
        e >>= 1
    return r
