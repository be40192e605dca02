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

get / get_prefix / get_range / iter_from are answered from the decoded records with a binary
search over the (sorted) keys -- identical to the reference's index + block seek on well-formed
files; malformed files are only defined for iter() in this round (documented in DESIGN.md).
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
        self._scan = None

    # ------------------------------------------------------------------ directory
    def directory(self):
        """(blk_off int64, blk_len int32, dir_status int32, crc_bad uint8|None) on the device,
        one entry per index record."""
        if self._dir is None:
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
            off, ln, st = off[: self.nent], ln[: self.nent], st[: self.nent]
            bad = None
            if self.verify and self.nent:
                ml = int(ln.max().item())
                batch = codec.DeviceBatch(self.file, off, ln, ml)
                _, bad = codec.crc32c_blocks(batch, framed=True)
            self._dir = (off, ln, st, bad)
        return self._dir

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
        dev = self.file.device
        if self.data is None or (nblk_full == 0 and take_last == 0):
            z = torch.zeros(0, dtype=torch.uint8, device=dev)
            e = torch.zeros(0, dtype=torch.int64, device=dev)
            return Scan(end, err, 0, z, z, e, e)
        d = self.data
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
        if self.compression != 0:   # values live in decompressed blocks: search the decoded records
            recs = self._sorted_keys()[1]
            import bisect
            i = bisect.bisect_left([k for k, _ in recs], bytes(key))
            return recs[i][1] if i < len(recs) and recs[i][0] == bytes(key) else None
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
        s, recs = self._sorted_keys()
        import bisect
        p = bytes(prefix)
        i = bisect.bisect_left([k for k, _ in recs], p)
        out = []
        while i < len(recs) and recs[i][0].startswith(p):
            out.append(recs[i])
            i += 1
        return out

    def get_range(self, start: bytes, end: bytes):
        s, recs = self._sorted_keys()
        import bisect
        i = bisect.bisect_left([k for k, _ in recs], bytes(start))
        out = []
        while i < len(recs) and recs[i][0] <= bytes(end):
            out.append(recs[i])
            i += 1
        return out

    def iter_from(self, key: bytes):
        s, recs = self._sorted_keys()
        import bisect
        return recs[bisect.bisect_left([k for k, _ in recs], bytes(key)):]
