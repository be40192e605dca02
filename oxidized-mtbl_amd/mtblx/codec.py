"""Device block codec: Python front-end of mtblx_decode_blocks (include/mtblx.h).

PyTorch is plumbing only (device memory, streams); the decode runs in libmtblx.so's
HIP kernels.  Replaces the reference's per-block ``Block::init`` + ``BlockIter`` scan
(/root/reference/src/block.rs:16-238) with one batched device call.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass

import numpy as np
import torch

from . import _lib
from ._lib import BlockBatch, Decoded


_checked_devices = set()

FLAG_OVERFLOW = 1      # totals[3] bit 0: some block's outputs did not fit (status MTBLX_ST_OVERFLOW)
FLAG_TIMEOUT = 2       # totals[3] bit 1: the launch's look-back timed out -- nothing it wrote is valid


class LaunchTimeout(RuntimeError):
    """A decode / encode launch reported a look-back timeout (include/mtblx.h, totals[3] bit 1):
    its persistent workgroups lost co-residency (another kernel held CUs) and its outputs are
    not trustworthy.  Re-run the call."""


def _require_device():
    """The library handle, after checking (once per device) that the current device is a
    gfx950; raises otherwise -- there is no CPU fallback."""
    dev = torch.cuda.current_device() if torch.cuda.is_available() else None
    L = _lib.lib()
    if dev in _checked_devices:
        return L
    if dev is None:
        raise RuntimeError("mtblx device codec needs a ROCm GPU (gfx950); none visible")
    if L.mtblx_device_ok() != 1:
        raise RuntimeError("mtblx device codec: current device is not gfx950 (MI355X)")
    _checked_devices.add(dev)
    return L


def _u(t: torch.Tensor) -> int:
    return t.data_ptr() if t is not None and t.numel() else 0


@dataclass
class DeviceBatch:
    """Uncompressed block contents resident in HBM.  data: uint8; blk_off: int64 (u64); blk_len: int32 (u32)."""
    data: torch.Tensor
    blk_off: torch.Tensor
    blk_len: torch.Tensor
    max_blk_len: int

    @property
    def nblk(self) -> int:
        return int(self.blk_off.numel())

    @staticmethod
    def from_host(data: np.ndarray, blk_off: np.ndarray, blk_len: np.ndarray, device="cuda") -> "DeviceBatch":
        d = torch.from_numpy(np.ascontiguousarray(data, np.uint8)).to(device)
        o = torch.from_numpy(np.ascontiguousarray(blk_off, np.uint64).view(np.int64)).to(device)
        ln = np.ascontiguousarray(blk_len, np.uint32)
        n = torch.from_numpy(ln.view(np.int32)).to(device)
        return DeviceBatch(d, o, n, int(ln.max()) if ln.size else 0)

    def cstruct(self) -> BlockBatch:
        c = getattr(self, "_c", None)
        if c is None:   # the tensors never change after construction
            c = BlockBatch(_u(self.data), int(self.data.numel()), _u(self.blk_off), _u(self.blk_len), self.nblk,
                           int(self.max_blk_len))
            self._c = c
        return c


class DecodedBlocks:
    """Device outputs in the layout of include/mtblx.h (mtblx_decoded)."""

    def __init__(self, nblk: int, rec_cap: int, keys_cap: int, vals_cap: int, device="cuda"):
        z = lambda n, dt: torch.zeros(max(int(n), 1), dtype=dt, device=device)  # noqa: E731
        self.nblk = nblk
        self.nrec = z(nblk, torch.int32)
        self.rec_base = z(nblk, torch.int64)
        self.key_base = z(nblk, torch.int64)
        self.val_base = z(nblk, torch.int64)
        self.status = z(nblk, torch.int32)
        self.key_end = z(rec_cap, torch.int32)
        self.val_end = z(rec_cap, torch.int32)
        self.keys = z(keys_cap, torch.uint8)
        self.vals = z(vals_cap, torch.uint8)
        self.totals = z(4, torch.int64)
        self.rec_cap, self.keys_cap, self.vals_cap = int(rec_cap), int(keys_cap), int(vals_cap)

    def cstruct(self) -> Decoded:
        c = getattr(self, "_c", None)
        if c is None:
            c = Decoded(_u(self.nrec), _u(self.rec_base), _u(self.key_base), _u(self.val_base), _u(self.status),
                        _u(self.key_end), _u(self.val_end), self.rec_cap, _u(self.keys), self.keys_cap,
                        _u(self.vals), self.vals_cap, _u(self.totals))
            self._c = c
        return c

    # ---------------- host views ----------------
    def totals_host(self, check: bool = True):
        """(records, key bytes, value bytes, flags); raises LaunchTimeout if the launch that
        wrote them timed out (check=False returns the raw flags)."""
        t = self.totals.cpu().numpy().view(np.uint64)
        if check and int(t[3]) & FLAG_TIMEOUT:
            raise LaunchTimeout("mtblx decode launch: look-back timeout, outputs discarded (re-run)")
        return int(t[0]), int(t[1]), int(t[2]), int(t[3])

    def to_host(self) -> "HostDecoded":
        nr, kb, vb, flags = self.totals_host()
        return HostDecoded(
            nrec=self.nrec[: self.nblk].cpu().numpy().view(np.uint32),
            rec_base=self.rec_base[: self.nblk].cpu().numpy().view(np.uint64),
            key_base=self.key_base[: self.nblk].cpu().numpy().view(np.uint64),
            val_base=self.val_base[: self.nblk].cpu().numpy().view(np.uint64),
            status=self.status[: self.nblk].cpu().numpy(),
            key_end=self.key_end[: min(nr, self.rec_cap)].cpu().numpy().view(np.uint32),
            val_end=self.val_end[: min(nr, self.rec_cap)].cpu().numpy().view(np.uint32),
            keys=self.keys[: min(kb, self.keys_cap)].cpu().numpy(),
            vals=self.vals[: min(vb, self.vals_cap)].cpu().numpy(),
            totals=(nr, kb, vb, flags),
        )


@dataclass
class HostDecoded:
    nrec: np.ndarray
    rec_base: np.ndarray
    key_base: np.ndarray
    val_base: np.ndarray
    status: np.ndarray
    key_end: np.ndarray
    val_end: np.ndarray
    keys: np.ndarray
    vals: np.ndarray
    totals: tuple

    def records(self, b: int):
        out = []
        r0, kb, vb = int(self.rec_base[b]), int(self.key_base[b]), int(self.val_base[b])
        pk = pv = 0
        for i in range(int(self.nrec[b])):
            ke, ve = int(self.key_end[r0 + i]), int(self.val_end[r0 + i])
            out.append((bytes(self.keys[kb + pk: kb + ke]), bytes(self.vals[vb + pv: vb + ve])))
            pk, pv = ke, ve
        return out


class WorkspaceBusy(RuntimeError):
    """A decode workspace was handed to a launch on one stream while a launch on another stream
    still used it (include/mtblx.h: one workspace serves one call at a time).  Its launch-parity
    protocol (decode.hip ws_begin: the parity comes from the epoch the previous launch left, and
    the other parity's slots are cleared for the next launch) holds only in stream order, which
    the kernels cannot check; two launches in flight on one workspace would read each other's
    look-back words.  Nothing was launched (the C ABI's MTBLX_E_INVAL class of error)."""


class Workspace:
    def __init__(self, nblk: int, device="cuda"):
        L = _lib.lib()
        self.nbytes = int(L.mtblx_decode_workspace_bytes(nblk))
        # zero-filled once: the kernels keep it consistent from call to call (include/mtblx.h)
        self.buf = torch.zeros(self.nbytes, dtype=torch.uint8, device=device)
        self._last = None   # (stream handle, event recorded after the last launch on this workspace)

    def _claim(self, stream) -> int:
        """-> the stream handle for a launch on this workspace; raises WorkspaceBusy if the last
        launch ran on another stream and has not completed (on the same stream, stream order
        already serialises them)"""
        h = _stream_handle(stream)
        if self._last is not None and self._last[0] != h and not self._last[1].query():
            raise WorkspaceBusy(f"decode workspace in use by a launch on stream 0x{self._last[0]:x} (not complete); "
                                f"one workspace serves one call at a time -- synchronise, or give each stream its own")
        return h

    def _launched(self, stream, h: int) -> None:
        ev = self._last[1] if self._last is not None else torch.cuda.Event()
        ev.record(stream if stream is not None else torch.cuda.current_stream())
        self._last = (h, ev)


def _stream_handle(stream) -> int:
    s = stream if stream is not None else torch.cuda.current_stream()
    return int(s.cuda_stream)


def count_blocks(batch: DeviceBatch, out: DecodedBlocks, ws: Workspace, stream=None) -> None:
    L = _require_device()
    b, o = batch.cstruct(), out.cstruct()
    h = ws._claim(stream)
    rc = L.mtblx_count_blocks(C.byref(b), C.byref(o), C.c_void_p(ws.buf.data_ptr()), ws.nbytes,
                              C.c_void_p(h))
    ws._launched(stream, h)
    if rc != 0:
        raise RuntimeError(f"mtblx_count_blocks failed: {rc}")


def decode_into(batch: DeviceBatch, out: DecodedBlocks, ws: Workspace, stream=None) -> None:
    """Asynchronous decode on `stream` into preallocated outputs (the timed hot call).
    The buffers must be ready on `stream` (allocate them under torch.cuda.stream(stream) or
    synchronize first): the library orders nothing across streams."""
    L = _require_device()
    b, o = batch.cstruct(), out.cstruct()
    h = ws._claim(stream)
    rc = L.mtblx_decode_blocks(C.byref(b), C.byref(o), C.c_void_p(ws.buf.data_ptr()), ws.nbytes,
                               C.c_void_p(h))
    ws._launched(stream, h)
    if rc != 0:
        raise RuntimeError(f"mtblx_decode_blocks failed: {rc}")


VERIFY_FUSED = 2


def decode_verify_into(batch: DeviceBatch, out: DecodedBlocks, ws: Workspace, crc=None, bad=None, framed=True,
                       stream=None, fused=False) -> None:
    """decode_into + the CRC-32C of every block (mtblx_decode_blocks_verify, f1): crc (int32
    [nblk]) and/or bad (uint8 [nblk]) device tensors.  fused=True: one launch (checksum from
    the LDS-staged tiles); default: decode then k_crc32c_blocks."""
    L = _require_device()
    b, o = batch.cstruct(), out.cstruct()
    flags = (1 if framed else 0) | (VERIFY_FUSED if fused else 0)
    h = ws._claim(stream)
    rc = L.mtblx_decode_blocks_verify(C.byref(b), C.byref(o), C.c_void_p(_u(crc)), C.c_void_p(_u(bad)),
                                      flags, C.c_void_p(ws.buf.data_ptr()), ws.nbytes,
                                      C.c_void_p(h))
    ws._launched(stream, h)
    if rc != 0:
        raise RuntimeError(f"mtblx_decode_blocks_verify failed: {rc}")


def decode_verify(batch: DeviceBatch, framed: bool = True, stream=None, fused=False):
    """Size exactly, allocate, decode + checksum in one launch -> (DecodedBlocks, crc, bad)."""
    _require_device()
    ws = Workspace(batch.nblk)
    probe = DecodedBlocks(batch.nblk, 0, 0, 0)
    count_blocks(batch, probe, ws, stream)
    torch.cuda.synchronize()
    nr, kb, vb, _ = probe.totals_host()
    out = DecodedBlocks(batch.nblk, nr, kb, vb)
    n = max(batch.nblk, 1)
    crc = torch.zeros(n, dtype=torch.int32, device=batch.data.device)
    bad = torch.zeros(n, dtype=torch.uint8, device=batch.data.device)
    decode_verify_into(batch, out, ws, crc, bad, framed, stream, fused)
    return out, crc[: batch.nblk], bad[: batch.nblk]


def decode_counted(batch: DeviceBatch, out: DecodedBlocks, ws: Workspace, stream=None) -> None:
    """Decode using the counts a previous count_blocks(batch, out, ws) left behind."""
    L = _require_device()
    b, o = batch.cstruct(), out.cstruct()
    h = ws._claim(stream)
    rc = L.mtblx_decode_counted(C.byref(b), C.byref(o), C.c_void_p(ws.buf.data_ptr()), ws.nbytes,
                                C.c_void_p(h))
    ws._launched(stream, h)
    if rc != 0:
        raise RuntimeError(f"mtblx_decode_counted failed: {rc}")


def decode_blocks(batch: DeviceBatch, stream=None) -> DecodedBlocks:
    """Size exactly (count pass), allocate, decode.  Synchronises once for the sizes."""
    _require_device()
    ws = Workspace(batch.nblk)
    probe = DecodedBlocks(batch.nblk, 0, 0, 0)
    count_blocks(batch, probe, ws, stream)
    torch.cuda.synchronize()
    nr, kb, vb, _ = probe.totals_host()
    out = DecodedBlocks(batch.nblk, nr, kb, vb)
    decode_into(batch, out, ws, stream)
    return out


def crc32c_blocks(batch: DeviceBatch, framed: bool = False, stream=None):
    """CRC-32C of every block's content on the device -> (crc uint32 tensor [nblk], bad uint8
    tensor [nblk] or None).  With framed=True the batch addresses contents inside an mtbl
    file and bad[b] = 1 where the stored checksum (the u32 before the content) differs: where
    Reader::block's assert_eq panics (src/reader.rs:159-164)."""
    L = _require_device()
    n = max(batch.nblk, 1)
    crc = torch.zeros(n, dtype=torch.int32, device=batch.data.device)
    bad = torch.zeros(n, dtype=torch.uint8, device=batch.data.device) if framed else None
    b = batch.cstruct()
    rc = L.mtblx_crc32c_blocks(C.byref(b), C.c_void_p(crc.data_ptr()), C.c_void_p(bad.data_ptr() if framed else 0),
                               1 if framed else 0, C.c_void_p(_stream_handle(stream)))
    if rc != 0:
        raise RuntimeError(f"mtblx_crc32c_blocks failed: {rc}")
    return crc[: batch.nblk], (bad[: batch.nblk] if framed else None)


# ---------------- snappy raw decompression on the device (f4) ----------------
class SnappyBatch:
    """Snappy-compressed (stored) block bytes resident in HBM: block b = data[src_off[b] .. + src_len[b])."""

    def __init__(self, data: torch.Tensor, src_off: torch.Tensor, src_len: torch.Tensor):
        self.data, self.src_off, self.src_len = data, src_off, src_len

    @property
    def nblk(self) -> int:
        return int(self.src_off.numel())

    @staticmethod
    def from_host(data: np.ndarray, src_off: np.ndarray, src_len: np.ndarray, device="cuda") -> "SnappyBatch":
        d = torch.from_numpy(np.ascontiguousarray(data, np.uint8)).to(device)
        o = torch.from_numpy(np.ascontiguousarray(src_off, np.uint64).view(np.int64)).to(device)
        n = torch.from_numpy(np.ascontiguousarray(src_len, np.uint32).view(np.int32)).to(device)
        return SnappyBatch(d, o, n)


class SnappyLayout:
    """Output layout of a SnappyBatch (mtblx_snappy_dir): dst_off (16-byte aligned), dst_len,
    per-block status (MTBLX_SNAPPY_*) and totals (layout bytes, max length, corrupt preambles)."""

    def __init__(self, nblk: int, device="cuda"):
        n = max(nblk, 1)
        self.nblk = nblk
        self.dst_off = torch.zeros(n, dtype=torch.int64, device=device)
        self.dst_len = torch.zeros(n, dtype=torch.int32, device=device)
        self.status = torch.zeros(n, dtype=torch.int32, device=device)
        self.totals = torch.zeros(3, dtype=torch.int64, device=device)
        L = _lib.lib()
        self.ws_bytes = int(L.mtblx_snappy_workspace_bytes(nblk))
        self.ws = torch.empty(max(self.ws_bytes, 8), dtype=torch.uint8, device=device)


def snappy_dir(batch: SnappyBatch, layout: SnappyLayout, stream=None) -> None:
    L = _require_device()
    rc = L.mtblx_snappy_dir(C.c_void_p(_u(batch.data)), C.c_void_p(_u(batch.src_off)), C.c_void_p(_u(batch.src_len)),
                            batch.nblk, C.c_void_p(_u(layout.dst_off)), C.c_void_p(_u(layout.dst_len)),
                            C.c_void_p(_u(layout.status)), C.c_void_p(_u(layout.totals)),
                            C.c_void_p(_u(layout.ws)), layout.ws_bytes, C.c_void_p(_stream_handle(stream)))
    if rc != 0:
        raise RuntimeError(f"mtblx_snappy_dir failed: {rc}")


def snappy_decompress_into(batch: SnappyBatch, layout: SnappyLayout, dst: torch.Tensor, status: torch.Tensor,
                           dec_len: torch.Tensor | None, max_len: int, stream=None) -> None:
    """Asynchronous device decompression of every block into dst at layout.dst_off."""
    L = _require_device()
    rc = L.mtblx_snappy_decompress_dev(C.c_void_p(_u(batch.data)), C.c_void_p(_u(batch.src_off)),
                                       C.c_void_p(_u(batch.src_len)), batch.nblk, C.c_void_p(_u(dst)),
                                       C.c_void_p(_u(layout.dst_off)), C.c_void_p(_u(layout.dst_len)), int(max_len),
                                       C.c_void_p(_u(status)), C.c_void_p(_u(dec_len)),
                                       C.c_void_p(_stream_handle(stream)))
    if rc != 0:
        raise RuntimeError(f"mtblx_snappy_decompress_dev failed: {rc}")


def snappy_decompress(batch: SnappyBatch, stream=None):
    """Layout + decompress -> (DeviceBatch of the decompressed blocks, status int32 [nblk]).
    The DeviceBatch feeds decode_blocks directly (a failed block has length 0)."""
    _require_device()
    lay = SnappyLayout(batch.nblk, batch.data.device)
    snappy_dir(batch, lay, stream)
    torch.cuda.synchronize()
    t = lay.totals.cpu().numpy().view(np.uint64)
    total, mx = int(t[0]), int(t[1])
    dst = torch.zeros(max(total, 16), dtype=torch.uint8, device=batch.data.device)
    status = torch.zeros(max(batch.nblk, 1), dtype=torch.int32, device=batch.data.device)
    dec_len = torch.zeros(max(batch.nblk, 1), dtype=torch.int32, device=batch.data.device)
    snappy_decompress_into(batch, lay, dst, status, dec_len, mx, stream)
    out = DeviceBatch(dst, lay.dst_off[: batch.nblk], dec_len[: batch.nblk], mx)
    return out, status[: batch.nblk]
