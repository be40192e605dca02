"""End-to-end decode from host memory (include/mtblx.h, mtblx_pipe_decode).

The north star's full path: an mtbl file in host memory in (read or mmap'd), the caller's
host byte slices out.  Per data block it does what Reader::block + BlockIter do
(/root/reference/src/reader.rs:140-175, src/block.rs:16-238): host decompression for
CompressionType::Snappy (src/compression.rs:116-119 -- the north star keeps compression on
the host), H2D, the device decode, D2H.  The chunked three-stage pipeline is native C++
(csrc/pipe.cpp); this module only owns pinned host buffers.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _lib, codec
from ._lib import Decoded, PipeStats


class PinnedArray:
    """A numpy view of pinned host memory (mtblx_host_alloc); freed with the object."""

    def __init__(self, n: int, dtype):
        self.n = max(int(n), 1)
        self.dtype = np.dtype(dtype)
        p = C.c_void_p()
        if _lib.lib().mtblx_host_alloc(C.byref(p), self.n * self.dtype.itemsize) != 0:
            raise MemoryError("mtblx_host_alloc failed")
        self.ptr = p.value
        buf = (C.c_uint8 * (self.n * self.dtype.itemsize)).from_address(self.ptr)
        self.a = np.frombuffer(buf, dtype=self.dtype)

    def __del__(self):
        try:
            if getattr(self, "ptr", None):
                _lib.lib().mtblx_host_free(C.c_void_p(self.ptr))
                self.ptr = None
        except Exception:
            pass


class HostOutputs:
    """mtblx_decoded in (pinned) host memory: the caller's byte slices."""

    def __init__(self, nblk: int, rec_cap: int, keys_cap: int, vals_cap: int, pinned: bool = True):
        mk = (lambda n, dt: PinnedArray(n, dt)) if pinned else (lambda n, dt: _Plain(n, dt))
        self._bufs = [mk(nblk, np.uint32), mk(nblk, np.uint64), mk(nblk, np.uint64), mk(nblk, np.uint64),
                      mk(nblk, np.int32), mk(rec_cap, np.uint32), mk(rec_cap, np.uint32), mk(keys_cap, np.uint8),
                      mk(vals_cap, np.uint8), mk(4, np.uint64)]
        (self.nrec, self.rec_base, self.key_base, self.val_base, self.status, self.key_end, self.val_end, self.keys,
         self.vals, self.totals) = [b.a for b in self._bufs]
        self.nblk = nblk
        self.rec_cap, self.keys_cap, self.vals_cap = int(rec_cap), int(keys_cap), int(vals_cap)
        p = [b.a.ctypes.data for b in self._bufs]
        self.c = Decoded(p[0], p[1], p[2], p[3], p[4], p[5], p[6], self.rec_cap, p[7], self.keys_cap, p[8],
                         self.vals_cap, p[9])

    def records(self, b: int):
        out = []
        r0, kb, vb = int(self.rec_base[b]), int(self.key_base[b]), int(self.val_base[b])
        pk = pv = 0
        for i in range(int(self.nrec[b])):
            ke, ve = int(self.key_end[r0 + i]), int(self.val_end[r0 + i])
            out.append((bytes(self.keys[kb + pk: kb + ke]), bytes(self.vals[vb + pv: vb + ve])))
            pk, pv = ke, ve
        return out


class _Plain:
    def __init__(self, n, dtype):
        self.a = np.zeros(max(int(n), 1), dtype)


class HostPipe:
    """mtblx_pipe: chunked host -> device -> host decode with three chunks in flight."""

    def __init__(self, chunk_bytes: int = 64 << 20, max_blocks: int = 1 << 16, threads: int = 16,
                 device_snappy="auto"):
        codec._require_device()
        self._p = _lib.lib().mtblx_pipe_new(int(chunk_bytes), int(max_blocks), int(threads))
        if not self._p:
            raise RuntimeError("mtblx_pipe_new failed")
        # MTBLX_PIPE_DEVICE_SNAPPY: snappy blocks cross PCIe compressed, decompressed on the device
        # (True), on the host (False), or "auto" (the device: faster end to end on any snappy stream)
        mode = 2 if device_snappy == "auto" else (1 if device_snappy else 0)
        if _lib.lib().mtblx_pipe_set(self._p, 1, mode) != 0:
            raise RuntimeError("mtblx_pipe_set failed")
        self.stats = PipeStats()

    def decode(self, file: np.ndarray, blk_off: np.ndarray, blk_len: np.ndarray, out: HostOutputs,
               compression: int = 0) -> PipeStats:
        f = np.ascontiguousarray(file, np.uint8)
        off = np.ascontiguousarray(blk_off, np.uint64)
        ln = np.ascontiguousarray(blk_len, np.uint32)
        rc = _lib.lib().mtblx_pipe_decode(self._p, f.ctypes.data, f.size, int(compression), off.ctypes.data,
                                          ln.ctypes.data, off.size, C.byref(out.c), C.byref(self.stats))
        if rc == _lib.MTBLX_E_TIMEOUT:
            raise codec.LaunchTimeout("mtblx_pipe_decode: a chunk's decode timed out twice (look-back)")
        if rc != 0:
            raise RuntimeError(f"mtblx_pipe_decode failed: {rc}")
        return self.stats

    def __del__(self):
        try:
            if getattr(self, "_p", None):
                _lib.lib().mtblx_pipe_free(self._p)
                self._p = None
        except Exception:
            pass


def register(a: np.ndarray) -> None:
    """Pin an existing host array in place (hipHostRegister), e.g. a read or mmap'd file."""
    if _lib.lib().mtblx_host_register(a.ctypes.data, a.nbytes) != 0:
        raise RuntimeError("mtblx_host_register failed")


def unregister(a: np.ndarray) -> None:
    _lib.lib().mtblx_host_unregister(a.ctypes.data)


# ---------------- host snappy (src/compression.rs:116-130) ----------------
def snappy_compress(data: bytes) -> bytes:
    L = _lib.lib()
    src = np.frombuffer(bytes(data), np.uint8) if len(data) else np.zeros(1, np.uint8)
    cap = int(L.mtblx_snappy_max_compressed_len(len(data)))
    dst = np.zeros(cap, np.uint8)
    n = C.c_uint64(0)
    if L.mtblx_snappy_compress(src.ctypes.data, len(data), dst.ctypes.data, cap, C.byref(n)) != 0:
        raise RuntimeError("mtblx_snappy_compress failed")
    return dst[: n.value].tobytes()


def snappy_decompress(data: bytes):
    """-> bytes, or None where snap::raw::Decoder returns an error (-> Error::Io)."""
    L = _lib.lib()
    src = np.frombuffer(bytes(data), np.uint8) if len(data) else np.zeros(1, np.uint8)
    u = C.c_uint64(0)
    if L.mtblx_snappy_uncompressed_len(src.ctypes.data, len(data), C.byref(u)) != 0:
        return None
    dst = np.zeros(max(u.value, 1), np.uint8)
    n = C.c_uint64(0)
    if L.mtblx_snappy_decompress(src.ctypes.data, len(data), dst.ctypes.data, u.value, C.byref(n)) != 0:
        return None
    return dst[: n.value].tobytes()
