"""Writer / WriterBuilder mirror (reference /root/reference/src/writer.rs:15-201).

Same names, argument meaning and error behaviour: ``insert`` of an out-of-order key is a
panic in the reference (src/writer.rs:119-123); here it raises ``OutOfOrderKey`` and the
writer is poisoned.  ``block_size`` is clamped to MIN_BLOCK_SIZE = 1024 (:43-46).
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _lib

DEFAULT_BLOCK_SIZE = 8192            # src/lib.rs:5
DEFAULT_BLOCK_RESTART_INTERVAL = 16  # src/lib.rs:4
MIN_BLOCK_SIZE = 1024                # src/lib.rs:6


class CompressionType:
    """src/compression.rs:6-15"""
    None_ = 0
    Snappy = 1
    Zlib = 2
    Lz4 = 3
    Lz4hc = 4
    Zstd = 5


class WriterPanic(RuntimeError):
    """Where the reference's Writer panics: an assert in BlockBuilder::add (src/block_builder.rs:
    50-51) -- the insert after a flush whose compressor returned Err -- or use after a panic."""


class OutOfOrderKey(WriterPanic):
    """panic!("out-of-order key") (src/writer.rs:119-123)."""


class WriterIoError(OSError):
    """Err(io::Error) from Writer::insert / into_inner: the data block's compressor failed
    (Lz4 / Lz4hc: "unsupported", src/compression.rs:70-81).  Nothing was written."""


def _io_message(compression: int) -> str:
    # the crate's message for Lz4 / Lz4hc (it says "decompression" in compress(), sic)
    return {3: "unsupported Lz4 decompression", 4: "unsupported Lz4hc decompression"}.get(
        compression, f"compression {compression} failed")


class WriterBuilder:
    def __init__(self):
        self._compression = CompressionType.None_
        self._level = 0
        self._block_size = DEFAULT_BLOCK_SIZE
        self._interval = DEFAULT_BLOCK_RESTART_INTERVAL

    def compression_type(self, c: int) -> "WriterBuilder":
        self._compression = c
        return self

    def compression_level(self, level: int) -> "WriterBuilder":
        self._level = level
        return self

    def block_size(self, n: int) -> "WriterBuilder":
        self._block_size = max(int(n), MIN_BLOCK_SIZE)
        return self

    def block_restart_interval(self, n: int) -> "WriterBuilder":
        self._interval = int(n)
        return self

    def memory(self) -> "Writer":
        return Writer(self._block_size, self._interval, self._compression, self._level)

    build = memory


class Writer:
    def __init__(self, block_size=DEFAULT_BLOCK_SIZE, restart_interval=DEFAULT_BLOCK_RESTART_INTERVAL,
                 compression=CompressionType.None_, level=0):
        L = _lib.lib()
        self._w = L.mtblx_writer_new(int(block_size), int(restart_interval), int(compression))
        if not self._w:
            # Zstd without libzstd.so.1 on this host (the crate bundles its own); Lz4 / Lz4hc build
            # a writer whose data-block flushes return Err (WriterIoError), as the crate's do
            raise ValueError(f"compression {compression}: unknown, or Zstd without libzstd.so.1 on this host")
        self._compression = int(compression)
        L.mtblx_writer_set_level(self._w, int(level))
        self.block_dir = None

    @staticmethod
    def memory() -> "Writer":
        return WriterBuilder().memory()

    @staticmethod
    def builder() -> WriterBuilder:
        return WriterBuilder()

    def insert(self, key, val) -> None:
        k = bytes(key.encode() if isinstance(key, str) else key)
        v = bytes(val.encode() if isinstance(val, str) else val)
        kb = (C.c_uint8 * max(1, len(k))).from_buffer_copy(k or b"\0")
        vb = (C.c_uint8 * max(1, len(v))).from_buffer_copy(v or b"\0")
        rc = _lib.lib().mtblx_writer_insert(self._w, kb, len(k), vb, len(v))
        self._check(rc, "mtblx_writer_insert")

    def _check(self, rc: int, what: str) -> None:
        if rc == _lib.MTBLX_E_FORMAT:
            raise OutOfOrderKey("out-of-order key")
        if rc == _lib.MTBLX_E_IO:
            raise WriterIoError(_io_message(self._compression))
        if rc == _lib.MTBLX_E_INVAL:
            raise WriterPanic("BlockBuilder::add: assertion failed (a block left finished by a failed flush), "
                              "or the writer already panicked")
        if rc != 0:
            raise RuntimeError(f"{what}: {rc}")

    def insert_batch(self, keys: np.ndarray, key_end: np.ndarray, vals: np.ndarray, val_end: np.ndarray) -> None:
        """Bulk insert of n records given as concatenated bytes + u64 end offsets."""
        keys = np.ascontiguousarray(keys, np.uint8)
        vals = np.ascontiguousarray(vals, np.uint8)
        ke = np.ascontiguousarray(key_end, np.uint64)
        ve = np.ascontiguousarray(val_end, np.uint64)
        if keys.size == 0:
            keys = np.zeros(1, np.uint8)
        if vals.size == 0:
            vals = np.zeros(1, np.uint8)
        rc = _lib.lib().mtblx_writer_insert_batch(self._w, keys.ctypes.data_as(_lib.u8p), ke.ctypes.data_as(_lib.u64p),
                                                  vals.ctypes.data_as(_lib.u8p), ve.ctypes.data_as(_lib.u64p),
                                                  ke.size)
        self._check(rc, "mtblx_writer_insert_batch")

    def into_inner(self) -> bytes:
        """Writer::into_inner: the finished .mtbl bytes.  Also records the data-block directory."""
        L = _lib.lib()
        out = _lib.u8p()
        n = C.c_uint64(0)
        rc = L.mtblx_writer_finish(self._w, C.byref(out), C.byref(n))
        self._check(rc, "mtblx_writer_finish")
        arr = np.empty(n.value, np.uint8)   # (ctypes.string_at takes a C int size: no files >= 2 GiB)
        C.memmove(arr.ctypes.data, out, n.value)
        L.mtblx_free(out)
        data = arr.tobytes()
        del arr
        nb = int(L.mtblx_writer_block_count(self._w))
        off = np.zeros(max(nb, 1), np.uint64)
        ln = np.zeros(max(nb, 1), np.uint32)
        nr = np.zeros(max(nb, 1), np.uint32)
        L.mtblx_writer_block_dir(self._w, off.ctypes.data_as(_lib.u64p), ln.ctypes.data_as(_lib.u32p),
                                 nr.ctypes.data_as(_lib.u32p))
        self.block_dir = (off[:nb], ln[:nb])
        self.block_nrec = nr[:nb]
        return data

    def into_inner_np(self) -> np.ndarray:
        """Same as into_inner, returned as a uint8 array without an extra bytes copy."""
        L = _lib.lib()
        out = _lib.u8p()
        n = C.c_uint64(0)
        rc = L.mtblx_writer_finish(self._w, C.byref(out), C.byref(n))
        self._check(rc, "mtblx_writer_finish")
        arr = np.empty(n.value, np.uint8)
        C.memmove(arr.ctypes.data, out, n.value)
        L.mtblx_free(out)
        nb = int(L.mtblx_writer_block_count(self._w))
        off = np.zeros(max(nb, 1), np.uint64)
        ln = np.zeros(max(nb, 1), np.uint32)
        nr = np.zeros(max(nb, 1), np.uint32)
        L.mtblx_writer_block_dir(self._w, off.ctypes.data_as(_lib.u64p), ln.ctypes.data_as(_lib.u32p),
                                 nr.ctypes.data_as(_lib.u32p))
        self.block_dir = (off[:nb], ln[:nb])
        self.block_nrec = nr[:nb]
        return arr

    finish = into_inner

    def __del__(self):
        try:
            if getattr(self, "_w", None):
                _lib.lib().mtblx_writer_free(self._w)
                self._w = None
        except Exception:
            pass
