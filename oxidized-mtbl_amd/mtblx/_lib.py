"""ctypes binding of libmtblx.so (include/mtblx.h, include/mtblx_host.h).

The library is built in-tree (``make -C oxidized-mtbl_amd``).  There is no fallback:
if the shared object is missing, importing the codec raises.
"""
from __future__ import annotations

import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
# MTBLX_LIB selects the diagnostic stamps build (bench.py --stamps); default is the product build
LIB_PATH = os.environ.get("MTBLX_LIB") or os.path.join(_HERE, "libmtblx.so")

u8p = C.POINTER(C.c_uint8)
u32p = C.POINTER(C.c_uint32)
u64p = C.POINTER(C.c_uint64)
i32p = C.POINTER(C.c_int32)

MTBLX_OK, MTBLX_E_INVAL, MTBLX_E_HIP, MTBLX_E_NODEV, MTBLX_E_FORMAT, MTBLX_E_TIMEOUT, MTBLX_E_IO = 0, -1, -2, -3, -4, -5, -6
ST_OK, ST_INVALID_BLOCK, ST_CORRUPT, ST_LOOP, ST_UNSUPPORTED, ST_OVERFLOW, ST_DECOMPRESS = range(7)
SNAPPY_OK, SNAPPY_CORRUPT, SNAPPY_TOO_SMALL, SNAPPY_TIMEOUT = range(4)
CODEC_OK, CODEC_CORRUPT, CODEC_UNSUPPORTED = range(3)
DIR_OK, DIR_PANIC, DIR_UNSUPPORTED = range(3)
GET_FOUND, GET_NONE, GET_PANIC, GET_ERR, GET_LOOP, GET_MISSING = range(6)
SEEK_OK, SEEK_ERR, SEEK_PANIC, SEEK_LOOP, SEEK_UNSUPPORTED = range(5)
EMIT_END, EMIT_PANIC, EMIT_LOOP, EMIT_MAX, EMIT_OVERFLOW = range(5)

# every symbol the public headers declare (checked by tests/test_abi.py)
EXPORTS = [
    "mtblx_abi_version", "mtblx_device_ok", "mtblx_decode_workspace_bytes", "mtblx_decode_blocks",
    "mtblx_count_blocks", "mtblx_decode_counted", "mtblx_decode_blocks_verify", "mtblx_crc32c_blocks", "mtblx_block_dir", "mtblx_get", "mtblx_get_decompressed", "mtblx_crc32c", "mtblx_varint_decode64", "mtblx_read_footer", "mtblx_frame_block",
    "mtblx_writer_new", "mtblx_writer_insert", "mtblx_writer_insert_batch", "mtblx_writer_finish",
    "mtblx_writer_block_count", "mtblx_writer_block_dir", "mtblx_writer_free", "mtblx_free",
    "mtblx_snappy_max_compressed_len", "mtblx_snappy_uncompressed_len", "mtblx_snappy_decompress",
    "mtblx_snappy_compress", "mtblx_snappy_decompress_blocks", "mtblx_pipe_new", "mtblx_pipe_free",
    "mtblx_pipe_decode", "mtblx_pipe_set", "mtblx_host_alloc", "mtblx_host_free", "mtblx_host_register", "mtblx_host_unregister",
    "mtblx_encode_plan", "mtblx_encode_workspace_bytes", "mtblx_encode_blocks", "mtblx_plan_keep_bytes",
    "mtblx_encode_plan_keep", "mtblx_encode_blocks_planned", "mtblx_plan_release", "mtblx_plan_workspace_bytes",
    "mtblx_plan_serial_workspace_bytes",
    "mtblx_snappy_workspace_bytes", "mtblx_snappy_dir", "mtblx_snappy_decompress_dev", "mtblx_stream_copy", "mtblx_encode_index",
    "mtblx_codec_available", "mtblx_decompress", "mtblx_compress", "mtblx_decompress_blocks", "mtblx_writer_set_level",
    "mtblx_index_seek_batch", "mtblx_block_seek_batch", "mtblx_block_seek_batch_kbuf", "mtblx_block_seek_batch_ex", "mtblx_copy_ranges", "mtblx_entry_offsets",
    "mtblx_key_filter",
]
PLAN_OUT_OF_ORDER, PLAN_PANIC, PLAN_TOO_LONG = 1, 2, 4


class BlockBatch(C.Structure):
    _fields_ = [("data", C.c_void_p), ("data_len", C.c_uint64), ("blk_off", C.c_void_p), ("blk_len", C.c_void_p),
                ("nblk", C.c_uint32), ("max_blk_len", C.c_uint32)]


class Decoded(C.Structure):
    _fields_ = [("nrec", C.c_void_p), ("rec_base", C.c_void_p), ("key_base", C.c_void_p), ("val_base", C.c_void_p),
                ("status", C.c_void_p), ("key_end", C.c_void_p), ("val_end", C.c_void_p), ("rec_cap", C.c_uint64),
                ("keys", C.c_void_p), ("keys_cap", C.c_uint64), ("vals", C.c_void_p), ("vals_cap", C.c_uint64),
                ("totals", C.c_void_p)]


class Records(C.Structure):
    _fields_ = [("keys", C.c_void_p), ("key_end", C.c_void_p), ("vals", C.c_void_p), ("val_end", C.c_void_p),
                ("n", C.c_uint64)]


class PipeStats(C.Structure):
    _fields_ = [("seconds", C.c_double), ("stage_seconds", C.c_double), ("decode_ms", C.c_double),
                ("block_bytes", C.c_uint64), ("h2d_bytes", C.c_uint64), ("d2h_bytes", C.c_uint64),
                ("chunks", C.c_uint32), ("decompress_errors", C.c_uint32)]


class IndexSeek(C.Structure):   # mtblx_index_seek
    _fields_ = [("status", C.c_int32), ("valid", C.c_int32), ("entry", C.c_uint64), ("block_off", C.c_uint64),
                ("block_status", C.c_int32), ("pad", C.c_int32), ("data_off", C.c_uint64), ("data_len", C.c_uint64)]


class BlockSeek(C.Structure):   # mtblx_block_seek
    _fields_ = [("data_off", C.c_uint64), ("data_len", C.c_uint64), ("kcap", C.c_uint64), ("max_records", C.c_uint64),
                ("first", C.c_int32), ("status", C.c_int32), ("end", C.c_int32), ("has_val", C.c_int32),
                ("entry", C.c_uint64), ("nrec", C.c_uint64), ("key_bytes", C.c_uint64), ("val_bytes", C.c_uint64),
                ("last_voff", C.c_uint64), ("last_vlen", C.c_uint64), ("resume_off", C.c_uint64),
                ("stop_off", C.c_uint64), ("early", C.c_int32), ("pad", C.c_int32)]


class Footer(C.Structure):
    _fields_ = [("meta", C.c_uint64 * 9), ("version", C.c_uint32), ("err", C.c_int32)]


_lib = None


def lib() -> C.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(f"libmtblx.so not built ({LIB_PATH}); run `make -C oxidized-mtbl_amd` "
                              "(no CPU fallback exists for the device codec)")
        # torch bundles its own libamdhip64.so.7 (same soname as /opt/rocm's): whichever loads
        # first serves the whole process.  Load torch first, so the device pointers and streams
        # torch hands us and libmtblx's kernels live in one HIP runtime (the order every
        # product path takes); without torch, libmtblx uses the system runtime.
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
        L = C.CDLL(LIB_PATH)
        L.mtblx_abi_version.restype = C.c_int
        L.mtblx_device_ok.restype = C.c_int
        L.mtblx_decode_workspace_bytes.argtypes = [C.c_uint32]
        L.mtblx_decode_workspace_bytes.restype = C.c_size_t
        for f in (L.mtblx_decode_blocks, L.mtblx_count_blocks, L.mtblx_decode_counted):
            f.argtypes = [C.POINTER(BlockBatch), C.POINTER(Decoded), C.c_void_p, C.c_size_t, C.c_void_p]
            f.restype = C.c_int
        L.mtblx_decode_blocks_verify.argtypes = [C.POINTER(BlockBatch), C.POINTER(Decoded), C.c_void_p, C.c_void_p,
                                                 C.c_int, C.c_void_p, C.c_size_t, C.c_void_p]
        L.mtblx_decode_blocks_verify.restype = C.c_int
        L.mtblx_crc32c_blocks.argtypes = [C.POINTER(BlockBatch), C.c_void_p, C.c_void_p, C.c_int, C.c_void_p]
        L.mtblx_crc32c_blocks.restype = C.c_int
        L.mtblx_block_dir.argtypes = [C.c_void_p, C.c_uint64, C.c_uint32, C.c_void_p, C.c_void_p, C.c_uint64,
                                      C.c_uint32, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]
        L.mtblx_block_dir.restype = C.c_int
        L.mtblx_get.argtypes = [C.c_void_p, C.c_uint64, C.c_uint32, C.c_int, C.c_uint64, C.c_uint64, C.c_void_p,
                                C.c_void_p, C.c_uint32, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]
        L.mtblx_get.restype = C.c_int
        L.mtblx_get_decompressed.argtypes = [C.c_void_p, C.c_uint64, C.c_uint32, C.c_int, C.c_uint64, C.c_uint64,
                                             C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint32, C.c_void_p,
                                             C.c_void_p, C.c_void_p, C.c_uint32, C.c_void_p, C.c_void_p, C.c_void_p,
                                             C.c_void_p]
        L.mtblx_get_decompressed.restype = C.c_int
        L.mtblx_crc32c.argtypes = [u8p, C.c_uint64]
        L.mtblx_crc32c.restype = C.c_uint32
        L.mtblx_varint_decode64.argtypes = [u8p, C.c_uint64, u64p]
        L.mtblx_varint_decode64.restype = C.c_int
        L.mtblx_read_footer.argtypes = [u8p, C.c_uint64, C.POINTER(Footer)]
        L.mtblx_read_footer.restype = C.c_int
        L.mtblx_frame_block.argtypes = [u8p, C.c_uint64, C.c_uint32, C.c_uint64, C.c_int, u64p, u64p,
                                        C.POINTER(C.c_int)]
        L.mtblx_frame_block.restype = C.c_int
        L.mtblx_writer_new.argtypes = [C.c_uint64, C.c_uint64, C.c_uint32]
        L.mtblx_writer_new.restype = C.c_void_p
        L.mtblx_writer_insert.argtypes = [C.c_void_p, u8p, C.c_uint64, u8p, C.c_uint64]
        L.mtblx_writer_insert.restype = C.c_int
        L.mtblx_writer_insert_batch.argtypes = [C.c_void_p, u8p, u64p, u8p, u64p, C.c_uint64]
        L.mtblx_writer_insert_batch.restype = C.c_int
        L.mtblx_writer_finish.argtypes = [C.c_void_p, C.POINTER(u8p), u64p]
        L.mtblx_writer_finish.restype = C.c_int
        L.mtblx_writer_block_count.argtypes = [C.c_void_p]
        L.mtblx_writer_block_count.restype = C.c_uint64
        L.mtblx_writer_block_dir.argtypes = [C.c_void_p, u64p, u32p, u32p]
        L.mtblx_writer_block_dir.restype = C.c_int
        L.mtblx_writer_free.argtypes = [C.c_void_p]
        L.mtblx_free.argtypes = [C.c_void_p]
        L.mtblx_snappy_max_compressed_len.argtypes = [C.c_uint64]
        L.mtblx_snappy_max_compressed_len.restype = C.c_uint64
        L.mtblx_snappy_uncompressed_len.argtypes = [C.c_void_p, C.c_uint64, u64p]
        L.mtblx_snappy_uncompressed_len.restype = C.c_int
        L.mtblx_snappy_decompress.argtypes = [C.c_void_p, C.c_uint64, C.c_void_p, C.c_uint64, u64p]
        L.mtblx_snappy_decompress.restype = C.c_int
        L.mtblx_snappy_compress.argtypes = [C.c_void_p, C.c_uint64, C.c_void_p, C.c_uint64, u64p]
        L.mtblx_snappy_compress.restype = C.c_int
        L.mtblx_snappy_decompress_blocks.argtypes = [C.c_void_p] * 7 + [C.c_uint64, C.c_uint32]
        L.mtblx_snappy_decompress_blocks.restype = C.c_uint64
        L.mtblx_pipe_new.argtypes = [C.c_uint64, C.c_uint32, C.c_uint32]
        L.mtblx_pipe_new.restype = C.c_void_p
        L.mtblx_pipe_free.argtypes = [C.c_void_p]
        L.mtblx_pipe_decode.argtypes = [C.c_void_p, C.c_void_p, C.c_uint64, C.c_uint32, C.c_void_p, C.c_void_p,
                                        C.c_uint32, C.POINTER(Decoded), C.POINTER(PipeStats)]
        L.mtblx_pipe_decode.restype = C.c_int
        L.mtblx_pipe_set.argtypes = [C.c_void_p, C.c_int, C.c_int64]
        L.mtblx_pipe_set.restype = C.c_int
        L.mtblx_encode_plan.argtypes = [C.POINTER(Records), C.c_void_p, C.c_uint32, C.c_uint64, C.c_uint32,
                                        C.c_void_p, C.c_uint64, u64p, u32p, C.c_void_p, C.c_size_t, C.c_void_p]
        L.mtblx_encode_plan.restype = C.c_int
        L.mtblx_encode_workspace_bytes.argtypes = [C.c_uint32]
        L.mtblx_encode_workspace_bytes.restype = C.c_size_t
        L.mtblx_encode_blocks.argtypes = [C.POINTER(Records), C.c_void_p, C.c_uint32, C.c_uint32, C.c_int, C.c_void_p,
                                          C.c_uint64, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
                                          C.c_size_t, C.c_void_p]
        L.mtblx_encode_blocks.restype = C.c_int
        L.mtblx_plan_keep_bytes.argtypes = [C.c_uint64]
        L.mtblx_plan_keep_bytes.restype = C.c_size_t
        L.mtblx_encode_plan_keep.argtypes = L.mtblx_encode_plan.argtypes[:-3] + [C.c_void_p, C.c_size_t, C.c_void_p,
                                                                                 C.c_size_t, C.c_void_p]
        L.mtblx_plan_workspace_bytes.argtypes = [C.c_uint64, C.c_uint32, C.c_uint32, C.c_int]
        L.mtblx_plan_workspace_bytes.restype = C.c_size_t
        L.mtblx_plan_serial_workspace_bytes.argtypes = [C.c_uint32]
        L.mtblx_plan_serial_workspace_bytes.restype = C.c_size_t
        L.mtblx_encode_plan_keep.restype = C.c_int
        L.mtblx_encode_blocks_planned.argtypes = L.mtblx_encode_blocks.argtypes[:-1] + [C.c_void_p, C.c_void_p]
        L.mtblx_encode_blocks_planned.restype = C.c_int
        L.mtblx_snappy_workspace_bytes.argtypes = [C.c_uint32]
        L.mtblx_snappy_workspace_bytes.restype = C.c_size_t
        L.mtblx_snappy_dir.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint32, C.c_void_p, C.c_void_p,
                                       C.c_void_p, C.c_void_p, C.c_void_p, C.c_size_t, C.c_void_p]
        L.mtblx_snappy_dir.restype = C.c_int
        L.mtblx_snappy_decompress_dev.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint32, C.c_void_p,
                                                  C.c_void_p, C.c_void_p, C.c_uint32, C.c_void_p, C.c_void_p,
                                                  C.c_void_p]
        L.mtblx_snappy_decompress_dev.restype = C.c_int
        L.mtblx_encode_index.argtypes = [C.POINTER(Records), C.c_void_p, C.c_uint32, C.c_uint64, C.c_uint32, C.c_void_p,
                                         C.c_uint64, C.c_uint64, C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint64, u64p,
                                         C.c_void_p]
        L.mtblx_encode_index.restype = C.c_int
        L.mtblx_codec_available.argtypes = [C.c_uint32]
        L.mtblx_codec_available.restype = C.c_int
        L.mtblx_decompress.argtypes = [C.c_uint32, C.c_void_p, C.c_uint64, C.POINTER(u8p), u64p]
        L.mtblx_decompress.restype = C.c_int
        L.mtblx_compress.argtypes = [C.c_uint32, C.c_uint32, C.c_void_p, C.c_uint64, C.POINTER(u8p), u64p]
        L.mtblx_compress.restype = C.c_int
        L.mtblx_decompress_blocks.argtypes = [C.c_uint32, C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint64, C.c_uint32,
                                              C.POINTER(u8p), C.c_void_p, C.c_void_p, C.c_void_p]
        L.mtblx_decompress_blocks.restype = C.c_uint64
        L.mtblx_writer_set_level.argtypes = [C.c_void_p, C.c_uint32]
        L.mtblx_writer_set_level.restype = C.c_int
        L.mtblx_stream_copy.argtypes = [C.c_void_p, C.c_void_p, C.c_uint64, C.c_int, C.c_void_p]
        L.mtblx_stream_copy.restype = C.c_int
        L.mtblx_index_seek_batch.argtypes = [C.c_void_p, C.c_uint64, C.c_uint32, C.c_int, C.c_uint64, C.c_uint64,
                                             C.c_void_p, C.c_void_p, C.c_uint32, C.c_void_p, C.c_void_p]
        L.mtblx_index_seek_batch.restype = C.c_int
        L.mtblx_block_seek_batch.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint32, C.c_void_p, C.c_void_p,
                                             C.c_uint64, C.c_void_p, C.c_uint64, C.c_void_p, C.c_void_p, C.c_void_p,
                                             C.c_uint64, C.c_void_p]
        L.mtblx_block_seek_batch.restype = C.c_int
        L.mtblx_block_seek_batch_kbuf.argtypes = L.mtblx_block_seek_batch.argtypes[:-1] + [C.c_void_p, C.c_uint64,
                                                                                          C.c_void_p]
        L.mtblx_block_seek_batch_kbuf.restype = C.c_int
        L.mtblx_block_seek_batch_ex.argtypes = L.mtblx_block_seek_batch_kbuf.argtypes[:-1] + [C.c_void_p, C.c_void_p]
        L.mtblx_block_seek_batch_ex.restype = C.c_int
        L.mtblx_copy_ranges.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
                                        C.c_uint32, C.c_uint64, C.c_void_p]
        L.mtblx_copy_ranges.restype = C.c_int
        L.mtblx_entry_offsets.argtypes = [C.c_void_p, C.c_uint64, C.c_void_p, C.c_uint64, C.c_void_p, C.c_void_p,
                                           C.c_void_p]
        L.mtblx_entry_offsets.restype = C.c_int
        L.mtblx_key_filter.argtypes = [C.c_void_p, C.c_void_p, C.c_uint64, C.c_int32, C.c_void_p, C.c_uint64,
                                       C.c_void_p, C.c_void_p]
        L.mtblx_key_filter.restype = C.c_int
        L.mtblx_host_alloc.argtypes = [C.POINTER(C.c_void_p), C.c_uint64]
        L.mtblx_host_alloc.restype = C.c_int
        L.mtblx_host_free.argtypes = [C.c_void_p]
        L.mtblx_host_free.restype = C.c_int
        L.mtblx_host_register.argtypes = [C.c_void_p, C.c_uint64]
        L.mtblx_host_register.restype = C.c_int
        L.mtblx_host_unregister.argtypes = [C.c_void_p]
        L.mtblx_host_unregister.restype = C.c_int
        _lib = L
    return _lib
