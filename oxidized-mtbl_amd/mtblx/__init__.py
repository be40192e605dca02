"""mtblx — MI355X-native mtbl block codec (drop-in for Kerollmops/oxidized-mtbl's block decode path).

Package layout
  _lib.py     ctypes binding of libmtblx.so (include/mtblx.h, include/mtblx_host.h)
  codec.py    device batch decode (HIP kernels in csrc/decode.hip)
  writer.py   Writer / WriterBuilder mirror of src/writer.rs
  synth.py    deterministic synthetic workloads of BASELINE.json's configs
"""
from ._lib import EXPORTS, LIB_PATH, lib  # noqa: F401
from .writer import CompressionType, OutOfOrderKey, Writer, WriterBuilder  # noqa: F401

__all__ = ["Writer", "WriterBuilder", "CompressionType", "OutOfOrderKey", "lib", "LIB_PATH", "EXPORTS"]
