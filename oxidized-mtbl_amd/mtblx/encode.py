"""Device encode side: the Writer's block cut + BlockBuilder + write_block framing.

Python front-end of mtblx_encode_plan / mtblx_encode_blocks (include/mtblx.h, csrc/encode.hip):
    Writer::insert flush rule   /root/reference/src/writer.rs:125-130
    BlockBuilder::add / finish  src/block_builder.rs:49-104
    write_block framing + crc   src/writer.rs:203-237
Records stay on the device (torch tensors as plumbing); the kernels do the work.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass

import torch

from . import _lib, codec
from ._lib import Records


class WriterPanic(RuntimeError):
    """Where Writer::insert / BlockBuilder::add panic (flags: _lib.PLAN_*)."""

    def __init__(self, flags: int):
        super().__init__(f"writer panic flags={flags}")
        self.flags = flags


@dataclass
class DeviceRecords:
    """keys/vals: uint8; key_end/val_end: int64 END offsets (u64) from record 0."""
    keys: torch.Tensor
    key_end: torch.Tensor
    vals: torch.Tensor
    val_end: torch.Tensor

    @property
    def n(self) -> int:
        return int(self.key_end.numel())

    def cstruct(self) -> Records:
        u = codec._u
        return Records(u(self.keys), u(self.key_end), u(self.vals), u(self.val_end), self.n)

    @staticmethod
    def from_list(records, device="cuda") -> "DeviceRecords":
        import numpy as np
        ks = b"".join(bytes(k) for k, _ in records)
        vs = b"".join(bytes(v) for _, v in records)
        ke = np.cumsum([len(k) for k, _ in records], dtype=np.int64) if records else np.zeros(0, np.int64)
        ve = np.cumsum([len(v) for _, v in records], dtype=np.int64) if records else np.zeros(0, np.int64)
        t = lambda b: torch.frombuffer(bytearray(b or b"\0"), dtype=torch.uint8).to(device)  # noqa: E731
        return DeviceRecords(t(ks), torch.from_numpy(ke).to(device), t(vs), torch.from_numpy(ve).to(device))


class PlanWorkspace:
    """Caller-owned scratch of the block cut (mtblx_plan_workspace_bytes): sized for up to `nrec`
    records in `nshard` shards, reusable across calls (one call at a time).  The library keeps no
    scratch of its own (include/mtblx.h)."""

    def __init__(self, nrec: int, nshard: int = 1, restart_interval: int = 16, keep: bool = False, device="cuda",
                 serial: bool = False):
        L = _lib.lib()
        if serial:   # the serial walk's 16 B per shard (same cut, one wave per shard)
            self.nbytes = int(L.mtblx_plan_serial_workspace_bytes(max(int(nshard), 1)))
        else:
            self.nbytes = int(L.mtblx_plan_workspace_bytes(max(int(nrec), 0), max(int(nshard), 1),
                                                           int(restart_interval), 1 if keep else 0))
        self.buf = torch.empty(self.nbytes + 256, dtype=torch.uint8, device=device)
        self.ptr = (self.buf.data_ptr() + 255) & ~255   # 256-byte aligned


KEEP_MAX_RECORDS = (1 << 32) - 16   # mtblx_encode_plan_keep: 32-bit next / waypoint arrays


def plan(recs: DeviceRecords, block_size: int = 8192, restart_interval: int = 16, shard_rec=None,
         stream=None, keep: bool = False, workspace: "PlanWorkspace | None" = None):
    """-> blk_rec (device int64 [nblk + 1]): block b = records [blk_rec[b], blk_rec[b+1]).
    shard_rec: record boundaries of independent Writers (default: one Writer over all).
    keep=True (restart_interval >= 1): -> (blk_rec, Plan), the cut's sums kept for encode_into.
    workspace: a PlanWorkspace to reuse (default: one allocated for this call; without keep, a
    workspace that does not fit falls back to the serial walk's 16 B per shard)."""
    L = codec._require_device()
    dev = recs.key_end.device
    if shard_rec is None:
        shard_rec = torch.tensor([0, recs.n], dtype=torch.int64, device=dev)
    nsh = int(shard_rec.numel()) - 1
    if workspace is None:
        try:
            workspace = PlanWorkspace(recs.n, nsh, restart_interval, keep, device=dev)
        except torch.OutOfMemoryError:
            if keep:
                raise
            workspace = PlanWorkspace(recs.n, nsh, restart_interval, device=dev, serial=True)
    rc_ = recs.cstruct()
    nb = C.c_uint64(0)
    fl = C.c_uint32(0)
    st = C.c_void_p(codec._stream_handle(stream))
    # one call: every block holds >= 1 record, so the shards' record count + 1 always suffices
    cap = max(recs.n, 0) + 1
    blk = torch.empty(cap, dtype=torch.int64, device=dev)
    args = [C.byref(rc_), C.c_void_p(shard_rec.data_ptr()), nsh, int(block_size), int(restart_interval),
            C.c_void_p(blk.data_ptr()), cap, C.byref(nb), C.byref(fl)]
    ws = [C.c_void_p(workspace.ptr), workspace.nbytes]
    kept = None
    if keep:
        kb = int(L.mtblx_plan_keep_bytes(recs.n))
        kept = Plan(torch.empty(kb + 256, dtype=torch.uint8, device=dev), int(restart_interval))
        rc = L.mtblx_encode_plan_keep(*args, C.c_void_p(kept.ptr), kb, *ws, st)
    else:
        rc = L.mtblx_encode_plan(*args, *ws, st)
    if rc == _lib.MTBLX_E_FORMAT:
        raise WriterPanic(int(fl.value))
    if rc != 0:
        raise RuntimeError(f"mtblx_encode_plan failed: {rc}")
    blk = blk[: int(nb.value) + 1]
    return (blk, kept) if keep else blk


@dataclass
class Plan:
    """the block cut's kept sums (mtblx_encode_plan_keep): lets encode_into skip the size pass and
    the look-back (mtblx_encode_blocks_planned)"""
    buf: torch.Tensor
    restart_interval: int

    @property
    def ptr(self) -> int:
        """the plan's 256-byte aligned start inside buf"""
        return (self.buf.data_ptr() + 255) & ~255


@dataclass
class Encoded:
    out: torch.Tensor       # uint8: blocks (framed: back to back from 0)
    blk_off: torch.Tensor   # int64 content offsets
    blk_len: torch.Tensor   # int32 content lengths
    status: torch.Tensor    # int32 MTBLX_ST_*
    totals: torch.Tensor    # int64 [2]: bytes, flags

    def check(self) -> "Encoded":
        """raise codec.LaunchTimeout if the encode launch's look-back timed out (totals[1] bit 1)"""
        if int(self.totals[1].item()) & codec.FLAG_TIMEOUT:
            raise codec.LaunchTimeout("mtblx_encode_blocks: look-back timeout, outputs discarded (re-run)")
        return self

    def batch(self) -> codec.DeviceBatch:
        """the encoded blocks as a decode batch (mtblx_decode_blocks input)"""
        ml = int(self.blk_len.max().item()) if self.blk_len.numel() else 0
        return codec.DeviceBatch(self.out, self.blk_off, self.blk_len, ml)


class EncodeBuffers:
    """Output + workspace of mtblx_encode_blocks, sized once for a record set and plan."""

    def __init__(self, recs: DeviceRecords, nblk: int, device="cuda"):
        L = _lib.lib()
        n = recs.n
        cap = int(recs.keys.numel()) + int(recs.vals.numel()) + 19 * n + 30 * nblk + 64
        self.out = torch.empty(cap, dtype=torch.uint8, device=device)
        m = max(nblk, 1)
        self.blk_off = torch.empty(m, dtype=torch.int64, device=device)
        self.blk_len = torch.empty(m, dtype=torch.int32, device=device)
        self.status = torch.empty(m, dtype=torch.int32, device=device)
        self.totals = torch.zeros(2, dtype=torch.int64, device=device)
        self.ws_bytes = int(L.mtblx_encode_workspace_bytes(m))
        self.ws = torch.empty(self.ws_bytes, dtype=torch.uint8, device=device)
        self.nblk = nblk


def encode_into(recs: DeviceRecords, blk_rec: torch.Tensor, bufs: EncodeBuffers, restart_interval: int = 16,
                framed: bool = True, stream=None, plan: "Plan | None" = None) -> Encoded:
    """mtblx_encode_blocks; with a kept plan (plan(..., keep=True)) mtblx_encode_blocks_planned"""
    L = codec._require_device()
    nblk = int(blk_rec.numel()) - 1
    rc_ = recs.cstruct()
    args = [C.byref(rc_), C.c_void_p(blk_rec.data_ptr()), nblk, int(restart_interval), 1 if framed else 0,
            C.c_void_p(bufs.out.data_ptr()), bufs.out.numel(), C.c_void_p(bufs.blk_off.data_ptr()),
            C.c_void_p(bufs.blk_len.data_ptr()), C.c_void_p(bufs.status.data_ptr()), C.c_void_p(bufs.totals.data_ptr()),
            C.c_void_p(bufs.ws.data_ptr()), bufs.ws_bytes]
    if plan is not None:
        rc = L.mtblx_encode_blocks_planned(*args, C.c_void_p(plan.ptr), C.c_void_p(codec._stream_handle(stream)))
    else:
        rc = L.mtblx_encode_blocks(*args, C.c_void_p(codec._stream_handle(stream)))
    if rc != 0:
        raise RuntimeError(f"mtblx_encode_blocks failed: {rc}")
    return Encoded(bufs.out, bufs.blk_off[:nblk], bufs.blk_len[:nblk], bufs.status[:nblk], bufs.totals)


def encode_blocks(recs: DeviceRecords, blk_rec: torch.Tensor, restart_interval: int = 16, framed: bool = True,
                  stream=None, plan: "Plan | None" = None) -> Encoded:
    bufs = EncodeBuffers(recs, int(blk_rec.numel()) - 1, device=recs.key_end.device)
    return encode_into(recs, blk_rec, bufs, restart_interval, framed, stream, plan)


def write_file(recs: DeviceRecords, block_size: int = 8192, restart_interval: int = 16, stream=None) -> torch.Tensor:
    """The crate's Writer on the device for ONE file (src/writer.rs): insert every record
    (block cut: plan; BlockBuilder + write_block: encode_blocks, framed), then into_inner
    (index block + footer: mtblx_encode_index).  -> the file bytes (device uint8), byte-identical
    to Writer::into_inner for the same records (CompressionType::None)."""
    L = codec._require_device()
    dev = recs.key_end.device
    kept = None
    if 1 <= restart_interval and recs.n < KEEP_MAX_RECORDS:
        try:   # the cut's sums drive the encode (no size pass, no look-back)
            blk, kept = plan(recs, block_size, restart_interval, stream=stream, keep=True)
        except torch.OutOfMemoryError:   # keep mode's plan + scratch (~70 B per record) did not fit
            kept = None
    if kept is None:   # the cut alone (serial walk if even its scratch does not fit) + the self-contained encode
        blk = plan(recs, block_size, restart_interval, stream=stream)
    nblk = int(blk.numel()) - 1
    kbytes = int(recs.key_end[-1].item()) if recs.n else 0
    if nblk:
        e = encode_blocks(recs, blk, restart_interval, framed=True, stream=stream, plan=kept)
        torch.cuda.synchronize()
        e.check()
        if int(e.totals[1].item()) & 1:
            raise WriterPanic(int((e.status != 0).nonzero()[0].item()) if bool((e.status != 0).any()) else 0)
        data_bytes = int(e.totals[0].item())
        data, off, ln = e.out, e.blk_off, e.blk_len
    else:
        data_bytes = 0
        data = off = ln = None
    # index block: separators (<= last key + 2 B) + varint64 offsets + headers + restarts + framing
    cap = data_bytes + kbytes + 36 * nblk + 64 + 512
    file = torch.empty(cap, dtype=torch.uint8, device=dev)
    n = C.c_uint64(0)
    rc_ = recs.cstruct()
    u = codec._u
    rc = L.mtblx_encode_index(C.byref(rc_), C.c_void_p(u(blk)), nblk, int(block_size), int(restart_interval),
                              C.c_void_p(u(data) if data is not None else u(file)), 0, data_bytes,
                              C.c_void_p(u(off) if off is not None else 0), C.c_void_p(u(ln) if ln is not None else 0),
                              C.c_void_p(file.data_ptr()), cap, C.byref(n), C.c_void_p(codec._stream_handle(stream)))
    if rc == _lib.MTBLX_E_TIMEOUT:
        raise codec.LaunchTimeout("mtblx_encode_index: look-back timeout")
    if rc != 0:
        raise RuntimeError(f"mtblx_encode_index failed: {rc}")
    return file[: n.value]
