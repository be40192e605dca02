// index.hip — MI355X (gfx950) tail of the device Writer: the index block and the footer.
//
//   Writer::insert's pending index entry   /root/reference/src/writer.rs:132-138
//   bytes_shortest_separator               src/writer.rs:239-265  (write_u16 APPENDS: kept)
//   Writer::into_inner                     src/writer.rs:155-181  (last entry, index write_block)
//   Metadata::write_to_bytes               src/metadata.rs:61-79  (512-byte footer)
//
// mtblx_encode_blocks (encode.hip) writes the data blocks of a file framed, back to back.
// For every data block b the Writer adds one index entry: key = the shortest separator
// between b's last key and block b+1's first key (the last block keeps the file's last
// key), value = varint64 of b's file offset (the offset of its framing).  Here:
//   k_index_len    one thread per block: separator length, varint length of the offset
//   k_scan2        one workgroup: exclusive -> END offsets of both (the index records' layout)
//   k_index_write  one thread per block: separator bytes, varint bytes
// then the entries are built into ONE block by mtblx_encode_blocks itself (BlockBuilder::add /
// finish with the same restart interval, framed, CompressionType::None: writer.rs:165-173),
// placed right after the data blocks, and the footer follows.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "mtblx.h"
#include "bounds.h"

namespace mtblx_idx {

constexpr int kThreads = 256;

__device__ __forceinline__ uint32_t vlen64(uint64_t v) {
  uint32_t n = 1;
  while (v >= 128) { v >>= 7; ++n; }
  return n;
}

struct Key {
  const uint8_t* p;
  uint64_t n;
};

__device__ __forceinline__ Key key_of(const mtblx_records& R, uint64_t r) {
  const uint64_t k0 = r ? R.key_end[r - 1] : 0;
  return Key{R.keys + k0, R.key_end[r] - k0};
}

// bytes_shortest_separator(start, limit) (src/writer.rs:239-265), release arithmetic:
//   di = common prefix length; di >= min_len -> unchanged;
//   start[di] < 255 && start[di] + 1 < limit[di] -> start[..di] + (start[di] + 1);
//   else if di < min_len - 2 (saturating): u = BE16(start[di..]) + 1 (wrapping) and
//     BE16(start[di..]) <= u <= BE16(limit[di..]) -> start + u as 2 BE bytes APPENDED
//     (write_u16 on a Vec appends, :254-262);
//   else unchanged.
// kind: 0 unchanged, 1 bump (length di + 1), 2 append (length |start| + 2).
struct Sep {
  uint64_t len, di;
  uint32_t kind;
  uint16_t u;
};

__device__ Sep separator(const Key& s, const Key& l) {
  const uint64_t m = s.n < l.n ? s.n : l.n;
  uint64_t di = 0;
  while (di < m && s.p[di] == l.p[di]) ++di;
  Sep r{s.n, di, 0, 0};
  if (di >= m) return r;
  const uint32_t db = s.p[di];
  if (db < 255u && db + 1u < l.p[di]) {
    r.len = di + 1;
    r.kind = 1;
  } else if (di < (m >= 2 ? m - 2 : 0)) {
    const uint16_t us = (uint16_t)((s.p[di] << 8) | s.p[di + 1]);
    const uint16_t ul = (uint16_t)((l.p[di] << 8) | l.p[di + 1]);
    const uint16_t ub = (uint16_t)(us + 1u);
    if (us <= ub && ub <= ul) {
      r.len = s.n + 2;
      r.kind = 2;
      r.u = ub;
    }
  }
  return r;
}

struct Args {
  mtblx_records R;
  const uint64_t* blk_rec;
  uint32_t nblk;
  const uint64_t* blk_off;
  const uint32_t* blk_len;
  uint64_t region_off;
  uint64_t* key_end;   // [nblk]: lengths, then END offsets
  uint64_t* val_end;
  uint8_t* keys;
  uint8_t* vals;
};

__device__ __forceinline__ Sep entry_key(const Args& a, uint32_t b, Key& start) {
  start = key_of(a.R, a.blk_rec[b + 1] - 1);                  // last key of block b
  if (b + 1 < a.nblk) return separator(start, key_of(a.R, a.blk_rec[b + 1]));   // vs the next block's first key
  return Sep{start.n, 0, 0, 0};                                // into_inner: the last key itself
}

__device__ __forceinline__ uint64_t entry_offset(const Args& a, uint32_t b) {
  // the block's file offset = its framing (varint64 len | crc32c) before the content
  return a.blk_off[b] - 4u - vlen64(a.blk_len[b]) - a.region_off;
}

__global__ void __launch_bounds__(kThreads) k_index_len(Args a) {
  const uint32_t b = blockIdx.x * kThreads + threadIdx.x;
  if (b >= a.nblk) return;
  Key s;
  a.key_end[b] = entry_key(a, b, s).len;
  a.val_end[b] = vlen64(entry_offset(a, b));
}

// in-place inclusive scan of two u64 arrays of n elements, one workgroup (index entries only)
__global__ void __launch_bounds__(1024) k_scan2(uint64_t* x, uint64_t* y, uint32_t n) {
  __shared__ uint64_t wx[16], wy[16];
  __shared__ uint64_t cx, cy;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  if (tid == 0) { cx = 0; cy = 0; }
  __syncthreads();
  for (uint32_t base = 0; base < n; base += 1024) {
    const uint32_t i = base + tid;
    uint64_t vx = i < n ? x[i] : 0, vy = i < n ? y[i] : 0;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const uint64_t ux = __shfl_up(vx, d, 64), uy = __shfl_up(vy, d, 64);
      if (lane >= d) { vx += ux; vy += uy; }
    }
    if (lane == 63) { wx[wv] = vx; wy[wv] = vy; }
    __syncthreads();
    uint64_t ox = cx, oy = cy;
    for (int k = 0; k < wv; ++k) { ox += wx[k]; oy += wy[k]; }
    if (i < n) { x[i] = ox + vx; y[i] = oy + vy; }
    __syncthreads();
    if (tid == 1023) { cx = ox + vx; cy = oy + vy; }
    __syncthreads();
  }
}

__global__ void __launch_bounds__(kThreads) k_index_write(Args a) {
  const uint32_t b = blockIdx.x * kThreads + threadIdx.x;
  if (b >= a.nblk) return;
  Key s;
  const Sep sp = entry_key(a, b, s);
  uint8_t* k = a.keys + (b ? a.key_end[b - 1] : 0);
  const uint64_t keep = sp.kind == 1 ? sp.di : s.n;
  for (uint64_t i = 0; i < keep; ++i) k[i] = s.p[i];
  if (sp.kind == 1) k[sp.di] = (uint8_t)(s.p[sp.di] + 1u);
  if (sp.kind == 2) { k[s.n] = (uint8_t)(sp.u >> 8); k[s.n + 1] = (uint8_t)sp.u; }
  uint64_t v = entry_offset(a, b);                                // varint_encode64 (src/varint.rs:63-76)
  uint8_t* vp = a.vals + (b ? a.val_end[b - 1] : 0);
  while (v >= 128) { *vp++ = (uint8_t)(v | 128); v >>= 7; }
  *vp = (uint8_t)v;
}

}  // namespace mtblx_idx

namespace {
struct DevMem {   // temporaries of this (synchronous, once-per-file) call
  void* p = nullptr;
  ~DevMem() { if (p) (void)hipFree(p); }
  bool alloc(size_t n) {   // MTBLX_DEBUG_POISON (test knob): fresh memory filled with 0xFF
    return hipMalloc(&p, n ? n : 1) == hipSuccess && (!getenv("MTBLX_DEBUG_POISON") || hipMemset(p, 0xFF, n ? n : 1) == hipSuccess);
  }
  template <class T> T* as(size_t byte_off = 0) const { return reinterpret_cast<T*>(static_cast<uint8_t*>(p) + byte_off); }
};
}  // namespace

extern "C" int mtblx_encode_index(const mtblx_records* rec, const uint64_t* blk_rec, uint32_t nblk,
                                  uint64_t block_size, uint32_t restart_interval, const uint8_t* data,
                                  uint64_t region_off, uint64_t data_bytes, const uint64_t* blk_off,
                                  const uint32_t* blk_len, uint8_t* file, uint64_t file_cap, uint64_t* file_len,
                                  void* stream) {
  using namespace mtblx_idx;
  if (!rec || !file || !file_len || (nblk && (!blk_rec || !blk_off || !blk_len || !data))) return MTBLX_E_INVAL;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  if (block_size < 1024) block_size = 1024;   // WriterBuilder::block_size clamp (src/writer.rs:43-46)
  if (data_bytes + 13 + 512 > file_cap) return MTBLX_E_INVAL;
  if (nblk && file != data + region_off &&
      hipMemcpyAsync(file, data + region_off, data_bytes, hipMemcpyDeviceToDevice, s) != hipSuccess)
    return MTBLX_E_HIP;
  // the index records: nblk entries (END offsets + bytes), the index block's directory
  DevMem ends;
  if (!ends.alloc(16ull * nblk + 64)) return MTBLX_E_HIP;
  uint64_t* key_end = ends.as<uint64_t>();
  uint64_t* val_end = key_end + nblk;
  uint64_t* small = val_end + nblk;   // [0..1] blk_rec of the index block, [2..3] totals, [4] blk_off, [5] len|status
  Args a{*rec, blk_rec, nblk, blk_off, blk_len, region_off, key_end, val_end, nullptr, nullptr};
  uint64_t kbytes = 0, vbytes = 0;
  if (nblk) {
    const dim3 g((nblk + kThreads - 1) / kThreads);
    MTBLX_LAUNCH((blk_off, blk_len, key_end, val_end, blk_rec), k_index_len, g, dim3(kThreads), 0, s, a);
    MTBLX_LAUNCH((key_end, val_end), k_scan2, dim3(1), dim3(1024), 0, s, key_end, val_end, nblk);
    if (hipGetLastError() != hipSuccess || hipMemcpyAsync(&kbytes, key_end + nblk - 1, 8, hipMemcpyDeviceToHost, s) ||
        hipMemcpyAsync(&vbytes, val_end + nblk - 1, 8, hipMemcpyDeviceToHost, s) || hipStreamSynchronize(s))
      return MTBLX_E_HIP;
  }
  DevMem kv;
  if (!kv.alloc(kbytes + vbytes + 16)) return MTBLX_E_HIP;
  a.keys = kv.as<uint8_t>();
  a.vals = kv.as<uint8_t>(kbytes + 8);
  if (nblk) {
    MTBLX_LAUNCH((blk_off, blk_len, key_end, val_end, blk_rec, kv.p), k_index_write, dim3((nblk + kThreads - 1) / kThreads), dim3(kThreads), 0, s, a);
    if (hipGetLastError() != hipSuccess) return MTBLX_E_HIP;
  }
  // Writer::into_inner: the index block, written like any block (write_block, None, framed)
  const uint64_t idx_rec[2] = {0, nblk};
  if (hipMemcpyAsync(small, idx_rec, 16, hipMemcpyHostToDevice, s) != hipSuccess) return MTBLX_E_HIP;
  const size_t wsb = mtblx_encode_workspace_bytes(1);
  DevMem ws;
  if (!ws.alloc(wsb)) return MTBLX_E_HIP;
  const mtblx_records ir{a.keys, key_end, a.vals, val_end, nblk};
  int rc = mtblx_encode_blocks(&ir, small, 1, restart_interval, 1, file + data_bytes, file_cap - data_bytes - 512,
                               small + 4, reinterpret_cast<uint32_t*>(small + 5),
                               reinterpret_cast<int32_t*>(small + 5) + 1, small + 2, ws.p, wsb, stream);
  if (rc != MTBLX_OK) return rc;
  uint64_t h[6] = {0, 0, 0, 0, 0, 0};
  if (hipMemcpyAsync(h, small, 48, hipMemcpyDeviceToHost, s) != hipSuccess || hipStreamSynchronize(s) != hipSuccess)
    return MTBLX_E_HIP;
  const int32_t ist = static_cast<int32_t>(h[5] >> 32);
  if (h[3] & 2ull) return MTBLX_E_TIMEOUT;
  if (ist != MTBLX_ST_OK || (h[3] & 1ull)) return ist == MTBLX_ST_OVERFLOW ? MTBLX_E_INVAL : MTBLX_E_FORMAT;
  const uint64_t idx_bytes = h[2];
  // Metadata::write_to_bytes (src/metadata.rs:61-79): 9 x u64 LE, zero pad, magic u32 LE at 508
  uint64_t r0 = 0, r1 = 0, k0 = 0, k1 = 0, v0 = 0, v1 = 0;
  if (nblk) {
    if (hipMemcpy(&r0, blk_rec, 8, hipMemcpyDeviceToHost) || hipMemcpy(&r1, blk_rec + nblk, 8, hipMemcpyDeviceToHost))
      return MTBLX_E_HIP;
    if (r0 && (hipMemcpy(&k0, rec->key_end + r0 - 1, 8, hipMemcpyDeviceToHost) ||
               hipMemcpy(&v0, rec->val_end + r0 - 1, 8, hipMemcpyDeviceToHost)))
      return MTBLX_E_HIP;
    if (r1 && (hipMemcpy(&k1, rec->key_end + r1 - 1, 8, hipMemcpyDeviceToHost) ||
               hipMemcpy(&v1, rec->val_end + r1 - 1, 8, hipMemcpyDeviceToHost)))
      return MTBLX_E_HIP;
  }
  uint8_t foot[512];
  memset(foot, 0, sizeof foot);
  const uint64_t meta[9] = {data_bytes, block_size, 0, r1 - r0, nblk, data_bytes, idx_bytes, k1 - k0, v1 - v0};
  memcpy(foot, meta, sizeof meta);   // little-endian host (x86-64)
  const uint32_t magic = 0x4D54424Cu;   // FormatV2 (src/lib.rs:17-20)
  memcpy(foot + 508, &magic, 4);
  if (hipMemcpyAsync(file + data_bytes + idx_bytes, foot, 512, hipMemcpyHostToDevice, s) != hipSuccess ||
      hipStreamSynchronize(s) != hipSuccess)
    return MTBLX_E_HIP;
  *file_len = data_bytes + idx_bytes + 512;
  return MTBLX_OK;
}
