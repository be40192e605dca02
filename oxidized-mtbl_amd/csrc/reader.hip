// reader.hip — MI355X (gfx950) index block -> data-block directory.
//
// The reference walks the index block one entry at a time (ReaderIntoIter::next,
// /root/reference/src/reader.rs:337-405) and, per entry, decodes the data block offset
// from the entry's value and frames the block:
//   block_at_index   src/reader.rs:177-186   varint_decode64(value) -> file offset
//   Reader::block    src/reader.rs:139-174   assert offset < len; varint64 (V2) / u32 (V1)
//                                            content length; crc32c; content slice
// Here the index block is first decoded like any other block (mtblx_decode_blocks), then
// one thread per entry does the offset decode + framing for every entry at once.  The CRC
// and Block::init checks of Reader::block are done by mtblx_crc32c_blocks (framed) and by
// the decode kernel's per-block status, over the directory this kernel writes.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "mtblx.h"

namespace mtblx_rd {

// varint_length_packed over d[0..n) (src/varint.rs:1-10): 0 if no terminator
__device__ __forceinline__ uint32_t length_packed(const uint8_t* d, uint64_t n) {
  for (uint64_t i = 0; i < n; ++i)
    if (!(d[i] & 0x80u)) return (uint32_t)i + 1;
  return 0;
}

// varint_decode64 on the slice d[0..n) (src/varint.rs:78-97 with varint_decode32 :44-61).
// Returns the consumed length (0 = unterminated), or -1 where the reference panics
// (n == 0: it indexes data[0]; fewer than 4 bytes on the 64-bit path: data[1..3]).
__device__ __forceinline__ int dec64(const uint8_t* d, uint64_t n, uint64_t& v) {
  if (n == 0) return -1;
  const uint32_t l = length_packed(d, n < 10 ? n : 10);
  if (l < 5) {
    const uint32_t l32 = length_packed(d, n < 5 ? n : 5);
    uint32_t val = d[0] & 0x7fu;
    if (l32 > 1) val |= (uint32_t)(d[1] & 0x7fu) << 7;
    if (l32 > 2) val |= (uint32_t)(d[2] & 0x7fu) << 14;
    if (l32 > 3) val |= (uint32_t)(d[3] & 0x7fu) << 21;
    if (l32 > 4) val |= (uint32_t)d[4] << 28;
    v = val;
    return (int)l32;
  }
  uint64_t val = (uint64_t)(d[0] & 0x7fu) | ((uint64_t)(d[1] & 0x7fu) << 7) | ((uint64_t)(d[2] & 0x7fu) << 14) |
                 ((uint64_t)(d[3] & 0x7fu) << 21);
  uint32_t shift = 28;
  for (uint32_t i = 4; i < l; ++i) {
    val |= (uint64_t)(d[i] & 0x7fu) << shift;
    shift += 7;
  }
  v = val;
  return (int)l;
}

__global__ void k_block_dir(const uint8_t* file, uint64_t file_len, uint32_t version, const uint8_t* vals,
                            const uint32_t* val_end, uint64_t val_base, uint32_t nent, uint64_t* blk_off,
                            uint32_t* blk_len, int32_t* dir_st) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nent) return;
  const uint64_t v0 = val_base + (i ? val_end[i - 1] : 0u), v1 = val_base + val_end[i];
  uint64_t off = 0, start = 0, sz = 0;
  int32_t st = MTBLX_DIR_OK;
  // block_at_index: varint_decode64(value, &mut offset), return length ignored
  if (dec64(vals + v0, v1 - v0, off) < 0) st = MTBLX_DIR_PANIC;
  // Reader::block
  if (st == MTBLX_DIR_OK && !(off < file_len)) st = MTBLX_DIR_PANIC;   // assert!(offset < len)
  uint64_t ll = 0;
  if (st == MTBLX_DIR_OK) {
    if (version == 0) {  // FormatV1: u32 LE length
      if (off + 4 > file_len) st = MTBLX_DIR_PANIC;
      else {
        ll = 4;
        sz = (uint64_t)file[off] | ((uint64_t)file[off + 1] << 8) | ((uint64_t)file[off + 2] << 16) |
             ((uint64_t)file[off + 3] << 24);
      }
    } else {
      const int k = dec64(file + off, file_len - off, sz);
      if (k < 0) st = MTBLX_DIR_PANIC;
      else ll = (uint64_t)k;
    }
  }
  if (st == MTBLX_DIR_OK) {
    start = off + ll + 4;
    if (start > file_len || sz > file_len - start) st = MTBLX_DIR_PANIC;   // BytesView::slice assert
    else if (sz > 0xFFFFFFFFull) st = MTBLX_DIR_UNSUPPORTED;
  }
  blk_off[i] = st == MTBLX_DIR_OK ? start : 0;
  blk_len[i] = st == MTBLX_DIR_OK ? (uint32_t)sz : 0u;
  dir_st[i] = st;
}

}  // namespace mtblx_rd

extern "C" int mtblx_block_dir(const uint8_t* file, uint64_t file_len, uint32_t version, const uint8_t* vals,
                               const uint32_t* val_end, uint64_t val_base, uint32_t nent, uint64_t* blk_off,
                               uint32_t* blk_len, int32_t* dir_st, void* stream) {
  if (nent == 0) return MTBLX_OK;
  if (!file || !vals || !val_end || !blk_off || !blk_len || !dir_st || version > 1) return MTBLX_E_INVAL;
  const uint32_t threads = 256;
  hipLaunchKernelGGL(mtblx_rd::k_block_dir, dim3((nent + threads - 1) / threads), dim3(threads), 0,
                     reinterpret_cast<hipStream_t>(stream), file, file_len, version, vals, val_end, val_base, nent,
                     blk_off, blk_len, dir_st);
  return hipGetLastError() == hipSuccess ? MTBLX_OK : MTBLX_E_HIP;
}
