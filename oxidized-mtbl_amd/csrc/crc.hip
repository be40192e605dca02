// crc.hip — MI355X (gfx950) CRC-32C of block contents: the checksum Reader::block verifies
// before it decodes a block (/root/reference/src/reader.rs:159-164, crate crc32c 0.4:
// CRC-32C Castagnoli, reflected polynomial 0x82F63B78, init/xorout 0xFFFFFFFF).
//
// One wave per block.  The block is cut into 64-byte chunks counted from its END; lane j
// computes the raw (init 0, no xorout) table-driven CRC of chunk j, then shifts it to its
// place by a GF(2) multiply with x^(8*64*j) mod P:
//   crc_raw(A || B) = multmodp(x^(8|B|), crc_raw(A)) ^ crc_raw(B)
// and the wave XOR-reduces.  The 0xFFFFFFFF init is folded in by complementing the first 4
// content bytes (equivalent for blocks of >= 4 bytes); the result is complemented at the end.
// x^(512 m) for any chunk index m comes from three 512-entry tables (9 bits each), computed
// at compile time (crc_dev.h).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "crc_dev.h"
#include "mtblx.h"

namespace mtblx_crc {

__global__ void __launch_bounds__(kThreads) k_crc32c_blocks(const uint8_t* data, uint64_t data_len, const uint64_t* blk_off,
                                                            const uint32_t* blk_len, uint32_t nblk, uint32_t* crc_out,
                                                            uint8_t* bad, int framed) {
  __shared__ uint32_t T[256];
  for (int i = threadIdx.x; i < 256; i += kThreads) T[i] = kTab.byte[i];
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const uint32_t waves = gridDim.x * (kThreads / kWave);
  for (uint32_t b = blockIdx.x * (kThreads / kWave) + (threadIdx.x >> 6); b < nblk; b += waves) {
    const uint64_t off = blk_off[b];
    const uint64_t L = blk_len[b];
    const uint8_t* d = data + off;
    // a window past the buffer: the reference's slice panics before the checksum (bad = 1)
    const bool oob = off + L > data_len;
    const uint32_t acc = oob ? 0u : wave_crc32c(d, L, T, lane);
    if (lane == 0) {
      if (crc_out) crc_out[b] = acc;
      if (bad && oob) {
        bad[b] = 1;
      } else if (bad) {
        uint32_t stored = 0;
        if (framed && off >= 4)
          stored = (uint32_t)d[-4] | ((uint32_t)d[-3] << 8) | ((uint32_t)d[-2] << 16) | ((uint32_t)d[-1] << 24);
        bad[b] = (framed && off >= 4) ? (uint8_t)(stored != acc) : (uint8_t)0;
      }
    }
  }
}

}  // namespace mtblx_crc

extern "C" int mtblx_crc32c_blocks(const mtblx_block_batch* in, uint32_t* crc, uint8_t* bad, int framed,
                                   void* stream) {
  if (!in || (!crc && !bad && in->nblk)) return MTBLX_E_INVAL;
  if (in->nblk == 0) return MTBLX_OK;
  if (!in->data || !in->blk_off || !in->blk_len) return MTBLX_E_INVAL;
  static int grid = 0;
  if (!grid) {
    int dev = 0, ncu = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
    grid = (ncu > 0 ? ncu : 256) * 8;   // 32 waves per CU in flight
  }
  const uint32_t need = (in->nblk + 3u) / 4u;
  hipLaunchKernelGGL(mtblx_crc::k_crc32c_blocks, dim3(need < (uint32_t)grid ? need : (uint32_t)grid),
                     dim3(mtblx_crc::kThreads), 0, reinterpret_cast<hipStream_t>(stream), in->data, in->data_len, in->blk_off,
                     in->blk_len, in->nblk, crc, bad, framed);
  return hipGetLastError() == hipSuccess ? MTBLX_OK : MTBLX_E_HIP;
}
