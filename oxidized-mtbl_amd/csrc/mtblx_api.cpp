// mtblx_api.cpp — C ABI entry points of libmtblx.so (declared in include/mtblx.h).
//
// Thin, allocation-free glue: argument checks, then the kernel pipeline in decode.hip
// on the caller's stream.  See include/mtblx.h for the contract and the reference
// interfaces each entry point replaces.
#include <hip/hip_runtime.h>
#include <string.h>

#include "mtblx.h"

extern "C" size_t mtblx_impl_ws_bytes(uint32_t nblk);
extern "C" int mtblx_impl_run(const mtblx_block_batch* in, const mtblx_decoded* out, void* ws, size_t ws_bytes,
                              int write, hipStream_t s, int verify, uint32_t* crc, uint8_t* crc_bad, int framed);

extern "C" int mtblx_crc32c_blocks(const mtblx_block_batch* in, uint32_t* crc, uint8_t* bad, int framed,
                                   void* stream);

extern "C" int mtblx_abi_version(void) { return MTBLX_ABI_VERSION; }

extern "C" int mtblx_device_ok(void) {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return 0;
  hipDeviceProp_t p;
  if (hipGetDeviceProperties(&p, dev) != hipSuccess) return 0;
  return strncmp(p.gcnArchName, "gfx950", 6) == 0 ? 1 : 0;
}

extern "C" size_t mtblx_decode_workspace_bytes(uint32_t nblk) {
  return mtblx_impl_ws_bytes(nblk) + 256u;
}

static int check_common(const mtblx_block_batch* in, const mtblx_decoded* out, void* ws, size_t wsb, void* stream) {
  if (!in || !out) return MTBLX_E_INVAL;
  if (in->nblk == 0) {  // empty batch: zero totals, nothing else to do
    if (out->totals && hipMemsetAsync(out->totals, 0, 32, reinterpret_cast<hipStream_t>(stream)) != hipSuccess)
      return MTBLX_E_HIP;
    return MTBLX_OK;
  }
  if (!in->data || !in->blk_off || !in->blk_len) return MTBLX_E_INVAL;
  if (!out->nrec || !out->rec_base || !out->key_base || !out->val_base || !out->status || !out->totals)
    return MTBLX_E_INVAL;
  if (!ws || wsb < mtblx_decode_workspace_bytes(in->nblk)) return MTBLX_E_INVAL;
  if ((reinterpret_cast<uintptr_t>(ws) & 7u) != 0) return MTBLX_E_INVAL;
  return 1;
}

extern "C" int mtblx_count_blocks(const mtblx_block_batch* in, const mtblx_decoded* out, void* ws, size_t wsb,
                                  void* stream) {
  int c = check_common(in, out, ws, wsb, stream);
  if (c != 1) return c;
  return mtblx_impl_run(in, out, ws, wsb, 0, reinterpret_cast<hipStream_t>(stream), 0, nullptr, nullptr, 0);
}

extern "C" int mtblx_decode_counted(const mtblx_block_batch* in, const mtblx_decoded* out, void* ws, size_t wsb,
                                    void* stream) {
  int c = check_common(in, out, ws, wsb, stream);
  if (c != 1) return c;
  if ((!out->keys && out->keys_cap) || (!out->vals && out->vals_cap) || (!out->key_end && out->rec_cap) ||
      (!out->val_end && out->rec_cap))
    return MTBLX_E_INVAL;
  // single-pass kernel: counting is fused into the decode, so this is a full decode
  return mtblx_impl_run(in, out, ws, wsb, 1, reinterpret_cast<hipStream_t>(stream), 0, nullptr, nullptr, 0);
}

extern "C" int mtblx_decode_blocks(const mtblx_block_batch* in, const mtblx_decoded* out, void* ws, size_t wsb,
                                   void* stream) {
  int c = check_common(in, out, ws, wsb, stream);
  if (c != 1) return c;
  if ((!out->keys && out->keys_cap) || (!out->vals && out->vals_cap) || (!out->key_end && out->rec_cap) ||
      (!out->val_end && out->rec_cap))
    return MTBLX_E_INVAL;
  return mtblx_impl_run(in, out, ws, wsb, 1, reinterpret_cast<hipStream_t>(stream), 0, nullptr, nullptr, 0);
}

extern "C" int mtblx_decode_blocks_verify(const mtblx_block_batch* in, const mtblx_decoded* out, uint32_t* crc,
                                          uint8_t* crc_bad, int framed, void* ws, size_t wsb, void* stream) {
  int c = check_common(in, out, ws, wsb, stream);
  if (c != 1) return c;
  if ((!out->keys && out->keys_cap) || (!out->vals && out->vals_cap) || (!out->key_end && out->rec_cap) ||
      (!out->val_end && out->rec_cap) || (!crc && !crc_bad))
    return MTBLX_E_INVAL;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  if (framed & MTBLX_VERIFY_FUSED)   // one launch: the CRC from the LDS-staged tiles
    return mtblx_impl_run(in, out, ws, wsb, 1, s, 1, crc, crc_bad, framed & 1);
  // default: the decode, then the CRC-32C kernel (k_crc32c_mfma) on the same stream
  const int rc = mtblx_impl_run(in, out, ws, wsb, 1, s, 0, nullptr, nullptr, 0);
  if (rc != MTBLX_OK) return rc;
  return mtblx_crc32c_blocks(in, crc, crc_bad, framed & 1, stream);
}

// ---- bounds-checked diagnostic build only (csrc/bounds.h, Makefile target `bounds`) ----
#ifdef MTBLX_BOUNDS
#include <stdio.h>

#include <mutex>
#include <string>
static std::mutex g_bounds_mu;
static unsigned long long g_bounds_viol = 0, g_bounds_fault = 0;
static std::string g_bounds_first;

extern "C" void mtblx_bounds_note(const char* kernel, uint64_t line, uint64_t addr, uint64_t nbytes, int fault) {
  std::lock_guard<std::mutex> lk(g_bounds_mu);
  if (fault) ++g_bounds_fault;
  else ++g_bounds_viol;
  if (g_bounds_first.empty()) {
    char buf[512];
    snprintf(buf, sizeof(buf), "%s %s line %llu addr 0x%llx bytes %llu", fault ? "FAULT" : "OOB", kernel,
             (unsigned long long)line, (unsigned long long)addr, (unsigned long long)nbytes);
    g_bounds_first = buf;
  }
}
#endif

// Violations recorded by the bounds-checked build (violations | faults << 32), the first one
// described in buf.  The product build has nothing to report: -1.
extern "C" long long mtblx_bounds_report(char* buf, size_t cap) {
#ifdef MTBLX_BOUNDS
  std::lock_guard<std::mutex> lk(g_bounds_mu);
  if (buf && cap) snprintf(buf, cap, "%s", g_bounds_first.c_str());
  return (long long)(g_bounds_viol | (g_bounds_fault << 32));
#else
  (void)buf;
  (void)cap;
  return -1;
#endif
}
