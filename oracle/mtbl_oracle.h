/*
 * mtbl_oracle.h — CPU ORACLE for the mtbl block codec.  TEST INFRASTRUCTURE ONLY.
 *
 * This is a plain-C restatement of the reference Rust crate (Kerollmops/oxidized-mtbl)
 * for the decode hot path and the framing around it.  Every function cites the
 * reference file:line it restates.  It exists to CHECK the product (the HIP decoder
 * behind include/mtblx.h); only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load it.  The product never links or calls it.
 *
 * Parity pinning: the reference is Rust and cannot be built here (no cargo/rustc, see
 * DESIGN.md).  The oracle is pinned by the hand-derived known-answer vectors of
 * SURVEY.md §2.2 (byte-exact one_key / empty files, block CRCs) and the CRC-32C check
 * value, committed under tests/golden/, plus the reference's own test scenarios
 * restated in tests/test_oracle.py.
 *
 * Semantics notes (all documented in DESIGN.md §"Reference quirks"):
 *  - Rust RELEASE-mode arithmetic is emulated (wrapping usize/u32 arithmetic where the
 *    reference would only panic in debug builds).
 *  - Every reference panic is reported as MTBLX_ST_CORRUPT; records yielded before
 *    the panic are kept (the reference's iterator had already returned them).
 *  - An entry that makes zero forward progress makes the reference iterate forever;
 *    the oracle yields it once and reports MTBLX_ST_LOOP.
 *  - Vec<u8>::capacity() of the iterator's key buffer is emulated (Rust >= 1.50 growth
 *    policy: max(2*cap, len+add, 8)) because src/block.rs:132 asserts on it.
 */
#ifndef MTBL_ORACLE_H
#define MTBL_ORACLE_H

#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

/* per-block status codes: identical numbering to include/mtblx.h */
enum {
  ORC_ST_OK = 0,
  ORC_ST_INVALID_BLOCK = 1, /* Block::init returned None (src/block.rs:16-49)      */
  ORC_ST_CORRUPT = 2,       /* the reference panics while decoding this block      */
  ORC_ST_LOOP = 3,          /* zero-progress entry: the reference never terminates */
  ORC_ST_UNSUPPORTED = 4,
  ORC_ST_OVERFLOW = 5       /* caller's output capacity too small                  */
};

/* ---- varint (src/varint.rs) ---- */
uint32_t oracle_varint_length_packed(const uint8_t* data, uint64_t len);
uint32_t oracle_varint_encode32(uint8_t* out, uint32_t value);
uint32_t oracle_varint_encode64(uint8_t* out, uint64_t value);
/* returns consumed length (0 = unterminated, per reference); -1 = reference panic */
int32_t oracle_varint_decode32(const uint8_t* data, uint64_t len, uint32_t* value);
int32_t oracle_varint_decode64(const uint8_t* data, uint64_t len, uint64_t* value);

/* ---- snappy raw decompression (src/compression.rs:116-119, crate snap 1.x): 0 + malloc'd
 * *out, or 7 (ORC_ERR_IO) where the reference returns Err(Error::Io) ---- */
int32_t oracle_snappy_decompress(const uint8_t* src, uint64_t n, uint8_t** out, uint64_t* out_len);

/* ---- crc32c (crate crc32c 0.4: CRC-32C Castagnoli, reflected 0x82F63B78) ---- */
uint32_t oracle_crc32c(const uint8_t* data, uint64_t len);

/* ---- block decode (src/block.rs) ----
 * Batch form with the SAME output layout as mtblx_decode_blocks (include/mtblx.h):
 *   blocks b = [data + blk_off[b], +blk_len[b])
 *   per block: nrec[b], key_bytes[b], val_bytes[b], status[b]
 *   rec_base/key_base/val_base = exclusive prefix sums over blocks (computed here)
 *   per record (global index rec_base[b]+i): key_end/val_end = END offset of record i's
 *   key/value relative to key_base[b]/val_base[b].
 * Pass NULL output arrays to only count.  Returns 0, or ORC_ST_OVERFLOW if a capacity
 * was exceeded (counts are still complete). */
int32_t oracle_decode_blocks(const uint8_t* data, const uint64_t* blk_off, const uint32_t* blk_len,
                             uint32_t nblk, uint32_t* nrec, uint64_t* key_bytes, uint64_t* val_bytes,
                             int32_t* status, uint64_t* rec_base, uint64_t* key_base, uint64_t* val_base,
                             uint8_t* keys, uint64_t keys_cap, uint8_t* vals, uint64_t vals_cap,
                             uint32_t* key_end, uint32_t* val_end, uint64_t rec_cap);

/* CPU baseline (reference semantics, variant A of BASELINE.md): seek_to_first/next/get
 * per block, key rebuilt in a reused buffer, value borrowed, FNV-1a fold of every
 * (key,value) to defeat dead-code elimination.  Static block partition over nthreads.
 * Returns the fold; *ns = wall time of `iters` passes. */
uint64_t oracle_bench_scan(const uint8_t* data, const uint64_t* blk_off, const uint32_t* blk_len,
                           uint32_t nblk, int nthreads, int iters, uint64_t* ns, uint64_t* nrec_total);

/* ---- block builder + writer (src/block_builder.rs, src/writer.rs, src/metadata.rs) ---- */
typedef struct oracle_writer oracle_writer;
oracle_writer* oracle_writer_new(uint64_t block_size, uint64_t restart_interval, uint32_t compression);
/* returns 0, or -1 when the reference panics ("out-of-order key" / interval assert) */
int32_t oracle_writer_insert(oracle_writer* w, const uint8_t* key, uint64_t klen, const uint8_t* val,
                             uint64_t vlen);
/* finishes the file; *out is malloc'd (free with oracle_free). returns 0 / -1 */
int32_t oracle_writer_finish(oracle_writer* w, uint8_t** out, uint64_t* out_len);
void oracle_writer_free(oracle_writer* w);
void oracle_free(void* p);

/* single block via BlockBuilder: records given as concatenated keys/vals + end offsets */
int32_t oracle_build_block(uint64_t restart_interval, uint64_t nrec, const uint8_t* keys,
                           const uint64_t* key_end, const uint8_t* vals, const uint64_t* val_end,
                           uint8_t** out, uint64_t* out_len);

/* bytes_shortest_separator (src/writer.rs:239-265). start buffer must have room for len+2.
 * returns new length, or -1 when the reference asserts. */
int64_t oracle_shortest_separator(uint8_t* start, uint64_t start_len, const uint8_t* limit,
                                  uint64_t limit_len);

/* ---- file-level iteration (src/reader.rs ReaderBuilder::read + ReaderIntoIter::{new,next}) ----
 * Outcome codes for oracle_scan_result.end: */
enum {
  ORC_END_NONE = 0,      /* iterator returned None                              */
  ORC_END_ERR_OPEN = 1,  /* Reader::new / into_iter returned Err(err)           */
  ORC_END_ERR_NEXT = 2,  /* next() returned Some(Err(err))                      */
  ORC_END_PANIC = 3,     /* the reference panics                                */
  ORC_END_LOOP = 4       /* the reference yields the same record forever         */
};
enum { /* MtblError (src/error.rs:44-52) + Io */
  ORC_ERR_NONE = 0,
  ORC_ERR_INVALID_METADATA_SIZE = 1,
  ORC_ERR_INVALID_INDEX_BLOCK_OFFSET = 2,
  ORC_ERR_INVALID_INDEX_LENGTH = 3,
  ORC_ERR_INVALID_FORMAT_VERSION = 4,
  ORC_ERR_INVALID_COMPRESSION_ALGORITHM = 5,
  ORC_ERR_INVALID_BLOCK = 6,
  ORC_ERR_IO = 7
};
typedef struct {
  int32_t end;       /* ORC_END_*   */
  int32_t err;       /* ORC_ERR_*   */
  uint64_t nrec;
  uint8_t* keys;     /* malloc'd; free with oracle_scan_free */
  uint8_t* vals;
  uint64_t* key_end; /* absolute end offsets into keys/vals */
  uint64_t* val_end;
  uint64_t meta[9];  /* metadata fields in footer order (src/metadata.rs:27-59) */
  int32_t version;   /* 0 = V1, 1 = V2 */
} oracle_scan_result;
/* mode 0 = into_iter; 1 = get(key); 2 = iter_prefix(key); 3 = iter_range(key, key2); 4 = iter_from(key) */
int32_t oracle_file_scan(const uint8_t* data, uint64_t len, int32_t verify_checksums, int32_t mode,
                         const uint8_t* key, uint64_t klen, const uint8_t* key2, uint64_t klen2,
                         uint64_t max_records, oracle_scan_result* res);
/* ReaderIntoIter driven by a script (src/reader.rs:219-405 incl. seek :302-335): built like
 * file_scan's mode, then ops[i] >= 0 = up to ops[i] next() calls, ops[i] = -1 - j = seek(op key j)
 * (op keys concatenated, op_key_end = END offsets).  op_res[2i] = records the op yielded,
 * op_res[2i+1] = 0 / 1 None / 2 Err (res->err).  Records of all ops in res, in order. */
int32_t oracle_iter_script(const uint8_t* data, uint64_t len, int32_t verify, int32_t mode, const uint8_t* key,
                           uint64_t klen, const uint8_t* key2, uint64_t klen2, const int64_t* ops, uint64_t nops,
                           const uint8_t* op_keys, const uint64_t* op_key_end, int64_t* op_res,
                           oracle_scan_result* res);
void oracle_scan_free(oracle_scan_result* res);

/* Full-size parity checker (tests/test_cfg3_oracle_gpu.py): device-encoded framed blocks of
 * independent Writers (shards) against the oracle Writer shard by shard, and every block's decode
 * against the input records.  res[6] = {equal blocks, blocks, equal records, records, first bad
 * block (UINT64_MAX if none), shards that do not line up}.  See mtbl_oracle.c. */
int32_t oracle_check_writer_blocks(const uint8_t* file, uint64_t file_len, const uint64_t* blk_off,
                                   const uint32_t* blk_len, uint64_t nblk, const int64_t* blk_rec,
                                   const uint8_t* keys, const uint64_t* key_end, const uint8_t* vals,
                                   const uint64_t* val_end, const int64_t* shard_rec, uint64_t nshard,
                                   uint64_t block_size, uint64_t interval, int nthreads, uint64_t* res);

/* zlib / zstd block decompression (src/compression.rs:85-92, :140-145): 0 ok, *out malloc'd */
int32_t oracle_zlib_decompress(const uint8_t* s, uint64_t n, uint8_t** out, uint64_t* out_len);
int32_t oracle_zstd_decompress(const uint8_t* s, uint64_t n, uint8_t** out, uint64_t* out_len);

#ifdef __cplusplus
}
#endif
#endif
