/*
 * mtblx_host.h — host-side file layer of libmtblx.so (C ABI), around the device codec.
 *
 * Mirrors the reference's public file-level surface that sits either side of the
 * block codec:
 *   Writer::{insert, into_inner}        /root/reference/src/writer.rs:112-181
 *   write_block / shortest separator    src/writer.rs:203-265
 *   BlockBuilder (host build)           src/block_builder.rs:15-104
 *   Metadata footer                     src/metadata.rs:27-79
 *   ReaderBuilder::read framing         src/reader.rs:31-81
 *   Reader::block framing + CRC         src/reader.rs:140-164
 *   crc32c                              crate crc32c 0.4 (SSE4.2)
 * Decoding block contents is NOT done here: every block goes through
 * mtblx_decode_blocks (mtblx.h) on the device.
 *
 * Compression (src/compression.rs) stays on the host: snappy raw codec below; compressed
 * reads are host decompression feeding the same device path (mtblx_pipe_decode in mtblx.h,
 * mtblx/reader.py).
 */
#ifndef MTBLX_HOST_H
#define MTBLX_HOST_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* MtblError (src/error.rs:44-52) */
#define MTBLX_ERR_NONE 0
#define MTBLX_ERR_INVALID_METADATA_SIZE 1
#define MTBLX_ERR_INVALID_INDEX_BLOCK_OFFSET 2
#define MTBLX_ERR_INVALID_INDEX_LENGTH 3
#define MTBLX_ERR_INVALID_FORMAT_VERSION 4
#define MTBLX_ERR_INVALID_COMPRESSION_ALGORITHM 5
#define MTBLX_ERR_INVALID_BLOCK 6
#define MTBLX_ERR_IO 7

typedef struct mtblx_footer {
  uint64_t meta[9];  /* index_block_offset, data_block_size, compression_algorithm, count_entries,
                        count_data_blocks, bytes_data_blocks, bytes_index_block, bytes_keys, bytes_values */
  uint32_t version;  /* 0 = FormatV1, 1 = FormatV2 */
  int32_t err;       /* MTBLX_ERR_* when the call returns MTBLX_E_FORMAT */
} mtblx_footer;

/* crc32c of n bytes (replaces crc32c::crc32c, src/reader.rs:73,162, src/writer.rs:218) */
uint32_t mtblx_crc32c(const uint8_t* data, uint64_t n);

/* varint_decode64 (src/varint.rs:78-97): consumed length, 0 = unterminated, -1 = reference panic */
int mtblx_varint_decode64(const uint8_t* data, uint64_t len, uint64_t* out);

/* Metadata::read_from_bytes + the offset sanity check of ReaderBuilder::read (src/reader.rs:31-49) */
int mtblx_read_footer(const uint8_t* file, uint64_t len, mtblx_footer* f);

/* framing of the block at file offset `off` (src/reader.rs:140-164): content window + CRC check.
 * *panic = 1 where the reference panics (out-of-range slice, CRC assert_eq). */
int mtblx_frame_block(const uint8_t* file, uint64_t len, uint32_t version, uint64_t off, int verify,
                      uint64_t* content_off, uint64_t* content_len, int* panic);

/* ---- snappy raw codec (CompressionType::Snappy, src/compression.rs:116-130, crate snap 1.x raw) ----
 * Host-side, as the north star keeps compression on the host.  Return codes: */
#define MTBLX_SNAPPY_OK 0
#define MTBLX_SNAPPY_CORRUPT 1   /* snap::raw::Decoder error -> io::Error -> Error::Io (src/compression.rs:117-118) */
#define MTBLX_SNAPPY_TOO_SMALL 2 /* destination capacity too small */
#define MTBLX_SNAPPY_TIMEOUT 3   /* device decompression only: a bounded internal wait (2 s) gave up --
                                    not a property of the stream; the block's output is not valid */
uint64_t mtblx_snappy_max_compressed_len(uint64_t n);
/* the length stored in the preamble (no validation of the body) */
int mtblx_snappy_uncompressed_len(const uint8_t* src, uint64_t n, uint64_t* out);
/* full decompression into dst[0..cap); *out_len = the preamble length */
int mtblx_snappy_decompress(const uint8_t* src, uint64_t n, uint8_t* dst, uint64_t cap, uint64_t* out_len);
/* valid snappy of src (bytes are not pinned to the reference encoder: SURVEY.md §8c); cap >= max_compressed_len */
int mtblx_snappy_compress(const uint8_t* src, uint64_t n, uint8_t* dst, uint64_t cap, uint64_t* out_len);
/* batch: block b's stored bytes file[blk_off[b] .. + blk_len[b]) -> dst[dst_off[b] .. + dst_len[b]),
 * `threads` host threads; st[b] (may be NULL) = MTBLX_SNAPPY_*; returns the number of failed blocks */
uint64_t mtblx_snappy_decompress_blocks(const uint8_t* file, const uint64_t* blk_off, const uint32_t* blk_len,
                                        uint8_t* dst, const uint64_t* dst_off, const uint64_t* dst_len, int32_t* st,
                                        uint64_t nblk, uint32_t threads);

/* ---- host block (de)compression, every CompressionType (src/compression.rs:57-81) ----
 * compression: 0 None, 1 Snappy (the in-repo raw codec above), 2 Zlib (system zlib: the
 * zlib-wrapped stream flate2's ZlibDecoder / ZlibEncoder read and write), 5 Zstd (libzstd.so.1
 * loaded at run time: the C library the crate zstd 0.5 wraps; all frames until the input
 * ends, stream::copy_decode); 3 Lz4 / 4 Lz4hc: the crate's Err "unsupported".  A decoder
 * error is the crate's io::Error -> Error::Io (Reader::block, src/reader.rs:166).
 * Compressed BYTES are not pinned to the crate's encoders. */
#define MTBLX_CODEC_OK 0
#define MTBLX_CODEC_CORRUPT 1       /* decoder / encoder error -> Error::Io */
#define MTBLX_CODEC_UNSUPPORTED 2   /* Lz4 / Lz4hc / unknown, or libzstd.so.1 not loadable */
int mtblx_codec_available(uint32_t compression);   /* 1 if this host can (de)compress it */
/* *out malloc'd (free with mtblx_free); returns MTBLX_CODEC_* */
int mtblx_decompress(uint32_t compression, const uint8_t* src, uint64_t n, uint8_t** out, uint64_t* out_len);
int mtblx_compress(uint32_t compression, uint32_t level, const uint8_t* src, uint64_t n, uint8_t** out,
                   uint64_t* out_len);
/* batch for Reader::block's decompression step: block b's stored bytes file[blk_off[b] ..
 * + blk_len[b]) decompressed by `threads` host threads (0 = 16) into ONE malloc'd buffer *dst
 * (mtblx_free): block b at (*dst)[dst_off[b] .. + dst_len[b]) (16-byte aligned starts, length 0
 * on failure); st[b] (may be NULL) = MTBLX_CODEC_*; returns the number of failed blocks.  The
 * {*dst, dst_off, dst_len} triple is directly a decode batch directory (mtblx_block_batch). */
uint64_t mtblx_decompress_blocks(uint32_t compression, const uint8_t* file, const uint64_t* blk_off,
                                 const uint32_t* blk_len, uint64_t nblk, uint32_t threads, uint8_t** dst,
                                 uint64_t* dst_off, uint64_t* dst_len, int32_t* st);

/* Writer (src/writer.rs).  compression: 0 None, 1 Snappy, 2 Zlib, 5 Zstd: data blocks are
 * compressed with mtblx_compress (the index block never, src/writer.rs:165-173); returns NULL
 * for other values or a codec this host lacks.  mtblx_writer_set_level =
 * WriterBuilder::compression_level (default 0, src/lib.rs:8). */
typedef struct mtblx_writer mtblx_writer;
mtblx_writer* mtblx_writer_new(uint64_t block_size, uint64_t restart_interval, uint32_t compression);
int mtblx_writer_set_level(mtblx_writer* w, uint32_t level);
/* MTBLX_OK, or MTBLX_E_FORMAT where the reference panics ("out-of-order key", ...) */
int mtblx_writer_insert(mtblx_writer* w, const uint8_t* key, uint64_t klen, const uint8_t* val, uint64_t vlen);
int mtblx_writer_insert_batch(mtblx_writer* w, const uint8_t* keys, const uint64_t* key_end, const uint8_t* vals,
                              const uint64_t* val_end, uint64_t n);
/* Writer::into_inner: *out malloc'd (free with mtblx_free) */
int mtblx_writer_finish(mtblx_writer* w, uint8_t** out, uint64_t* out_len);
/* data-block directory of the finished file: content offset / length / record count per
 * data block (blk_nrec may be NULL) */
uint64_t mtblx_writer_block_count(const mtblx_writer* w);
int mtblx_writer_block_dir(const mtblx_writer* w, uint64_t* blk_off, uint32_t* blk_len, uint32_t* blk_nrec);
void mtblx_writer_free(mtblx_writer* w);
void mtblx_free(void* p);

#ifdef __cplusplus
}
#endif
#endif /* MTBLX_HOST_H */
