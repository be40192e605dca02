/*
 * mtblx.h — C ABI of the MI355X-native mtbl block codec (libmtblx.so).
 *
 * Drop-in boundary for Kerollmops/oxidized-mtbl's block decode seam:
 *   Reader::block -> Block::init -> BlockIter::{init, seek_to_first, next, get}
 *   (reference src/reader.rs:140-186, src/block.rs:16-49, :75-93, :119-143, :145-213,
 *    driven per record by ReaderIntoIter::next src/reader.rs:337-405).
 * The reference exposes no FFI of its own (Block/BlockIter are crate-private,
 * src/lib.rs:32-33); these entry points are what a Rust `extern "C"` shim would bind
 * to replace that seam with one batched device call (INTEGRATION.md shows the binding).
 *
 * Conventions
 *  - plain pointers + sizes only; no HIP or torch types (streams are `void*`,
 *    i.e. a hipStream_t, NULL = the null stream).
 *  - "device" = memory the kernels read/write (hipMalloc'd or host-pinned mapped).
 *  - the library never allocates on a hot call: the caller passes every buffer,
 *    including the workspace sized by mtblx_decode_workspace_bytes().
 *  - the workspace carries state from call to call (a launch counter and the per-tile
 *    look-back words of both launch parities), so a call needs no fill: ZERO-FILL IT ONCE
 *    after allocating it, then reuse it for any sequence of batches of at most the
 *    nblk it was sized for.  One workspace serves one call at a time (per stream).
 *  - calls are asynchronous on `stream` and re-entrant: the library keeps no mutable state
 *    between calls -- every scratch buffer is the caller's (the block cut's too, since ABI v3);
 *    the one process-wide datum is a per-device cache of what the hardware is (compute-unit
 *    counts, kernel occupancy: csrc/devinfo.h), filled on first use with relaxed atomics.
 *  - return value: MTBLX_OK or a negative MTBLX_E_* (argument / HIP launch errors).
 *    Per-block outcomes are reported in `status[]` (MTBLX_ST_*), never by aborting.
 */
#ifndef MTBLX_H
#define MTBLX_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MTBLX_ABI_VERSION 3   /* 3: the block cut takes a caller-owned workspace (round 6) */

/* ---- API return codes ---- */
#define MTBLX_OK 0
#define MTBLX_E_INVAL (-1)    /* bad argument (NULL pointer, workspace too small, ...) */
#define MTBLX_E_HIP (-2)      /* a HIP runtime call failed                              */
#define MTBLX_E_NODEV (-3)    /* no gfx950 device visible                               */
#define MTBLX_E_FORMAT (-4)   /* host-side file/format error (reader API)               */
#define MTBLX_E_TIMEOUT (-5)  /* a decode launch reported a look-back timeout (totals[3] bit 1) twice:
                                 its outputs were discarded (synchronous entry points only).
                                 Worst case: a waiting wave gives up after 20 s (look-back) or
                                 21 s (hand-off inside a workgroup); with the one retry a stuck
                                 launch returns this after about 42-45 s                      */
#define MTBLX_E_IO (-6)       /* the writer's compressor returned Err (Writer::insert / into_inner's
                                 io::Error: Lz4 / Lz4hc "unsupported", src/compression.rs:70-81;
                                 a codec failure); nothing was written, but the records of the
                                 block being flushed are lost and the next insert fails (the
                                 reference's BlockBuilder::finish already ran, :85-104)       */

/* ---- per-block status (status[b]) ----
 * Exact correspondence with the reference's behaviour on the same bytes:         */
#define MTBLX_ST_OK 0            /* decoded; identical records to src/block.rs    */
#define MTBLX_ST_INVALID_BLOCK 1 /* Block::init returns None -> MtblError::InvalidBlock (src/block.rs:16-49) */
#define MTBLX_ST_CORRUPT 2       /* the reference panics (assert/unwrap/slice, src/block.rs:59,79,131-135,217-235);
                                    nrec[b] = records the reference yielded before the panic          */
#define MTBLX_ST_LOOP 3          /* zero-progress entry: the reference yields it forever; emitted once */
#define MTBLX_ST_UNSUPPORTED 4   /* block >= 4 GiB (u64 restart arrays): not decoded by this batched
                                    call (u32 lengths); mtblx_block_seek_batch decodes such blocks    */
#define MTBLX_ST_OVERFLOW 5      /* caller's key/value/record capacity exceeded; block not written    */
#define MTBLX_ST_DECOMPRESS 6    /* (mtblx_pipe_decode) host decompression failed: Reader::block returns
                                    Err(Error::Io) (src/reader.rs:166, src/compression.rs:57-68)      */

/* A batch of uncompressed block contents already resident on the device.
 * Block b occupies data[blk_off[b] .. blk_off[b] + blk_len[b]). */
typedef struct mtblx_block_batch {
  const uint8_t* data;      /* device */
  uint64_t data_len;        /* bytes readable at `data` (bounds for staging loads) */
  const uint64_t* blk_off;  /* device [nblk] */
  const uint32_t* blk_len;  /* device [nblk] */
  uint32_t nblk;
  uint32_t max_blk_len;     /* host hint: max of blk_len (selects the kernel variant); 0 = unknown */
} mtblx_block_batch;

/* Output layout (the north star's "keys and values laid out contiguously"):
 *   records of block b are global records rec_base[b] .. rec_base[b] + nrec[b]
 *   key of record i of block b  = keys[key_base[b] + (i ? key_end[r-1] : 0) .. key_base[b] + key_end[r]]
 *   value                        = vals[val_base[b] + (i ? val_end[r-1] : 0) .. val_base[b] + val_end[r]]
 *   with r = rec_base[b] + i; key_end/val_end are u32 END offsets relative to the block's base.
 * Records keep the reference's order within and across blocks. */
typedef struct mtblx_decoded {
  uint32_t* nrec;       /* device [nblk] */
  uint64_t* rec_base;   /* device [nblk] exclusive prefix of nrec            */
  uint64_t* key_base;   /* device [nblk] exclusive prefix of key bytes       */
  uint64_t* val_base;   /* device [nblk] exclusive prefix of value bytes     */
  int32_t* status;      /* device [nblk] MTBLX_ST_*                          */
  uint32_t* key_end;    /* device [rec_cap] */
  uint32_t* val_end;    /* device [rec_cap] */
  uint64_t rec_cap;
  uint8_t* keys;        /* device [keys_cap] */
  uint64_t keys_cap;
  uint8_t* vals;        /* device [vals_cap] */
  uint64_t vals_cap;
  uint64_t* totals;     /* device [4]: records, key bytes, value bytes, flags:
                             bit0 = some block's outputs overflowed the caller's capacity (its
                                    status is MTBLX_ST_OVERFLOW; totals[0..2] are still exact)
                             bit1 = LOOK-BACK TIMEOUT: NOTHING this launch wrote may be used.
                           The decode is one persistent launch whose workgroups (one per CU) hand
                           their tiles' output sizes to each other; it relies on all of them being
                           resident at once.  If another kernel holds CUs for long enough, a bounded
                           wait gives up and sets bit1.  Every reader surface of this library
                           (mtblx/codec.py, reader.py, include/mtbl.hpp, mtblx_pipe_decode) checks
                           it and raises / re-runs; a direct caller must check it too and re-run.
                           Env MTBLX_DEBUG_FLAGS (test knob): bits ORed into every launch's totals[3]. */
} mtblx_decoded;

/* Library identity / device check. */
int mtblx_abi_version(void);
int mtblx_device_ok(void); /* 1 if the current HIP device is gfx950, else 0 */

/* Workspace bytes needed by mtblx_decode_blocks for a batch of up to nblk blocks
 * (zero-fill once before first use, see above). */
size_t mtblx_decode_workspace_bytes(uint32_t nblk);

/* Decode every block of `in` into `out` (replaces Block::init + the BlockIter scan
 * seek_to_first/next/get of src/block.rs for each block; see header comment). */
int mtblx_decode_blocks(const mtblx_block_batch* in, const mtblx_decoded* out, void* workspace,
                        size_t workspace_bytes, void* stream);

/* Sizes only (nrec, status, bases, totals); no key/value bytes are written.
 * Lets a caller size `out` exactly before mtblx_decode_blocks. */
int mtblx_count_blocks(const mtblx_block_batch* in, const mtblx_decoded* out, void* workspace,
                       size_t workspace_bytes, void* stream);

/* Second half of a count/decode split (count to size the outputs, then write).  The
 * kernel is single-pass (counting fused into the decode), so this is the same work as
 * mtblx_decode_blocks; kept so callers written against the split stay valid. */
int mtblx_decode_counted(const mtblx_block_batch* in, const mtblx_decoded* out, void* workspace,
                         size_t workspace_bytes, void* stream);

/* CRC-32C (Castagnoli, crate crc32c 0.4) of every block's content bytes: crc[b] (device
 * [nblk]).  This is the checksum Reader::block verifies before decoding a block
 * (src/reader.rs:159-164, on by default, ReaderBuilder::verify_checksums src/reader.rs:22).
 * With framed != 0 the batch addresses contents inside an mtbl file, whose framing stores
 * the checksum as the u32 LE right before each content (varint len | crc32c | content,
 * src/writer.rs:213-225): bad[b] = 1 where it differs from crc[b] -- exactly where the
 * reference's assert_eq panics -- else 0.  crc or bad may be NULL (not both).
 * Kernel: k_crc32c_mfma (CRC-32C as fp4 / f16 matrix-core GEMMs over 1 KiB steps, one
 * persistent 16-wave workgroup per CU); MTBLX_CRC_KERNEL=lanes in the environment selects the
 * VALU table kernel k_crc32c_blocks (A/B only).  Same checksums either way. */
int mtblx_crc32c_blocks(const mtblx_block_batch* in, uint32_t* crc, uint8_t* bad, int framed, void* stream);

/* mtblx_decode_blocks + the checksum of every block (f1): crc / crc_bad as
 * mtblx_crc32c_blocks (either may be NULL, not both; `framed` bit 0 as there).  The records
 * are decoded regardless -- the caller applies Reader::block's order (checksum assert before
 * Block::init, src/reader.rs:159-172).
 * Default: the decode launch, then the matrix-core CRC kernel (k_crc32c_mfma, as
 * mtblx_crc32c_blocks) on the same stream.  With
 * MTBLX_VERIFY_FUSED in `framed` the checksum is computed inside the decode launch from the
 * tiles already staged in LDS (by the look-back and loader waves); blocks above ~64 KiB
 * still take a second launch.  On gfx950 the fused form measures slower (DESIGN.md §4:
 * table-driven CRC-32C needs one LDS lookup per byte, more than the decode leaves spare). */
#define MTBLX_VERIFY_FUSED 2
int mtblx_decode_blocks_verify(const mtblx_block_batch* in, const mtblx_decoded* out, uint32_t* crc, uint8_t* crc_bad,
                               int framed, void* workspace, size_t workspace_bytes, void* stream);

/* ---- index block -> data-block directory (f3) ----
 * The index block is decoded with mtblx_decode_blocks like any block; its values are the
 * varint64 file offsets of the data blocks.  For every index entry i this does what
 * block_at_index + the framing part of Reader::block do (src/reader.rs:177-186, :139-157):
 * varint_decode64 of the value, then (FormatV1 u32 | FormatV2 varint64) content length,
 * and the content window [blk_off[i], blk_off[i] + blk_len[i]) of the file.
 * vals/val_end/val_base: the decoded index block (values blob, its block-relative value end
 * offsets, and its val_base); file: the whole mtbl file on the device.  version: 0 = V1,
 * 1 = V2 (mtblx_footer.version).  dir_st[i]: */
#define MTBLX_DIR_OK 0          /* framed; checksum and Block::init are checked by
                                   mtblx_crc32c_blocks (framed) and mtblx_decode_blocks */
#define MTBLX_DIR_PANIC 1       /* the reference panics: offset >= file length, varint on an
                                   empty value, content slice past the end of the file   */
#define MTBLX_DIR_UNSUPPORTED 2 /* content >= 4 GiB: blk_off = the content start, blk_len 0 (a batch
                                   cannot carry it); decode it with mtblx_block_seek_batch, first=1 */
int mtblx_block_dir(const uint8_t* file, uint64_t file_len, uint32_t version, const uint8_t* vals,
                    const uint32_t* val_end, uint64_t val_base, uint32_t nent, uint64_t* blk_off,
                    uint32_t* blk_len, int32_t* dir_st, void* stream);

/* ---- batched point lookups (f2) ----
 * Reader::get (src/reader.rs:111-122) for nq keys at once: index_iter.seek(key) ->
 * block_at_index -> BlockIter::seek(key) -> the first record if its key equals `key`
 * (the next index entry's first record when the seek runs past the block), with the
 * reference's exact BlockIter::seek (src/block.rs:154-194) on the raw index and data blocks.
 * Quirk kept: when the seek runs past the block and the NEXT block fails Block::init
 * (InvalidBlock), Reader::get returns the value of the last entry the seek parsed in the old
 * block (FOUND with that value), or None if it parsed none -- not an error.
 * file: the whole mtbl file on the device; index_off/index_len: the index block content
 * (host-side framing, mtblx_frame_block); verify: check each data block's crc32c as
 * Reader::block does.  keys[key_end[q-1] .. key_end[q]) = query q (device).
 * Per query: status[q], and for FOUND the value at file[val_off[q] .. + val_len[q]). */
#define MTBLX_GET_FOUND 0
#define MTBLX_GET_NONE 1    /* Ok(None)                                      */
#define MTBLX_GET_PANIC 2   /* the reference panics                          */
#define MTBLX_GET_ERR 3     /* Err(InvalidBlock)                             */
#define MTBLX_GET_LOOP 4    /* the reference never returns (zero-progress entry) */
#define MTBLX_GET_MISSING 5 /* mtblx_get_decompressed only: the lookup reached a stored block the
                               caller's table does not hold; val_off / val_len = its stored content
                               (framing valid, checksum verified when verify).  Decompress it, add
                               it to the table and run the query again. */
int mtblx_get(const uint8_t* file, uint64_t file_len, uint32_t version, int verify, uint64_t index_off,
              uint64_t index_len, const uint8_t* keys, const uint64_t* key_end, uint32_t nq, int32_t* status,
              uint64_t* val_off, uint64_t* val_len, void* stream);

/* The same for a compressed file (Snappy / Zlib / Zstd: the crate's decompress step of
 * Reader::block, src/reader.rs:166-170).  Framing and the checksum stay on the stored bytes in
 * `file`; the blocks are scanned in their decompressed form, which the caller provides (the
 * host codecs, mtblx_decompress_blocks, or the device snappy): a table of ntab blocks sorted by
 * tab_start = the file offset of the stored content (Reader::block's raw_start), whose content
 * is dec[tab_doff[i] .. + tab_dlen[i]) when tab_st[i] == 0, and Err(Io) otherwise (the
 * crate's decompress error; reported like Err(InvalidBlock)).  A stored block missing from the
 * table is reported as MTBLX_GET_MISSING with its stored extent: a corrupt index read with
 * verification off can land a seek on a block the caller's linear walk of the index never
 * reached (the reference reads, decompresses and scans it like any other).  val_off of FOUND is
 * an offset into `dec`. */
int mtblx_get_decompressed(const uint8_t* file, uint64_t file_len, uint32_t version, int verify,
                           uint64_t index_off, uint64_t index_len, const uint64_t* tab_start,
                           const uint64_t* tab_doff, const uint64_t* tab_dlen, const int32_t* tab_st, uint32_t ntab,
                           const uint8_t* dec, const uint8_t* keys, const uint64_t* key_end, uint32_t nq,
                           int32_t* status, uint64_t* val_off, uint64_t* val_len, void* stream);

/* ---- seek-based iteration (ReaderIntoIter::new_from / seek, src/reader.rs:256-335) ----
 * Three device primitives; the host drives the iterator state (block_offset quirk, first /
 * valid, index position) exactly as src/reader.rs:219-405 does, and decodes the blocks after
 * the sought one with mtblx_decode_blocks -- only the blocks the iteration touches.
 *
 * (1) index_iter.seek(key) + the landed entry's block_at_index / Reader::block
 *     (src/block.rs:154-194, src/reader.rs:139-186), one wave per query, starting from a fresh
 *     index iterator.  ReaderIntoIter::seek re-seeks its LIVE index iterator (:303); from a
 *     regular index block (mtblx_entry_offsets) every start lands on the same entry, so the
 *     drivers use this primitive there, and otherwise seek the index block itself with
 *     mtblx_block_seek_batch from the live iterator's state and key capacity
 *     (mtblx/iterator.py, include/mtbl.hpp ReaderIntoIter).  All fields are outputs. */
#define MTBLX_SEEK_OK 0
#define MTBLX_SEEK_ERR 1          /* Err(InvalidBlock) from Block::init                       */
#define MTBLX_SEEK_PANIC 2        /* the reference panics                                     */
#define MTBLX_SEEK_LOOP 3         /* the reference never returns (zero-progress entry)        */
#define MTBLX_SEEK_UNSUPPORTED 4  /* a key > 64 KiB in mtblx_block_seek_batch's LDS key (retry with
                                     mtblx_block_seek_batch_kbuf); blocks >= 4 GiB with u64
                                     restart arrays are handled: src/block.rs:25-42, :95-104    */
typedef struct mtblx_index_seek {
  int32_t status;          /* of the index seek: OK / PANIC / LOOP                               */
  int32_t valid;           /* index_iter.get() is Some after the seek                             */
  uint64_t entry;          /* the index iterator's current entry offset in the index block        */
  uint64_t block_off;      /* varint_decode64(entry value): the file offset ReaderIntoIter keeps  */
  int32_t block_status;    /* Reader::block(block_off): OK / ERR / PANIC (UNSUPPORTED >= 4 GiB);
                              ERR / UNSUPPORTED come from Block::init on the stored bytes, which
                              is only meaningful for uncompressed files                        */
  int32_t pad;
  uint64_t data_off, data_len;   /* the block content (framed; crc32c checked when verify)       */
} mtblx_index_seek;
int mtblx_index_seek_batch(const uint8_t* file, uint64_t file_len, uint32_t version, int verify,
                           uint64_t index_off, uint64_t index_len, const uint8_t* keys, const uint64_t* key_end,
                           uint32_t nq, mtblx_index_seek* out, void* stream);

/* (2) BlockIter::seek(key) (or seek_to_first) on one block content, then the records the
 *     iterator yields from there (get / next until get() is None), keys materialised.  One
 *     workgroup per query.  kcap = the iterator's key Vec capacity (src/block.rs:132 asserts
 *     on it): 0 for a fresh BlockIter::init, or a re-seeked iterator's.  Query q writes its
 *     records to out_keys + q*keys_cap, out_vals + q*vals_cap, and END offsets (relative to
 *     the query's base) to key_end_out/val_end_out + q*rec_cap, plus the iterator's key
 *     capacity at each record to kcap_out + q*rec_cap (may be NULL).  On OVERFLOW the counts
 *     are what is needed.  keys: the seek targets (ignored for first). */
#define MTBLX_EMIT_END 0        /* get() returned None: the block is exhausted                 */
#define MTBLX_EMIT_PANIC 1      /* next() / get() panics after the emitted records             */
#define MTBLX_EMIT_LOOP 2       /* next() never returns after the emitted records              */
#define MTBLX_EMIT_MAX 3        /* max_records emitted                                         */
#define MTBLX_EMIT_OVERFLOW 4   /* a capacity was too small (counts = needed)                  */
typedef struct mtblx_block_seek {
  uint64_t data_off, data_len;   /* in: block content in `data`                                  */
  uint64_t kcap;                 /* in: key capacity (0 = fresh); out: after the emitted records  */
  uint64_t max_records;          /* in                                                            */
  int32_t first;                 /* in: 0 = seek(key); 1 = seek_to_first; 2 = resume: the iterator
                                    holds key = keys[q] (its current key bytes) and kcap, and its
                                    next() parses the entry at resume_off (BlockIter::next,
                                    src/block.rs:196-202) -- the records from there are emitted  */
  int32_t status;                /* out: MTBLX_SEEK_* of Block::init / BlockIter::init / the seek */
  int32_t end;                   /* out: MTBLX_EMIT_*                                             */
  int32_t has_val;               /* out: an entry was parsed (BlockIter::val is Some)             */
  uint64_t entry;                /* out: the iterator's current entry offset after the seek       */
  uint64_t nrec, key_bytes, val_bytes;   /* out                                                   */
  uint64_t last_voff, last_vlen; /* out: `val` of the last parsed entry (content offsets) -- what
                                    Reader::get returns when next() hits Err (src/reader.rs:111-122) */
  uint64_t resume_off;           /* in (first == 2): offset of the entry next() parses            */
  uint64_t stop_off;             /* out: the iterator's current entry offset when the emission
                                    stopped; after MTBLX_EMIT_MAX: the entry after the last
                                    emitted record (resume there with that record's key / kcap) */
  int32_t early;                 /* out (first == 0): the binary search returned early on a restart
                                    entry with shared != 0 (src/block.rs:167-170): a live iterator
                                    keeps its previous position; nothing after it applies       */
  int32_t pad;
} mtblx_block_seek;
int mtblx_block_seek_batch(const uint8_t* data, const uint8_t* keys, const uint64_t* key_end, uint32_t nq,
                           mtblx_block_seek* q, uint8_t* out_keys, uint64_t keys_cap, uint8_t* out_vals,
                           uint64_t vals_cap, uint64_t* key_end_out, uint64_t* val_end_out, uint64_t* kcap_out,
                           uint64_t rec_cap, void* stream);
/* (2') the same with the iterator's key kept in a caller buffer, key_buf + q * key_buf_cap
 *      (device), instead of 64 KiB of LDS: keys of any length.  mtblx_block_seek_batch reports a
 *      key past 64 KiB as status MTBLX_SEEK_UNSUPPORTED; here that means past key_buf_cap.  A
 *      key never exceeds len(keys[q]) + data_len bytes (every byte after the target's comes from
 *      a distinct suffix in the block), so that capacity always suffices. */
int mtblx_block_seek_batch_kbuf(const uint8_t* data, const uint8_t* keys, const uint64_t* key_end, uint32_t nq,
                                mtblx_block_seek* q, uint8_t* out_keys, uint64_t keys_cap, uint8_t* out_vals,
                                uint64_t vals_cap, uint64_t* key_end_out, uint64_t* val_end_out, uint64_t* kcap_out,
                                uint64_t rec_cap, uint8_t* key_buf, uint64_t key_buf_cap, void* stream);
/* (2'') the same with the value bytes left to the caller (blocks >= 4 GiB hold values of GiBs):
 *      record r of query q gets val_end_out as above and val_src_out[q * rec_cap + r] = its value's
 *      offset in the block content; out_vals is not written (may be NULL) and vals_cap only sizes
 *      the emission.  The caller then moves the bytes with mtblx_copy_ranges (the whole grid).
 *      key_buf == NULL: the key in LDS as mtblx_block_seek_batch; else as _kbuf. */
int mtblx_block_seek_batch_ex(const uint8_t* data, const uint8_t* keys, const uint64_t* key_end, uint32_t nq,
                              mtblx_block_seek* q, uint8_t* out_keys, uint64_t keys_cap, uint8_t* out_vals,
                              uint64_t vals_cap, uint64_t* key_end_out, uint64_t* val_end_out, uint64_t* kcap_out,
                              uint64_t rec_cap, uint8_t* key_buf, uint64_t key_buf_cap, uint64_t* val_src_out,
                              void* stream);

/* (3) the offsets of the entries seek_to_first + next visit in a block (the index block: entry
 *     i <-> index record i <-> directory entry i), so a seek's landed entry maps to its index
 *     position.  Parallel over restart intervals when every interval's chain lands on the next
 *     restart point; otherwise one serial walk.  Writes min(count, cap) offsets; *count (device)
 *     = entries up to the end of the block or the first entry the scan cannot decode.
 *     *regular (device u32, may be NULL) = 1 when every interval's chain lands on the next
 *     restart point, every restart entry has shared == 0 and every other entry shared <= the
 *     previous key's length.  For such an index block a seek from ANY iterator state (fresh or
 *     live, any key capacity) never returns early, lands on the scan chain, rebuilds the scan's
 *     keys and cannot hit the key-capacity assert: the host may then follow the directory
 *     (entries i+1, i+2, ...) after a seek.  Otherwise the host drives the live index iterator
 *     with mtblx_block_seek_batch (seek / resume) over the index block.  Synchronous: returns
 *     after the launch completed (its scratch is freed then). */
int mtblx_entry_offsets(const uint8_t* block, uint64_t len, uint64_t* offs, uint64_t cap, uint64_t* count,
                        uint32_t* regular, void* stream);

/* (4) ReaderIntoIter's stop rules (src/reader.rs:385-402) over decoded records: the index of
 *     the first record whose key fails (type 1 Get: != k, 2 GetPrefix: !starts_with(k), 3
 *     GetRange: > k), or n.  key_end: absolute END offsets (int64).  *first_fail (device) is
 *     min-reduced: set it to n before the call. */
int mtblx_key_filter(const uint8_t* keys, const uint64_t* key_end, uint64_t n, int32_t type, const uint8_t* k,
                     uint64_t klen, uint64_t* first_fail, void* stream);

/* ---- encode side on the device: Writer's block cut + BlockBuilder + write_block framing ----
 * Records (device): key r = keys[r ? key_end[r-1] : 0 .. key_end[r]), value likewise (u64 END
 * offsets from record 0), in Writer::insert order (strictly increasing keys). */
typedef struct mtblx_records {
  const uint8_t* keys;
  const uint64_t* key_end;
  const uint8_t* vals;
  const uint64_t* val_end;
  uint64_t n;
} mtblx_records;

/* Writer::insert's flush rule (src/writer.rs:125-130 with BlockBuilder::current_size_estimate,
 * src/block_builder.rs:40-47): where the Writer would cut blocks.  Each shard s = records
 * [shard_rec[s], shard_rec[s+1]) (device) is an independent Writer (one file each; one shard
 * = one file); blocks of all shards are numbered consecutively: block b = records
 * [blk_rec[b], blk_rec[b+1]) (device, capacity blk_cap >= nblk + 1; blk_rec may be NULL to
 * count only).  block_size is clamped to >= 1024 like WriterBuilder::block_size.
 * Synchronous; *nblk_out = number of blocks.  Returns MTBLX_E_FORMAT where the Writer
 * panics; *flags_out tells why: */
#define MTBLX_PLAN_OUT_OF_ORDER 1u /* a key <= its predecessor: panic!("out-of-order key") (:119-123) */
#define MTBLX_PLAN_PANIC 2u        /* restart_interval 0 and a second entry: assert (src/block_builder.rs:50) */
#define MTBLX_PLAN_TOO_LONG 4u     /* a key or value >= 4 GiB (u32 varint lengths)                    */
/* Scratch (device, 256-byte aligned, no fill needed) of the parallel cut for up to `nrec` records in
 * `nshard` shards at this interval; keep != 0 for mtblx_encode_plan_keep (whose entry sizes live in
 * the plan buffer).  A bound that holds for any record sizes, ~50 B per record.  The library keeps
 * no scratch between calls: one workspace serves one call at a time. */
size_t mtblx_plan_workspace_bytes(uint64_t nrec, uint32_t nshard, uint32_t restart_interval, int keep);
/* The serial walk's scratch (one wave per shard, the round-1..4 cut): 16 B per shard. */
size_t mtblx_plan_serial_workspace_bytes(uint32_t nshard);
/* workspace: at least mtblx_plan_workspace_bytes(records of the shards, nshard, restart_interval, 0)
 * runs the parallel cut (every record's next block start at once + pointer doubling); a smaller one,
 * of at least mtblx_plan_serial_workspace_bytes(nshard), the serial walk (same cut; also taken for
 * record ranges of 2^32 - 16 or more and under MTBLX_PLAN=serial).  NULL or misaligned: MTBLX_E_INVAL. */
int mtblx_encode_plan(const mtblx_records* rec, const uint64_t* shard_rec, uint32_t nshard, uint64_t block_size,
                      uint32_t restart_interval, uint64_t* blk_rec, uint64_t blk_cap, uint64_t* nblk_out,
                      uint32_t* flags_out, void* workspace, size_t ws_bytes, void* stream);

/* The same block cut, keeping what the encode needs (round 5): `plan` (device, 256-byte aligned,
 * mtblx_plan_keep_bytes(number of records in the shards) bytes) receives every record's entry size
 * summed in order, the bytes a restart entry loses by not sharing summed along residue classes
 * mod restart_interval, and every record's shared-prefix length with its predecessor (across shard
 * starts too).  restart_interval must be >= 1, the shards must hold fewer than 2^32 - 16 records and
 * the workspace at least mtblx_plan_workspace_bytes(..., keep = 1): otherwise MTBLX_E_INVAL (no
 * serial fallback: cut with mtblx_encode_plan and encode with mtblx_encode_blocks instead).
 * Returns like mtblx_encode_plan. */
size_t mtblx_plan_keep_bytes(uint64_t nrec);
/* ABI v2 compatibility: a no-op (the cut used to cache its scratch; it keeps none now). */
void mtblx_plan_release(void);
int mtblx_encode_plan_keep(const mtblx_records* rec, const uint64_t* shard_rec, uint32_t nshard, uint64_t block_size,
                           uint32_t restart_interval, uint64_t* blk_rec, uint64_t blk_cap, uint64_t* nblk_out,
                           uint32_t* flags_out, void* plan, size_t plan_bytes, void* workspace, size_t ws_bytes,
                           void* stream);

/* BlockBuilder::add for every record of a block, then finish (src/block_builder.rs:49-104),
 * for every block b of blk_rec at once.  framed != 0 adds write_block's framing before each
 * content (varint64 len | crc32c | content, src/writer.rs:203-237, CompressionType::None):
 * the blocks then sit back to back from out[0], byte-identical to the data-block region of
 * the file Writer produces.  blk_off[b]/blk_len[b] = content window in `out` (the decode
 * batch directory); status[b] = MTBLX_ST_OK, _CORRUPT (BlockBuilder assert), _UNSUPPORTED
 * (>= 4 GiB), _OVERFLOW (out_cap); totals (device [2]) = bytes written, flags (bit 0: a
 * block not OK, bit 1: look-back timeout).  Asynchronous on `stream`; the workspace
 * (mtblx_encode_workspace_bytes) is cleared by the call. */
size_t mtblx_encode_workspace_bytes(uint32_t nblk);
int mtblx_encode_blocks(const mtblx_records* rec, const uint64_t* blk_rec, uint32_t nblk, uint32_t restart_interval,
                        int framed, uint8_t* out, uint64_t out_cap, uint64_t* blk_off, uint32_t* blk_len,
                        int32_t* status, uint64_t* totals, void* workspace, size_t ws_bytes, void* stream);
/* mtblx_encode_blocks reading a kept plan (mtblx_encode_plan_keep over the same records and
 * restart_interval; blk_rec may be any cut of records inside it): every block's length and file
 * offset come from the kept sums and one scan, so no block waits on its predecessors, and no
 * entry's shared prefix is recomputed.  Output identical to mtblx_encode_blocks.  Asynchronous
 * after one small synchronous read of the plan's header. */
int mtblx_encode_blocks_planned(const mtblx_records* rec, const uint64_t* blk_rec, uint32_t nblk,
                                uint32_t restart_interval, int framed, uint8_t* out, uint64_t out_cap,
                                uint64_t* blk_off, uint32_t* blk_len, int32_t* status, uint64_t* totals,
                                void* workspace, size_t ws_bytes, const void* plan, void* stream);

/* Writer::into_inner's tail on the device (src/writer.rs:132-138, :155-181, :239-265;
 * src/metadata.rs:61-79) for ONE file whose data blocks mtblx_encode_blocks wrote framed:
 * data[region_off .. region_off + data_bytes) holds them back to back; blk_off/blk_len (device
 * [nblk], offsets relative to `data`) and blk_rec (device [nblk + 1], absolute record indices
 * into rec) are that call's directory and plan for this file.  Writes the whole file to
 * `file` (device; the data region is copied unless file == data + region_off): the data
 * blocks, then the index block -- one entry per data block, key = bytes_shortest_separator(
 * its last key, the next block's first key) with the crate's write_u16 APPEND quirk (the
 * last block's entry keeps the file's last key), value = varint64(the block's file offset)
 * -- built by BlockBuilder with `restart_interval` and framed with CompressionType::None,
 * then the 512-byte footer (block_size clamped to >= 1024 as WriterBuilder::block_size).
 * nblk == 0 writes the empty file.  Synchronous (allocates its temporaries: once per file);
 * *file_len = bytes written.  Byte-identical to the crate's Writer for the same records. */
int mtblx_encode_index(const mtblx_records* rec, const uint64_t* blk_rec, uint32_t nblk, uint64_t block_size,
                       uint32_t restart_interval, const uint8_t* data, uint64_t region_off, uint64_t data_bytes,
                       const uint64_t* blk_off, const uint32_t* blk_len, uint8_t* file, uint64_t file_cap,
                       uint64_t* file_len, void* stream);

/* ---- snappy raw decompression on the device (f4) ----
 * Reader::block's decompression step for CompressionType::Snappy (src/reader.rs:166-170 ->
 * src/compression.rs:57-68, :116-119, snap::raw::Decoder::decompress_vec), for a batch of
 * blocks at once.  Block b's STORED bytes are src[src_off[b] .. + src_len[b]) (device).
 * Status codes are mtblx_host.h's MTBLX_SNAPPY_*: OK, CORRUPT (snap errors -> Err(Error::Io)),
 * TOO_SMALL (the preamble length exceeds dst_len[b]).
 *
 * mtblx_snappy_dir: the output layout from the preambles: dst_len[b] = the stored
 * uncompressed length (0 if the preamble is corrupt, status[b] = CORRUPT), dst_off[b] = the
 * exclusive prefix of dst_len rounded up to 16 bytes; totals (device [3]) = bytes of the
 * layout, max dst_len, corrupt preambles.  workspace: mtblx_snappy_workspace_bytes(nblk)
 * bytes of device memory (no fill needed).
 *
 * mtblx_snappy_decompress_dev: decompresses block b into dst[dst_off[b] .. + its length)
 * (dst_len[b] = capacity); status[b]; dec_len[b] (device [nblk], may be NULL) = the
 * decompressed length, or 0 if the block failed -- i.e. {dst, dst_off, dec_len} is directly
 * the mtblx_block_batch directory of the decompressed blocks.  max_dst_len: host hint (max
 * of dst_len; 0 = unknown) selecting the kernel variant; the environment variable
 * MTBLX_SNAPPY_KERNEL (read per call: auto | quads | lanes | two) forces one for A/B runs and
 * tests, with identical outputs and statuses.  Both calls are asynchronous on `stream`. */
size_t mtblx_snappy_workspace_bytes(uint32_t nblk);
int mtblx_snappy_dir(const uint8_t* src, const uint64_t* src_off, const uint32_t* src_len, uint32_t nblk,
                     uint64_t* dst_off, uint32_t* dst_len, int32_t* status, uint64_t* totals, void* workspace,
                     size_t workspace_bytes, void* stream);
int mtblx_snappy_decompress_dev(const uint8_t* src, const uint64_t* src_off, const uint32_t* src_len, uint32_t nblk,
                                uint8_t* dst, const uint64_t* dst_off, const uint32_t* dst_len, uint32_t max_dst_len,
                                int32_t* status, uint32_t* dec_len, void* stream);

/* ---- end-to-end decode from host memory (the PCIe-inclusive path of the north star) ----
 * An mtbl file in host memory in (mmap'd or read), the caller's host byte slices out:
 * for every data block, Reader::block's decompression (src/reader.rs:166-170, host: the
 * north star keeps src/compression.rs on the host) + Block::init + the BlockIter scan
 * (device).  Consecutive blocks are cut into chunks that flow through three stages with
 * three chunks in flight: host staging (nothing for a pinned uncompressed file; a parallel
 * copy into pinned memory for a pageable one; parallel snappy decompression), H2D +
 * mtblx_decode_blocks on the device, D2H of the chunk's outputs into `out`.
 *   file/blk_off/blk_len: host; block b's STORED content is file[blk_off[b] .. + blk_len[b])
 *   (the directory mtblx_writer_block_dir / mtblx_block_dir produce).  compression: the
 *   footer's compression_algorithm: 0 None, 1 Snappy (others: MTBLX_E_INVAL).
 *   out: mtblx_decoded whose pointers are HOST memory (pin it -- mtblx_host_alloc or
 *   mtblx_host_register -- for full PCIe rate), same layout and status codes as
 *   mtblx_decode_blocks plus MTBLX_ST_DECOMPRESS.  If a capacity is too small the outputs of
 *   the chunks that do not fit are skipped (their blocks: MTBLX_ST_OVERFLOW, totals[3] bit 0)
 *   and totals[0..2] still report the exact sizes, so a caller can size and call again.
 * Synchronous: returns when `out` is complete.  One call at a time per pipe. */
typedef struct mtblx_pipe mtblx_pipe;
typedef struct mtblx_pipe_stats {
  double seconds;          /* wall time of the call                                */
  double stage_seconds;    /* host staging (copies / decompression) on the calling path */
  double decode_ms;        /* device time of the decode launches (HIP events)     */
  uint64_t block_bytes;    /* uncompressed block content bytes decoded            */
  uint64_t h2d_bytes, d2h_bytes;
  uint32_t chunks;
  uint32_t decompress_errors;
} mtblx_pipe_stats;
/* chunk_bytes: uncompressed bytes per chunk (0 = 64 MiB); max_blocks: blocks per chunk
 * (0 = 65536); threads: host staging threads (0 = 16).  Binds to the current HIP device. */
mtblx_pipe* mtblx_pipe_new(uint64_t chunk_bytes, uint32_t max_blocks, uint32_t threads);
void mtblx_pipe_free(mtblx_pipe* p);
int mtblx_pipe_decode(mtblx_pipe* p, const uint8_t* file, uint64_t file_len, uint32_t compression,
                      const uint64_t* blk_off, const uint32_t* blk_len, uint32_t nblk, const mtblx_decoded* out,
                      mtblx_pipe_stats* stats);
/* pipe options.  MTBLX_PIPE_DEVICE_SNAPPY (value 1 = on, 0 = off, 2 = auto, the default):
 * snappy files cross PCIe as stored and are decompressed on the device
 * (mtblx_snappy_decompress_dev) right before the decode; off = host decompression in the
 * staging stage; auto = the device (measured faster end to end on poorly compressed and on
 * compressible streams alike).  Same outputs either way. */
#define MTBLX_PIPE_DEVICE_SNAPPY 1
int mtblx_pipe_set(mtblx_pipe* p, int option, int64_t value);
/* pinned host memory for the pipe's inputs / outputs */
int mtblx_host_alloc(void** p, uint64_t bytes);
int mtblx_host_free(void* p);
int mtblx_host_register(void* p, uint64_t bytes);   /* pin an existing range, e.g. an mmap'd file */
int mtblx_host_unregister(void* p);

/* ---- diagnostic: device copy at the HBM ceiling ----
 * dst[0 .. bytes) = src[0 .. bytes) (16-byte aligned, bytes % 16 == 0) by a plain gfx950
 * streaming kernel: 16 B per lane per access, 2^(variant & 3) accesses in flight per lane,
 * 8 workgroups per CU.  bench.py takes the best of a sweep as this box's copy ceiling, the
 * reference its roofline fraction is read against besides the 8 TB/s spec.  Asynchronous. */
#define MTBLX_COPY_NT_STORES 4
#define MTBLX_COPY_NT_LOADS 8
int mtblx_stream_copy(void* dst, const void* src, uint64_t bytes, int variant, void* stream);

/* n byte ranges src + src_off[i] -> dst + dst_off[i] (len[i] bytes each, device arrays) by the
 * whole grid: chunk_base[i] = the exclusive prefix of ceil(len / 16) over the ranges, nchunks its
 * total.  Asynchronous on `stream`.  Used with mtblx_block_seek_batch_ex for the values of blocks
 * >= 4 GiB (one wave would copy their GiBs at a few GB/s). */
int mtblx_copy_ranges(const uint8_t* src, const uint64_t* src_off, uint8_t* dst, const uint64_t* dst_off,
                      const uint64_t* len, const uint64_t* chunk_base, uint32_t n, uint64_t nchunks, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* MTBLX_H */
