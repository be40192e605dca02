/*
 * mtbl_oracle.c — CPU ORACLE (test infrastructure only; see mtbl_oracle.h header).
 *
 * Plain-C restatement of Kerollmops/oxidized-mtbl.  File:line citations refer to
 * /root/reference/.  Rust release-mode semantics; panics -> ORC_ST_CORRUPT /
 * ORC_END_PANIC.  Never linked into the product.
 */
#define _GNU_SOURCE
#include "mtbl_oracle.h"

#include <pthread.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#define PANIC (-1)
#define U32MAX 0xFFFFFFFFull

static uint32_t rd32(const uint8_t* p) { return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24); }
static uint64_t rd64(const uint8_t* p) { return (uint64_t)rd32(p) | ((uint64_t)rd32(p + 4) << 32); }
static void wr32(uint8_t* p, uint32_t v) { for (int i = 0; i < 4; i++) p[i] = (uint8_t)(v >> (8 * i)); }
static void wr64(uint8_t* p, uint64_t v) { for (int i = 0; i < 8; i++) p[i] = (uint8_t)(v >> (8 * i)); }

void oracle_free(void* p) { free(p); }

/* ============================ varint: src/varint.rs ============================ */

/* src/varint.rs:1-10 — index of the first byte with bit 7 clear, +1; 0 if none */
uint32_t oracle_varint_length_packed(const uint8_t* data, uint64_t len) {
  uint64_t i = 0;
  for (uint64_t k = 0; k < len; k++) {
    if ((data[i] & 0x80) == 0) break;
    i++;
  }
  return i == len ? 0 : (uint32_t)(i + 1);
}

/* src/varint.rs:12-42 */
uint32_t oracle_varint_encode32(uint8_t* b, uint32_t v) {
  if (v < (1u << 7)) { b[0] = (uint8_t)v; return 1; }
  if (v < (1u << 14)) { b[0] = (uint8_t)(v | 128); b[1] = (uint8_t)(v >> 7); return 2; }
  if (v < (1u << 21)) { b[0] = (uint8_t)(v | 128); b[1] = (uint8_t)((v >> 7) | 128); b[2] = (uint8_t)(v >> 14); return 3; }
  if (v < (1u << 28)) {
    b[0] = (uint8_t)(v | 128); b[1] = (uint8_t)((v >> 7) | 128); b[2] = (uint8_t)((v >> 14) | 128);
    b[3] = (uint8_t)(v >> 21); return 4;
  }
  b[0] = (uint8_t)(v | 128); b[1] = (uint8_t)((v >> 7) | 128); b[2] = (uint8_t)((v >> 14) | 128);
  b[3] = (uint8_t)((v >> 21) | 128); b[4] = (uint8_t)(v >> 28); return 5;
}

/* src/varint.rs:44-61.  `data` is the slice data[p..] of the reference: len = bytes
 * available to the end of the underlying buffer.  The reference indexes data[0]
 * unconditionally, so len == 0 panics. */
int32_t oracle_varint_decode32(const uint8_t* d, uint64_t len, uint32_t* value) {
  if (len == 0) return PANIC;
  uint32_t l = oracle_varint_length_packed(d, len < 5 ? len : 5);
  uint32_t val = d[0] & 0x7f;
  if (l > 1) {
    val |= (uint32_t)(d[1] & 0x7f) << 7;
    if (l > 2) {
      val |= (uint32_t)(d[2] & 0x7f) << 14;
      if (l > 3) {
        val |= (uint32_t)(d[3] & 0x7f) << 21;
        if (l > 4) val |= (uint32_t)d[4] << 28; /* unmasked; high bits fall off (:54) */
      }
    }
  }
  *value = val;
  return (int32_t)l;
}

/* src/varint.rs:63-76 */
uint32_t oracle_varint_encode64(uint8_t* b, uint64_t v) {
  uint32_t i = 0;
  while (v >= 128) { b[i++] = (uint8_t)((v & 127) | 128); v >>= 7; }
  b[i] = (uint8_t)v;
  return i + 1;
}

/* src/varint.rs:78-97 */
int32_t oracle_varint_decode64(const uint8_t* d, uint64_t len, uint64_t* value) {
  uint32_t l = oracle_varint_length_packed(d, len < 10 ? len : 10);
  if (l < 5) {
    uint32_t t = 0;
    int32_t r = oracle_varint_decode32(d, len, &t);
    if (r < 0) return r;
    *value = t;
    return r;
  }
  uint64_t val = (uint64_t)(d[0] & 0x7f) | ((uint64_t)(d[1] & 0x7f) << 7) | ((uint64_t)(d[2] & 0x7f) << 14) |
                 ((uint64_t)(d[3] & 0x7f) << 21);
  uint32_t shift = 28;
  for (uint32_t i = 4; i < l; i++) { val |= (uint64_t)(d[i] & 0x7f) << shift; shift += 7; }
  *value = val;
  return (int32_t)l;
}

/* ============================ crc32c (crate crc32c 0.4) ============================ */
static uint32_t crc_tab[256];
static pthread_once_t crc_once = PTHREAD_ONCE_INIT;
static void crc_init(void) {
  for (uint32_t i = 0; i < 256; i++) {
    uint32_t c = i;
    for (int k = 0; k < 8; k++) c = (c & 1) ? (c >> 1) ^ 0x82F63B78u : c >> 1;
    crc_tab[i] = c;
  }
}
uint32_t oracle_crc32c(const uint8_t* d, uint64_t len) {
  pthread_once(&crc_once, crc_init);
  uint32_t c = 0xFFFFFFFFu;
  for (uint64_t i = 0; i < len; i++) c = crc_tab[(c ^ d[i]) & 0xff] ^ (c >> 8);
  return c ^ 0xFFFFFFFFu;
}

/* ============================ block decode: src/block.rs ============================ */

typedef struct {
  const uint8_t* d;
  uint64_t L;
  uint64_t restarts;      /* Block::restart_offset */
  uint32_t n;             /* num_restarts          */
  uint64_t current;
  int has_next;
  uint64_t next;
  uint8_t* key;           /* real storage (>= kcap)                       */
  uint64_t klen, kcap;    /* kcap emulates Vec<u8>::capacity() (block.rs:132) */
  uint64_t kalloc;
  int has_val;
  uint64_t voff, vlen;
  uint8_t* owned;         /* decompressed block bytes (Cow::Owned), freed with the iterator */
} oiter;

/* Block::init (src/block.rs:16-49) + num_restarts (:58-61).  0 = Some, else status */
static int oblock_init(const uint8_t* d, uint64_t L, uint64_t* ro_out) {
  if (L < 4) return ORC_ST_INVALID_BLOCK;                 /* :19-20 */
  if (L < 8) return ORC_ST_CORRUPT;                       /* num_restarts assert :59 */
  uint32_t n = rd32(d + L - 4);
  uint64_t ro = L - (1 + (uint64_t)n) * 4;                /* :22, wrapping (release) */
  if (ro > U32MAX) {                                      /* :29-42 */
    ro = L - (4 + (uint64_t)n * 8);
    if (ro <= U32MAX) return ORC_ST_INVALID_BLOCK;
  }
  if (ro > L - 4) return ORC_ST_INVALID_BLOCK;            /* :44-46 */
  *ro_out = ro;
  return ORC_ST_OK;
}

/* BlockIter::restart_point (src/block.rs:95-104); 64-bit restarts keep the 4-byte stride */
static uint64_t orestart_point(const oiter* it, uint32_t idx) {
  uint64_t off = it->restarts + (uint64_t)idx * 4;
  if (it->restarts > U32MAX) return rd64(it->d + off);
  return rd32(it->d + off);
}

/* BlockIter::init (src/block.rs:75-93) */
static int oiter_init(oiter* it, const uint8_t* d, uint64_t L, uint64_t ro) {
  memset(it, 0, sizeof(*it));
  it->d = d; it->L = L; it->restarts = ro;
  it->n = rd32(d + L - 4);
  if (it->n == 0) return ORC_ST_CORRUPT;                  /* assert!(num_restarts > 0) :79 */
  it->current = ro;
  it->has_next = 0;
  return 0;
}

static void oiter_free(oiter* it) { free(it->key); it->key = NULL; free(it->owned); it->owned = NULL; }

/* Vec::extend_from_slice growth (RawVec::grow_amortized): max(2cap, len+add, 8) */
static void okey_extend(oiter* it, const uint8_t* src, uint64_t n) {
  if (n == 0) return;
  if (it->kcap - it->klen < n) {
    uint64_t c = it->kcap * 2, req = it->klen + n;
    if (req > c) c = req;
    if (c < 8) c = 8;
    it->kcap = c;
  }
  if (it->klen + n > it->kalloc) {
    uint64_t a = it->kalloc ? it->kalloc : 64;
    while (a < it->klen + n) a *= 2;
    it->key = (uint8_t*)realloc(it->key, a);
    it->kalloc = a;
  }
  memcpy(it->key + it->klen, src, n);
  it->klen += n;
}

/* decode_entry (src/block.rs:216-238), wrapping usize arithmetic, bounds-checked reads */
static int odecode_entry(const uint8_t* d, uint64_t L, uint64_t p, uint64_t limit, uint32_t* sh, uint32_t* ns,
                         uint32_t* vl, uint64_t* pout) {
  if (limit - p < 3) return PANIC;                        /* Err -> unwrap panic (:217-219) */
  if (p + 2 >= L) return PANIC;                           /* data[p+2] out of bounds */
  uint32_t a = d[p], b = d[p + 1], c = d[p + 2];
  if ((a | b | c) < 128) {
    p += 3;                                               /* fast path (:225-227) */
  } else {
    int32_t k;
    if (p > L) return PANIC;
    k = oracle_varint_decode32(d + p, L - p, &a); if (k < 0) return PANIC; p += (uint64_t)k;
    if (p > L) return PANIC;
    k = oracle_varint_decode32(d + p, L - p, &b); if (k < 0) return PANIC; p += (uint64_t)k;
    if (p > L) return PANIC;
    k = oracle_varint_decode32(d + p, L - p, &c); if (k < 0) return PANIC; p += (uint64_t)k;
    if (!(p <= limit)) return PANIC;                      /* assert (:232) */
  }
  /* assert!(!((limit - p) < (non_shared + value_length) as usize)) (:235).  The u32
   * sum overflows only when one operand is >= 2^31: in debug that panics here, in
   * release the later slice data[p..p+ns] or get()'s data[val] panics (block < 2 GiB).
   * Either way the record is never yielded: treat as panic. */
  uint64_t sum = (uint64_t)b + (uint64_t)c;
  if (sum > U32MAX) return PANIC;
  if ((limit - p) < sum) return PANIC;
  *sh = a; *ns = b; *vl = c; *pout = p;
  return 0;
}

/* parse_next_key (src/block.rs:119-143).  returns 1 = parsed, 0 = end, PANIC */
static int oparse_next_key(oiter* it) {
  it->current = it->has_next ? it->next : 0;              /* next_entry_offset :114-117 */
  if (it->current >= it->restarts) {
    it->current = it->restarts;
    return 0;
  }
  uint32_t sh, ns, vl;
  uint64_t p;
  if (odecode_entry(it->d, it->L, it->current, it->restarts, &sh, &ns, &vl, &p) < 0) return PANIC;
  if (!(it->kcap >= sh)) return PANIC;                    /* assert capacity (:132) */
  if (sh < it->klen) it->klen = sh;                       /* truncate (:134) */
  if (p + ns > it->L) return PANIC;
  okey_extend(it, it->d + p, ns);                         /* :135 */
  it->has_next = 1;
  it->next = p + ns + vl;                                 /* :137 */
  it->has_val = 1;
  it->voff = p + ns;
  it->vlen = vl;
  /* the restart_index catch-up loop (:139-141) only reads in-bounds restart words and
   * has no observable effect on the scan; it matters for nothing we emit. */
  return 1;
}

/* seek_to_restart_point (:106-112) */
static void oseek_to_restart_point(oiter* it, uint32_t idx) {
  it->klen = 0;
  it->has_next = 1;
  it->next = orestart_point(it, idx);
}

static int ovalid(const oiter* it) { return it->current < it->restarts; }

static int obytes_cmp(const uint8_t* a, uint64_t al, const uint8_t* b, uint64_t bl) {
  uint64_t m = al < bl ? al : bl;
  int c = m ? memcmp(a, b, m) : 0;
  if (c) return c < 0 ? -1 : 1;
  return al < bl ? -1 : (al > bl ? 1 : 0);
}

/* BlockIter::seek (src/block.rs:154-194).  returns 0 or PANIC */
static int oseek(oiter* it, const uint8_t* target, uint64_t tlen) {
  uint32_t left = 0, right = it->n - 1;
  while (left < right) {
    uint32_t mid = (uint32_t)(left + right + 1) / 2;
    uint64_t region = orestart_point(it, mid);
    uint32_t sh, ns, vl;
    uint64_t ko;
    if (odecode_entry(it->d, it->L, region, it->restarts, &sh, &ns, &vl, &ko) < 0) return PANIC;
    if (sh != 0) return 0;                                 /* corruption: early return */
    if (ko + ns > it->L) return PANIC;
    if (obytes_cmp(it->d + ko, ns, target, tlen) < 0) left = mid;
    else right = mid - 1;
  }
  oseek_to_restart_point(it, left);
  for (;;) {
    int r = oparse_next_key(it);
    if (r <= 0) return r < 0 ? PANIC : 0;
    if (obytes_cmp(it->key, it->klen, target, tlen) >= 0) return 0;
  }
}

/* get (:204-213): 1 = Some, 0 = None, PANIC on out-of-range value slice */
static int oget(const oiter* it) {
  if (!ovalid(it)) return 0;
  if (it->voff + it->vlen > it->L) return PANIC;
  return 1;
}

/* Decode one block with the scan used by ReaderIntoIter::next / examples/dump.rs:
 * seek_to_first, then get/next until get() is None.  Emits via callback. */
typedef int (*orec_cb)(void* ctx, const uint8_t* k, uint64_t kl, const uint8_t* v, uint64_t vl);
static int odecode_block(const uint8_t* d, uint64_t L, orec_cb cb, void* ctx, uint64_t* nrec_out) {
  uint64_t ro;
  uint64_t nrec = 0;
  *nrec_out = 0;
  int st = oblock_init(d, L, &ro);
  if (st) return st;
  oiter it;
  st = oiter_init(&it, d, L, ro);
  if (st) { oiter_free(&it); return st; }
  oseek_to_restart_point(&it, 0);                         /* seek_to_first (:149-152) */
  int r = oparse_next_key(&it);
  st = ORC_ST_OK;
  if (r < 0) { st = ORC_ST_CORRUPT; goto done; }
  for (;;) {
    int g = oget(&it);
    if (g < 0) { st = ORC_ST_CORRUPT; break; }
    if (g == 0) break;
    if (cb(ctx, it.key, it.klen, it.d + it.voff, it.vlen)) { st = ORC_ST_OVERFLOW; nrec++; break; }
    nrec++;
    uint64_t cur = it.current;
    if (it.next == cur) { st = ORC_ST_LOOP; break; }       /* zero progress: infinite loop */
    r = oparse_next_key(&it);                              /* next() (:196-202) */
    if (r < 0) { st = ORC_ST_CORRUPT; break; }
  }
done:
  *nrec_out = nrec;
  oiter_free(&it);
  return st;
}

typedef struct {
  uint64_t nrec, kb, vb;
  uint8_t* keys; uint64_t keys_cap, key_base;
  uint8_t* vals; uint64_t vals_cap, val_base;
  uint32_t* key_end; uint32_t* val_end; uint64_t rec_cap, rec_base;
  int overflow;
} obatch_ctx;

static int obatch_cb(void* c, const uint8_t* k, uint64_t kl, const uint8_t* v, uint64_t vl) {
  obatch_ctx* x = (obatch_ctx*)c;
  x->kb += kl; x->vb += vl; x->nrec++;
  if (!x->keys) return 0;
  uint64_t r = x->rec_base + x->nrec - 1;
  if (x->key_base + x->kb > x->keys_cap || x->val_base + x->vb > x->vals_cap || r >= x->rec_cap) {
    x->overflow = 1;
    return 0;
  }
  if (kl) memcpy(x->keys + x->key_base + x->kb - kl, k, kl);   /* k may be NULL when kl == 0 */
  if (vl) memcpy(x->vals + x->val_base + x->vb - vl, v, vl);
  x->key_end[r] = (uint32_t)x->kb;
  x->val_end[r] = (uint32_t)x->vb;
  return 0;
}

int32_t oracle_decode_blocks(const uint8_t* data, const uint64_t* blk_off, const uint32_t* blk_len, uint32_t nblk,
                             uint32_t* nrec, uint64_t* key_bytes, uint64_t* val_bytes, int32_t* status,
                             uint64_t* rec_base, uint64_t* key_base, uint64_t* val_base, uint8_t* keys,
                             uint64_t keys_cap, uint8_t* vals, uint64_t vals_cap, uint32_t* key_end,
                             uint32_t* val_end, uint64_t rec_cap) {
  uint64_t rb = 0, kb = 0, vb = 0;
  int any_over = 0;
  for (uint32_t b = 0; b < nblk; b++) {
    obatch_ctx x;
    memset(&x, 0, sizeof(x));
    x.keys = keys; x.keys_cap = keys_cap; x.key_base = kb;
    x.vals = vals; x.vals_cap = vals_cap; x.val_base = vb;
    x.key_end = key_end; x.val_end = val_end; x.rec_cap = rec_cap; x.rec_base = rb;
    uint64_t n = 0;
    int st = odecode_block(data + blk_off[b], blk_len[b], obatch_cb, &x, &n);
    if (x.overflow) any_over = 1;
    if (nrec) nrec[b] = (uint32_t)x.nrec;
    if (key_bytes) key_bytes[b] = x.kb;
    if (val_bytes) val_bytes[b] = x.vb;
    if (status) status[b] = st;
    if (rec_base) rec_base[b] = rb;
    if (key_base) key_base[b] = kb;
    if (val_base) val_base[b] = vb;
    rb += x.nrec; kb += x.kb; vb += x.vb;
  }
  return any_over ? ORC_ST_OVERFLOW : 0;
}

/* ---------------- CPU baseline: reference semantics (BASELINE.md CPU-A) ---------------- */
typedef struct {
  uint64_t h, n;
} ofnv_ctx;
static int ofnv_cb(void* c, const uint8_t* k, uint64_t kl, const uint8_t* v, uint64_t vl) {
  ofnv_ctx* x = (ofnv_ctx*)c;
  uint64_t h = x->h;
  /* fold lengths + first/last bytes + an 8-byte word of each: touches the key and value
   * memory like a consumer would without dominating the decode cost */
  h = (h ^ kl) * 0x100000001b3ull;
  h = (h ^ vl) * 0x100000001b3ull;
  for (uint64_t i = 0; i < kl; i++) h = (h ^ k[i]) * 0x100000001b3ull;
  if (vl) h = (h ^ v[0] ^ ((uint64_t)v[vl - 1] << 8)) * 0x100000001b3ull;
  x->h = h;
  x->n++;
  return 0;
}
typedef struct {
  const uint8_t* data; const uint64_t* off; const uint32_t* len;
  uint32_t b0, b1; int iters;
  uint64_t h, n;
} othr;
static void* othr_run(void* a) {
  othr* t = (othr*)a;
  ofnv_ctx x = {1469598103934665603ull, 0};
  for (int it = 0; it < t->iters; it++)
    for (uint32_t b = t->b0; b < t->b1; b++) {
      uint64_t n;
      odecode_block(t->data + t->off[b], t->len[b], ofnv_cb, &x, &n);
    }
  t->h = x.h; t->n = x.n;
  return NULL;
}
uint64_t oracle_bench_scan(const uint8_t* data, const uint64_t* blk_off, const uint32_t* blk_len, uint32_t nblk,
                           int nthreads, int iters, uint64_t* ns, uint64_t* nrec_total) {
  if (nthreads < 1) nthreads = 1;
  othr* ts = (othr*)calloc((size_t)nthreads, sizeof(othr));
  pthread_t* th = (pthread_t*)calloc((size_t)nthreads, sizeof(pthread_t));
  for (int i = 0; i < nthreads; i++) {
    ts[i].data = data; ts[i].off = blk_off; ts[i].len = blk_len; ts[i].iters = iters;
    ts[i].b0 = (uint32_t)((uint64_t)nblk * i / nthreads);
    ts[i].b1 = (uint32_t)((uint64_t)nblk * (i + 1) / nthreads);
  }
  struct timespec a, b;
  clock_gettime(CLOCK_MONOTONIC, &a);
  for (int i = 1; i < nthreads; i++) pthread_create(&th[i], NULL, othr_run, &ts[i]);
  othr_run(&ts[0]);
  for (int i = 1; i < nthreads; i++) pthread_join(th[i], NULL);
  clock_gettime(CLOCK_MONOTONIC, &b);
  *ns = (uint64_t)(b.tv_sec - a.tv_sec) * 1000000000ull + (uint64_t)(b.tv_nsec - a.tv_nsec);
  uint64_t h = 0, n = 0;
  for (int i = 0; i < nthreads; i++) { h ^= ts[i].h; n += ts[i].n; }
  if (nrec_total) *nrec_total = n;
  free(ts); free(th);
  return h;
}

/* ==================== block builder: src/block_builder.rs ==================== */
typedef struct {
  uint64_t interval;
  uint8_t* buf; uint64_t len, cap;
  uint8_t* last; uint64_t llen, lcap;
  uint64_t* restarts; uint64_t nrest, rcap;
  int finished;
  uint64_t counter;
} obuilder;

static void ogrow(uint8_t** p, uint64_t* cap, uint64_t need) {
  if (need <= *cap) return;
  uint64_t c = *cap ? *cap : 256;
  while (c < need) c *= 2;
  *p = (uint8_t*)realloc(*p, c);
  *cap = c;
}
static void oappend(obuilder* b, const void* s, uint64_t n) {
  ogrow(&b->buf, &b->cap, b->len + n);
  if (n) memcpy(b->buf + b->len, s, n);
  b->len += n;
}
static void opush_restart(obuilder* b, uint64_t v) {
  if (b->nrest == b->rcap) {
    b->rcap = b->rcap ? b->rcap * 2 : 64;
    b->restarts = (uint64_t*)realloc(b->restarts, b->rcap * sizeof(uint64_t));
  }
  b->restarts[b->nrest++] = v;
}
static void obuilder_init(obuilder* b, uint64_t interval) {   /* new (:16-25) */
  memset(b, 0, sizeof(*b));
  b->interval = interval;
  opush_restart(b, 0);
}
static void obuilder_reset(obuilder* b) {                      /* reset (:27-34) */
  b->len = 0; b->llen = 0; b->nrest = 0; opush_restart(b, 0);
  b->finished = 0; b->counter = 0;
}
static void obuilder_free(obuilder* b) { free(b->buf); free(b->last); free(b->restarts); }
static int obuilder_empty(const obuilder* b) { return b->len == 0; }   /* :36-38 */
static uint64_t obuilder_estimate(const obuilder* b) {                 /* :40-47 */
  uint64_t factor = b->len > U32MAX ? 8 : 4;
  return b->len + b->nrest * factor + 4;
}
static int obuilder_add(obuilder* b, const uint8_t* k, uint64_t kl, const uint8_t* v, uint64_t vl) { /* :49-83 */
  if (!(b->counter <= b->interval)) return PANIC;
  if (b->finished) return PANIC;
  uint64_t shared = 0;
  if (b->counter < b->interval) {
    uint64_t m = b->llen < kl ? b->llen : kl;
    while (shared < m && b->last[shared] == k[shared]) shared++;
  } else {
    opush_restart(b, b->len);
    b->counter = 0;
  }
  uint64_t non_shared = kl - shared;
  uint8_t t[10];
  uint32_t n;
  n = oracle_varint_encode32(t, (uint32_t)shared); oappend(b, t, n);
  n = oracle_varint_encode32(t, (uint32_t)non_shared); oappend(b, t, n);
  n = oracle_varint_encode32(t, (uint32_t)vl); oappend(b, t, n);
  oappend(b, k + shared, non_shared);
  oappend(b, v, vl);
  ogrow(&b->last, &b->lcap, kl);
  if (kl) memcpy(b->last, k, kl);
  b->llen = kl;
  b->counter++;
  return 0;
}
/* finish (:85-104): appends restarts + count; returns malloc'd content (builder keeps going) */
static uint8_t* obuilder_finish(obuilder* b, uint64_t* out_len) {
  int r64 = b->len > U32MAX;
  for (uint64_t i = 0; i < b->nrest; i++) {
    uint8_t t[8];
    if (r64) { wr64(t, b->restarts[i]); oappend(b, t, 8); }
    else { wr32(t, (uint32_t)b->restarts[i]); oappend(b, t, 4); }
  }
  uint8_t t[4];
  wr32(t, (uint32_t)b->nrest);
  oappend(b, t, 4);
  b->finished = 1;
  uint8_t* out = (uint8_t*)malloc(b->len ? b->len : 1);
  memcpy(out, b->buf, b->len);
  *out_len = b->len;
  b->len = 0;                                  /* mem::replace with a fresh Vec */
  return out;
}

int32_t oracle_build_block(uint64_t interval, uint64_t nrec, const uint8_t* keys, const uint64_t* key_end,
                           const uint8_t* vals, const uint64_t* val_end, uint8_t** out, uint64_t* out_len) {
  obuilder b;
  obuilder_init(&b, interval);
  uint64_t k0 = 0, v0 = 0;
  for (uint64_t i = 0; i < nrec; i++) {
    if (obuilder_add(&b, keys + k0, key_end[i] - k0, vals + v0, val_end[i] - v0) < 0) { obuilder_free(&b); return -1; }
    k0 = key_end[i]; v0 = val_end[i];
  }
  *out = obuilder_finish(&b, out_len);
  obuilder_free(&b);
  return 0;
}

/* ==================== writer: src/writer.rs + src/metadata.rs ==================== */
struct oracle_writer {
  uint8_t* out; uint64_t olen, ocap;
  uint64_t meta[9];           /* index_block_offset, data_block_size, compression, count_entries,
                                 count_data_blocks, bytes_data_blocks, bytes_index_block,
                                 bytes_keys, bytes_values */
  uint32_t compression;
  obuilder data, index;
  uint8_t* last_key; uint64_t lklen, lkcap;
  uint64_t last_offset, pending_offset;
  int pending_index_entry;
  int poisoned;
};
enum { M_IDX_OFF, M_BLOCK_SIZE, M_COMP, M_COUNT, M_NBLOCKS, M_BYTES_DATA, M_BYTES_INDEX, M_BYTES_KEYS, M_BYTES_VALS };

oracle_writer* oracle_writer_new(uint64_t block_size, uint64_t interval, uint32_t compression) {
  oracle_writer* w = (oracle_writer*)calloc(1, sizeof(*w));
  w->meta[M_BLOCK_SIZE] = block_size < 1024 ? 1024 : block_size;   /* WriterBuilder::block_size :43-46 */
  w->meta[M_COMP] = compression;
  w->compression = compression;
  obuilder_init(&w->data, interval);
  obuilder_init(&w->index, interval);
  return w;
}
void oracle_writer_free(oracle_writer* w) {
  if (!w) return;
  obuilder_free(&w->data); obuilder_free(&w->index);
  free(w->last_key); free(w->out); free(w);
}
static void wout(oracle_writer* w, const void* p, uint64_t n) {
  ogrow(&w->out, &w->ocap, w->olen + n);
  if (n) memcpy(w->out + w->olen, p, n);
  w->olen += n;
}
/* write_block (:203-237).  Only CompressionType::None is produced by the oracle writer:
 * compressed bytes are parity-unpinned and come from the product writer. */
static uint64_t owrite_block(oracle_writer* w, obuilder* b) {
  uint64_t clen;
  uint8_t* content = obuilder_finish(b, &clen);
  uint32_t crc = oracle_crc32c(content, clen);
  uint8_t lenbuf[10];
  uint32_t ll = oracle_varint_encode64(lenbuf, clen);
  uint8_t cb[4];
  wr32(cb, crc);
  wout(w, lenbuf, ll);
  wout(w, cb, 4);
  wout(w, content, clen);
  free(content);
  uint64_t written = ll + 4 + clen;
  w->last_offset = w->pending_offset;
  w->pending_offset += written;
  obuilder_reset(b);
  return written;
}
static int oflush(oracle_writer* w) {                       /* flush (:183-200) */
  if (obuilder_empty(&w->data)) return 0;
  if (w->pending_index_entry) return PANIC;
  w->meta[M_BYTES_DATA] += owrite_block(w, &w->data);
  w->meta[M_NBLOCKS] += 1;
  w->pending_index_entry = 1;
  return 0;
}

int64_t oracle_shortest_separator(uint8_t* s, uint64_t sl, const uint8_t* l, uint64_t ll) { /* :239-265 */
  uint64_t min_len = sl < ll ? sl : ll;
  uint64_t di = 0;
  while (di < min_len && s[di] == l[di]) di++;
  if (di >= min_len) return (int64_t)sl;
  uint8_t db = s[di];
  if (db < 255 && (uint8_t)(db + 1) < l[di]) {
    s[di] = (uint8_t)(db + 1);
    sl = di + 1;
  } else if (di < (min_len >= 2 ? min_len - 2 : 0)) {
    uint16_t us = (uint16_t)((s[di] << 8) | s[di + 1]);
    uint16_t ul = (uint16_t)((l[di] << 8) | l[di + 1]);
    uint16_t ub = (uint16_t)(us + 1);                      /* wrapping (release) */
    if (us <= ub && ub <= ul) {                             /* write_u16 APPENDS (:260) */
      s[sl] = (uint8_t)(ub >> 8);
      s[sl + 1] = (uint8_t)ub;
      sl += 2;
    }
  }
  if (!(obytes_cmp(s, sl, l, ll) < 0)) return -1;           /* assert!(start < limit) */
  return (int64_t)sl;
}

int32_t oracle_writer_insert(oracle_writer* w, const uint8_t* k, uint64_t kl, const uint8_t* v, uint64_t vl) {
  if (w->poisoned) return PANIC;
  if (w->meta[M_COUNT] > 0 && obytes_cmp(k, kl, w->last_key, w->lklen) <= 0) {
    w->poisoned = 1;
    return PANIC;                                           /* "out-of-order key" :119-123 */
  }
  uint64_t est = obuilder_estimate(&w->data) + 3 * 5 + kl + vl;   /* :125-126 */
  if (est >= w->meta[M_BLOCK_SIZE]) {
    if (oflush(w) < 0) { w->poisoned = 1; return PANIC; }
  }
  if (w->pending_index_entry) {                             /* :132-138 */
    if (!obuilder_empty(&w->data)) { w->poisoned = 1; return PANIC; }
    ogrow(&w->last_key, &w->lkcap, w->lklen + 2);
    int64_t nl = oracle_shortest_separator(w->last_key, w->lklen, k, kl);
    if (nl < 0) { w->poisoned = 1; return PANIC; }
    w->lklen = (uint64_t)nl;
    uint8_t enc[10];
    uint32_t el = oracle_varint_encode64(enc, w->last_offset);
    if (obuilder_add(&w->index, w->last_key, w->lklen, enc, el) < 0) { w->poisoned = 1; return PANIC; }
    w->pending_index_entry = 0;
  }
  ogrow(&w->last_key, &w->lkcap, kl + 2);
  if (kl) memcpy(w->last_key, k, kl);
  w->lklen = kl;
  w->meta[M_COUNT] += 1;
  w->meta[M_BYTES_KEYS] += kl;
  w->meta[M_BYTES_VALS] += vl;
  if (obuilder_add(&w->data, k, kl, v, vl) < 0) { w->poisoned = 1; return PANIC; }
  return 0;
}

int32_t oracle_writer_finish(oracle_writer* w, uint8_t** out, uint64_t* out_len) {  /* into_inner :155-181 */
  if (w->poisoned) return PANIC;
  if (oflush(w) < 0) return PANIC;
  if (w->pending_index_entry) {
    uint8_t enc[10];
    uint32_t el = oracle_varint_encode64(enc, w->last_offset);
    if (obuilder_add(&w->index, w->last_key, w->lklen, enc, el) < 0) return PANIC;
    w->pending_index_entry = 0;
  }
  w->meta[M_IDX_OFF] = w->pending_offset;
  w->meta[M_BYTES_INDEX] += owrite_block(w, &w->index);
  uint8_t md[512];                                          /* Metadata::write_to_bytes :61-79 */
  memset(md, 0, sizeof(md));
  for (int i = 0; i < 9; i++) wr64(md + 8 * i, w->meta[i]);
  wr32(md + 508, 0x4D54424Cu);
  wout(w, md, 512);
  *out = (uint8_t*)malloc(w->olen);
  memcpy(*out, w->out, w->olen);
  *out_len = w->olen;
  return 0;
}

/* ==================== zlib / zstd decompression ====================
 * src/compression.rs:85-92 (flate2 ZlibDecoder::read_to_end: a zlib-wrapped deflate stream,
 * bytes after its end unread, input ending first -> Err) and :140-145 (zstd::stream::copy_decode:
 * every frame until the input ends).  Both are format-defined; the oracle calls the system
 * zlib and libzstd.so.1 (the C library the zstd crate wraps) -- test infrastructure, the
 * crates themselves are not in /root/reference. */
#include <dlfcn.h>
#include <zlib.h>

int32_t oracle_zlib_decompress(const uint8_t* s, uint64_t n, uint8_t** out, uint64_t* out_len) {
  z_stream z;
  memset(&z, 0, sizeof z);
  if (inflateInit(&z) != Z_OK) return 1;
  uint64_t cap = 4096, len = 0;
  uint8_t* o = (uint8_t*)malloc(cap);
  z.next_in = (Bytef*)s;
  z.avail_in = (uInt)n;
  for (;;) {
    if (len == cap) { cap *= 2; o = (uint8_t*)realloc(o, cap); }
    z.next_out = o + len;
    z.avail_out = (uInt)(cap - len);
    int r = inflate(&z, Z_NO_FLUSH);
    len = cap - z.avail_out;
    if (r == Z_STREAM_END) break;
    if (r != Z_OK && !(r == Z_BUF_ERROR && z.avail_out == 0)) { inflateEnd(&z); free(o); return 1; }
  }
  inflateEnd(&z);
  *out = o; *out_len = len;
  return 0;
}

typedef struct { const void* src; size_t size; size_t pos; } ozin;
typedef struct { void* dst; size_t size; size_t pos; } ozout;
int32_t oracle_zstd_decompress(const uint8_t* s, uint64_t n, uint8_t** out, uint64_t* out_len) {
  static void* h = NULL;
  if (!h) h = dlopen("libzstd.so.1", RTLD_NOW | RTLD_LOCAL);
  if (!h) return 1;
  void* (*create)(void) = (void* (*)(void))dlsym(h, "ZSTD_createDStream");
  size_t (*freeds)(void*) = (size_t (*)(void*))dlsym(h, "ZSTD_freeDStream");
  size_t (*init)(void*) = (size_t (*)(void*))dlsym(h, "ZSTD_initDStream");
  size_t (*dec)(void*, ozout*, ozin*) = (size_t (*)(void*, ozout*, ozin*))dlsym(h, "ZSTD_decompressStream");
  unsigned (*iserr)(size_t) = (unsigned (*)(size_t))dlsym(h, "ZSTD_isError");
  if (!create || !freeds || !init || !dec || !iserr) return 1;
  void* d = create();
  if (!d || iserr(init(d))) { if (d) freeds(d); return 1; }
  uint64_t cap = 4096, len = 0;
  uint8_t* o = (uint8_t*)malloc(cap);
  ozin in = {s, (size_t)n, 0};
  size_t last = 0;
  for (;;) {
    if (len == cap) { cap *= 2; o = (uint8_t*)realloc(o, cap); }
    ozout ob = {o + len, (size_t)(cap - len), 0};
    last = dec(d, &ob, &in);
    if (iserr(last)) { freeds(d); free(o); return 1; }
    len += ob.pos;
    if (in.pos == in.size && ob.pos < ob.size) break;   /* input consumed, output drained */
  }
  freeds(d);
  if (last != 0) { free(o); return 1; }                   /* the input ended inside a frame */
  *out = o; *out_len = len;
  return 0;
}

/* ==================== snappy raw decompression ====================
 * src/compression.rs:116-119 calls snap::raw::Decoder::decompress_vec (crate snap 1.x, not in
 * /root/reference).  Restated from the published snappy format (format_description.txt):
 * varint32 uncompressed length, then literal / copy-1 / copy-2 / copy-4 elements; a copy
 * offset must be 1..produced; the output must be exactly the stated length.  Any error is
 * io::Error -> Err(Error::Io).  Byte-at-a-time on purpose (independent of the product's
 * memcpy-based decoder); pinned against libsnappy in tests/test_snappy.py.
 * returns 0 and a malloc'd buffer, or ORC_ERR_IO. */
int32_t oracle_snappy_decompress(const uint8_t* s, uint64_t n, uint8_t** out, uint64_t* out_len) {
  uint64_t want = 0, i = 0;
  int shift = 0, term = 0;
  while (i < n && i < 5) {
    uint8_t b = s[i++];
    want |= (uint64_t)(b & 0x7f) << shift;
    shift += 7;
    if (!(b & 0x80)) { term = 1; break; }
  }
  if (!term || want > 0xFFFFFFFFull) return ORC_ERR_IO;
  uint8_t* d = (uint8_t*)malloc(want ? want : 1);
  uint64_t o = 0;
  while (i < n) {
    uint32_t tag = s[i++];
    uint64_t len, off = 0;
    if ((tag & 3) == 0) {
      len = (tag >> 2) + 1;
      if (len > 60) {
        uint32_t nb = (uint32_t)len - 60;
        if (n - i < nb) goto bad;
        len = 0;
        for (uint32_t k = 0; k < nb; k++) len |= (uint64_t)s[i + k] << (8 * k);
        len += 1;
        i += nb;
      }
      if (n - i < len || want - o < len) goto bad;
      for (uint64_t k = 0; k < len; k++) d[o++] = s[i++];
      continue;
    }
    if ((tag & 3) == 1) {
      if (n - i < 1) goto bad;
      len = 4 + ((tag >> 2) & 7);
      off = ((uint64_t)(tag >> 5) << 8) | s[i++];
    } else if ((tag & 3) == 2) {
      if (n - i < 2) goto bad;
      len = 1 + (tag >> 2);
      off = (uint64_t)s[i] | ((uint64_t)s[i + 1] << 8);
      i += 2;
    } else {
      if (n - i < 4) goto bad;
      len = 1 + (tag >> 2);
      off = (uint64_t)s[i] | ((uint64_t)s[i + 1] << 8) | ((uint64_t)s[i + 2] << 16) | ((uint64_t)s[i + 3] << 24);
      i += 4;
    }
    if (off == 0 || off > o || want - o < len) goto bad;
    for (uint64_t k = 0; k < len; k++, o++) d[o] = d[o - off];
  }
  if (o != want) goto bad;
  *out = d;
  *out_len = want;
  return 0;
bad:
  free(d);
  return ORC_ERR_IO;
}

/* ==================== file-level iteration: src/reader.rs ==================== */
typedef struct {
  const uint8_t* d; uint64_t len;
  uint64_t meta[9]; int version; int verify;
  uint64_t ro_index;
  const uint8_t* index; uint64_t index_len;
} oreader;

/* ReaderBuilder::read (:31-81). returns 0, PANIC, or ORC_ERR_* (positive) */
static int oreader_open(oreader* r, const uint8_t* d, uint64_t len, int verify) {
  memset(r, 0, sizeof(*r));
  r->d = d; r->len = len; r->verify = verify;
  if (len < 512) return ORC_ERR_INVALID_METADATA_SIZE;
  const uint8_t* m = d + len - 512;
  uint32_t magic = rd32(m + 508);                           /* metadata.rs:28-33 */
  if (magic == 0x77846676u) r->version = 0;
  else if (magic == 0x4D54424Cu) r->version = 1;
  else return ORC_ERR_INVALID_FORMAT_VERSION;
  for (int i = 0; i < 9; i++) r->meta[i] = rd64(m + 8 * i);
  if (r->meta[M_COMP] > 5) return ORC_ERR_INVALID_COMPRESSION_ALGORITHM;
  uint64_t max_off = len - 512 - 13;                        /* wrapping usize (:46) */
  if (r->meta[M_IDX_OFF] > max_off) return ORC_ERR_INVALID_INDEX_BLOCK_OFFSET;
  uint64_t off = r->meta[M_IDX_OFF];
  uint64_t ll, il;
  if (off > len) return PANIC;                              /* &data[off..] */
  if (r->version == 0) {
    if (off + 4 > len) return PANIC;
    ll = 4; il = rd32(d + off);
  } else {
    uint64_t t;
    int32_t k = oracle_varint_decode64(d + off, len - off, &t);
    if (k < 0) return PANIC;
    ll = (uint64_t)k; il = t;
  }
  uint64_t start = off + ll + 4;
  if (start > len || il > len - start) return PANIC;       /* BytesView::slice assert */
  if (verify) {
    if (off + ll + 4 > len) return PANIC;
    if (rd32(d + off + ll) != oracle_crc32c(d + start, il)) return PANIC;   /* assert_eq :73 */
  }
  uint64_t ro;
  int st = oblock_init(d + start, il, &ro);
  if (st == ORC_ST_INVALID_BLOCK) return ORC_ERR_INVALID_BLOCK;
  if (st) return PANIC;
  r->index = d + start; r->index_len = il; r->ro_index = ro;
  return 0;
}

/* Reader::block (:140-175): 0 = ok (blk, blen point into the file), PANIC, ORC_ERR_* */
static int oreader_block(const oreader* r, uint64_t off, const uint8_t** blk, uint64_t* blen, uint64_t* ro,
                         uint8_t** owned) {
  *owned = NULL;
  if (!(off < r->len)) return PANIC;
  uint64_t ll, sz;
  if (r->version == 0) {
    if (off + 4 > r->len) return PANIC;
    ll = 4; sz = rd32(r->d + off);
  } else {
    uint64_t t;
    int32_t k = oracle_varint_decode64(r->d + off, r->len - off, &t);
    if (k < 0) return PANIC;
    ll = (uint64_t)k; sz = t;
  }
  uint64_t start = off + ll + 4;
  if (start > r->len || sz > r->len - start) return PANIC;
  if (r->verify && rd32(r->d + off + ll) != oracle_crc32c(r->d + start, sz)) return PANIC;
  const uint8_t* b = r->d + start;
  if (r->meta[M_COMP] == 1) {                               /* decompress (:166-170) */
    uint8_t* u; uint64_t ul;
    if (oracle_snappy_decompress(b, sz, &u, &ul)) return ORC_ERR_IO;
    *owned = u; b = u; sz = ul;
  } else if (r->meta[M_COMP] == 2 || r->meta[M_COMP] == 5) {
    uint8_t* u; uint64_t ul;
    const int e = r->meta[M_COMP] == 2 ? oracle_zlib_decompress(b, sz, &u, &ul) : oracle_zstd_decompress(b, sz, &u, &ul);
    if (e) return ORC_ERR_IO;
    *owned = u; b = u; sz = ul;
  } else if (r->meta[M_COMP] != 0) {
    return ORC_ERR_IO;   /* Lz4 / Lz4hc: the crate's Err "unsupported" (src/compression.rs:63-67) */
  }
  int st = oblock_init(b, sz, ro);
  if (st == ORC_ST_INVALID_BLOCK) { free(*owned); *owned = NULL; return ORC_ERR_INVALID_BLOCK; }
  if (st) { free(*owned); *owned = NULL; return PANIC; }
  *blk = b; *blen = sz;
  return 0;
}

typedef struct {
  oracle_scan_result* res;
  uint64_t kcap, vcap, rcap;
} oscan_out;
static void oscan_push(oscan_out* o, const uint8_t* k, uint64_t kl, const uint8_t* v, uint64_t vl) {
  oracle_scan_result* r = o->res;
  uint64_t kb = r->nrec ? r->key_end[r->nrec - 1] : 0, vb = r->nrec ? r->val_end[r->nrec - 1] : 0;
  ogrow(&r->keys, &o->kcap, kb + kl + 1);
  ogrow(&r->vals, &o->vcap, vb + vl + 1);
  if (r->nrec == o->rcap) {
    o->rcap = o->rcap ? o->rcap * 2 : 256;
    r->key_end = (uint64_t*)realloc(r->key_end, o->rcap * 8);
    r->val_end = (uint64_t*)realloc(r->val_end, o->rcap * 8);
  }
  if (kl) memcpy(r->keys + kb, k, kl);
  if (vl) memcpy(r->vals + vb, v, vl);
  r->key_end[r->nrec] = kb + kl;
  r->val_end[r->nrec] = vb + vl;
  r->nrec++;
}

/* block_at_index (:177-186) for the index iterator's current entry.
 * returns 1 = Some(block) into *bi, 0 = None, PANIC, or -(ORC_ERR_*) - 10 */
static int oblock_at_index(const oreader* r, const oiter* idx, oiter* bi) {
  int g = oget(idx);
  if (g < 0) return PANIC;
  if (g == 0) return 0;
  uint64_t off = 0;
  if (oracle_varint_decode64(idx->d + idx->voff, idx->vlen, &off) < 0) return PANIC;
  const uint8_t* blk; uint64_t blen, ro;
  uint8_t* owned;
  int e = oreader_block(r, off, &blk, &blen, &ro, &owned);
  if (e == PANIC) return PANIC;
  if (e > 0) return -10 - e;
  if (oiter_init(bi, blk, blen, ro)) { free(owned); return PANIC; }   /* BlockIter::init assert */
  bi->owned = owned;
  return 1;
}

int32_t oracle_file_scan(const uint8_t* data, uint64_t len, int32_t verify, int32_t mode, const uint8_t* key,
                         uint64_t klen, const uint8_t* key2, uint64_t klen2, uint64_t max_records,
                         oracle_scan_result* res) {
  memset(res, 0, sizeof(*res));
  oscan_out o = {res, 0, 0, 0};
  oreader r;
  int e = oreader_open(&r, data, len, verify);
  memcpy(res->meta, r.meta, sizeof(r.meta));
  res->version = r.version;
  if (e == PANIC) { res->end = ORC_END_PANIC; return 0; }
  if (e > 0) { res->end = ORC_END_ERR_OPEN; res->err = e; return 0; }

  oiter idx, bi;
  int have_bi = 0;
  memset(&bi, 0, sizeof(bi));
  if (oiter_init(&idx, r.index, r.index_len, r.ro_index)) { res->end = ORC_END_PANIC; return 0; }
  /* ReaderIntoIter::new (:231-254) or new_from (:256-279) */
  if (mode == 0) {
    oseek_to_restart_point(&idx, 0);
    if (oparse_next_key(&idx) < 0) { res->end = ORC_END_PANIC; goto out; }
  } else {
    if (oseek(&idx, key, klen) < 0) { res->end = ORC_END_PANIC; goto out; }
  }
  {
    int b = oblock_at_index(&r, &idx, &bi);
    if (b == PANIC) { res->end = ORC_END_PANIC; goto out; }
    if (b <= -10) { res->end = ORC_END_ERR_OPEN; res->err = -10 - b; goto out; }
    if (b == 1) {
      have_bi = 1;
      int s = (mode == 0) ? (oseek_to_restart_point(&bi, 0), oparse_next_key(&bi)) : oseek(&bi, key, klen);
      if (s < 0) { res->end = ORC_END_PANIC; goto out; }
    }
  }
  /* mode -> ReaderIterType: 0,4 Iter; 1 Get; 2 GetPrefix; 3 GetRange (k = end key) */
  const uint8_t* fk = (mode == 3) ? key2 : key;
  uint64_t fkl = (mode == 3) ? klen2 : klen;
  int first = 1, valid = 1;
  for (;;) {                                                /* ReaderIntoIter::next (:337-405) */
    if (res->nrec >= max_records) break;
    if (!valid) break;
    if (!have_bi) break;
    if (!first) {
      if (ovalid(&bi)) {
        if (bi.has_next && bi.next == bi.current) { res->end = ORC_END_LOOP; goto out; } /* never terminates */
        if (oparse_next_key(&bi) < 0) { res->end = ORC_END_PANIC; goto out; }
      }
    }
    first = 0;
    const uint8_t *k, *v;
    uint64_t kl, vl;
    int g = oget(&bi);
    if (g < 0) { res->end = ORC_END_PANIC; goto out; }
    if (g == 1) {
      k = bi.key; kl = bi.klen; v = bi.d + bi.voff; vl = bi.vlen;
    } else {
      valid = 0;
      if (!ovalid(&idx)) break;                               /* index_iter.next() == false */
      if (oparse_next_key(&idx) < 0) { res->end = ORC_END_PANIC; goto out; }
      if (!ovalid(&idx)) break;
      oiter nb;
      int b = oblock_at_index(&r, &idx, &nb);
      if (b == PANIC) { res->end = ORC_END_PANIC; goto out; }
      if (b <= -10) {
        if (mode == 1) {
          /* Reader::get (src/reader.rs:111-122) matches Some(_) -- this Some(Err) too -- and
           * returns Ok(ReaderIntoGet::new(iter.bi)): bi is still the OLD iterator (not
           * reassigned on Err, :376-379), so its last parsed value, or Ok(None) (:195-203) */
          if (bi.has_val && bi.voff + bi.vlen <= bi.L) oscan_push(&o, bi.key, bi.klen, bi.d + bi.voff, bi.vlen);
          break;
        }
        res->end = ORC_END_ERR_NEXT; res->err = -10 - b; goto out;
      }
      if (b == 0) break;
      oiter_free(&bi);
      bi = nb;
      oseek_to_restart_point(&bi, 0);
      if (oparse_next_key(&bi) < 0) { res->end = ORC_END_PANIC; goto out; }
      g = oget(&bi);
      if (g < 0) { res->end = ORC_END_PANIC; goto out; }
      valid = g == 1;
      if (!valid) break;                                      /* entry? -> None */
      k = bi.key; kl = bi.klen; v = bi.d + bi.voff; vl = bi.vlen;
    }
    if (mode == 1) { if (obytes_cmp(k, kl, fk, fkl) != 0) valid = 0; }
    else if (mode == 2) { if (!(fkl <= kl && (fkl == 0 || memcmp(k, fk, fkl) == 0))) valid = 0; }
    else if (mode == 3) { if (obytes_cmp(k, kl, fk, fkl) > 0) valid = 0; }
    if (!valid) break;
    oscan_push(&o, k, kl, v, vl);
    if (mode == 1) break;                                     /* Reader::get takes one */
  }
  res->end = ORC_END_NONE;
out:
  oiter_free(&idx);
  if (have_bi) oiter_free(&bi);
  return 0;
}

/* ============ ReaderIntoIter with mid-iteration seek: src/reader.rs:219-405 ============
 * The iterator as a state machine, driven by a script of next() / seek() calls, so the
 * stateful parts of the reference are pinned: ReaderIntoIter::seek (:302-335) re-loads the
 * block only when the landed index entry's offset differs from `block_offset` -- a field
 * that new/new_from set to 0 and next() never updates (:244-246, :269-271, :362-366) -- so a
 * seek can re-seek whatever block the iterator currently holds; the re-seeked BlockIter
 * keeps its key Vec capacity (:327-329, src/block.rs:106-112).  The index iterator is the
 * LIVE one (:303): a seek whose binary search returns early on a restart entry with
 * shared != 0 (src/block.rs:167-170) leaves it where it was, key capacity included, and
 * next() continues from wherever the seek's linear scan left it, on the scan chain or not.
 * The data block is seeked with the landed index entry's key (:305 shadows `key`). */
typedef struct {
  oreader r;
  oiter idx, bi;
  int have_bi, first, valid, type;   /* type: 0 Iter, 1 Get, 2 GetPrefix, 3 GetRange */
  const uint8_t* k; uint64_t kl;     /* ReaderIntoIter::k */
  uint64_t block_offset;
} ostate;

enum { OS_SOME = 1, OS_NONE = 0, OS_LOOP = -2 };   /* + PANIC (-1), -(10 + err) = Some(Err) / Err */

/* ReaderIntoIter::next (:337-405) */
static int ostate_next(ostate* s, const uint8_t** k, uint64_t* kl, const uint8_t** v, uint64_t* vl) {
  if (!s->valid) return OS_NONE;
  if (!s->have_bi) return OS_NONE;
  if (!s->first && ovalid(&s->bi)) {
    if (s->bi.has_next && s->bi.next == s->bi.current) return OS_LOOP;
    if (oparse_next_key(&s->bi) < 0) return PANIC;
  }
  s->first = 0;
  int g = oget(&s->bi);
  if (g < 0) return PANIC;
  if (g == 0) {
    s->valid = 0;
    if (!ovalid(&s->idx)) return OS_NONE;                      /* index_iter.next() == false */
    if (oparse_next_key(&s->idx) < 0) return PANIC;
    if (!ovalid(&s->idx)) return OS_NONE;
    oiter nb;
    int b = oblock_at_index(&s->r, &s->idx, &nb);
    if (b == PANIC) return PANIC;
    if (b <= -10) return b;                                   /* Some(Err(e)), valid stays false */
    if (b == 0) return OS_NONE;
    oiter_free(&s->bi);
    s->bi = nb;
    oseek_to_restart_point(&s->bi, 0);
    if (oparse_next_key(&s->bi) < 0) return PANIC;
    g = oget(&s->bi);
    if (g < 0) return PANIC;
    s->valid = g == 1;
    if (!s->valid) return OS_NONE;
  }
  *k = s->bi.key; *kl = s->bi.klen; *v = s->bi.d + s->bi.voff; *vl = s->bi.vlen;
  if (s->type == 1) { if (obytes_cmp(*k, *kl, s->k, s->kl) != 0) s->valid = 0; }
  else if (s->type == 2) { if (!(s->kl <= *kl && (s->kl == 0 || memcmp(*k, s->k, s->kl) == 0))) s->valid = 0; }
  else if (s->type == 3) { if (obytes_cmp(*k, *kl, s->k, s->kl) > 0) s->valid = 0; }
  return s->valid ? OS_SOME : OS_NONE;
}

/* ReaderIntoIter::seek (:302-335): 0 = Ok(true), PANIC, -(10 + err) = Err */
static int ostate_seek(ostate* s, const uint8_t* key, uint64_t kl) {
  if (oseek(&s->idx, key, kl) < 0) return PANIC;
  int g = oget(&s->idx);
  if (g < 0) return PANIC;
  if (g == 0) { s->valid = 0; return 0; }                     /* past the last key */
  uint64_t off = 0;
  if (oracle_varint_decode64(s->idx.d + s->idx.voff, s->idx.vlen, &off) < 0) return PANIC;
  if (s->block_offset != off) {
    s->block_offset = off;                                    /* updated before the load (:322) */
    const uint8_t* blk; uint64_t blen, ro; uint8_t* owned;
    int e = oreader_block(&s->r, off, &blk, &blen, &ro, &owned);
    if (e == PANIC) return PANIC;
    if (e > 0) return -10 - e;                                /* `?`: bi, first, valid unchanged */
    oiter nb;
    if (oiter_init(&nb, blk, blen, ro)) { free(owned); return PANIC; }
    nb.owned = owned;
    if (s->have_bi) oiter_free(&s->bi);
    s->bi = nb;
    s->have_bi = 1;
  }
  /* :305 shadows `key` with the landed INDEX entry's key (index_iter.get()), so :328 seeks
   * the data block to that separator, not to the caller's target */
  if (s->have_bi && oseek(&s->bi, s->idx.key, s->idx.klen) < 0) return PANIC;
  s->first = 1;
  s->valid = 1;
  return 0;
}

int32_t oracle_iter_script(const uint8_t* data, uint64_t len, int32_t verify, int32_t mode, const uint8_t* key,
                           uint64_t klen, const uint8_t* key2, uint64_t klen2, const int64_t* ops, uint64_t nops,
                           const uint8_t* op_keys, const uint64_t* op_key_end, int64_t* op_res,
                           oracle_scan_result* res) {
  memset(res, 0, sizeof(*res));
  for (uint64_t i = 0; i < nops; i++) op_res[2 * i] = op_res[2 * i + 1] = 0;
  oscan_out o = {res, 0, 0, 0};
  ostate s;
  memset(&s, 0, sizeof(s));
  int e = oreader_open(&s.r, data, len, verify);
  memcpy(res->meta, s.r.meta, sizeof(s.r.meta));
  res->version = s.r.version;
  if (e == PANIC) { res->end = ORC_END_PANIC; return 0; }
  if (e > 0) { res->end = ORC_END_ERR_OPEN; res->err = e; return 0; }
  if (oiter_init(&s.idx, s.r.index, s.r.index_len, s.r.ro_index)) { res->end = ORC_END_PANIC; return 0; }
  s.first = 1; s.valid = 1;
  s.type = mode == 1 ? 1 : mode == 2 ? 2 : mode == 3 ? 3 : 0;
  s.k = mode == 3 ? key2 : key;
  s.kl = mode == 3 ? klen2 : klen;
  if (mode == 0) {                                            /* new (:231-254) */
    oseek_to_restart_point(&s.idx, 0);
    if (oparse_next_key(&s.idx) < 0) { res->end = ORC_END_PANIC; goto out; }
  } else if (oseek(&s.idx, key, klen) < 0) {                  /* new_from (:256-279) */
    res->end = ORC_END_PANIC; goto out;
  }
  {
    int b = oblock_at_index(&s.r, &s.idx, &s.bi);
    if (b == PANIC) { res->end = ORC_END_PANIC; goto out; }
    if (b <= -10) { res->end = ORC_END_ERR_OPEN; res->err = -10 - b; goto out; }
    if (b == 1) {
      s.have_bi = 1;
      int r = (mode == 0) ? (oseek_to_restart_point(&s.bi, 0), oparse_next_key(&s.bi)) : oseek(&s.bi, key, klen);
      if (r < 0) { res->end = ORC_END_PANIC; goto out; }
    }
  }
  /* ops: n >= 0 = up to n next() calls (stops at the first None / Err); -1 - j = seek(op key j).
   * op_res[2i] = records yielded (next) / 0; op_res[2i+1] = 0 Some..., 1 None, 2 Err (res->err),
   * for seek 0 Ok / 2 Err.  A panic or loop ends the script (res->end). */
  for (uint64_t i = 0; i < nops; i++) {
    if (ops[i] >= 0) {
      for (int64_t n = 0; n < ops[i]; n++) {
        const uint8_t *k, *v; uint64_t kl, vl;
        int r = ostate_next(&s, &k, &kl, &v, &vl);
        if (r == OS_SOME) { oscan_push(&o, k, kl, v, vl); op_res[2 * i]++; continue; }
        if (r == OS_NONE) { op_res[2 * i + 1] = 1; break; }
        if (r == PANIC) { res->end = ORC_END_PANIC; goto out; }
        if (r == OS_LOOP) { res->end = ORC_END_LOOP; goto out; }
        op_res[2 * i + 1] = 2; res->err = -10 - r; break;
      }
    } else {
      const uint64_t j = (uint64_t)(-1 - ops[i]);
      const uint64_t a = j ? op_key_end[j - 1] : 0;
      int r = ostate_seek(&s, op_keys + a, op_key_end[j] - a);
      if (r == PANIC) { res->end = ORC_END_PANIC; goto out; }
      if (r <= -10) { op_res[2 * i + 1] = 2; res->err = -10 - r; }
    }
  }
  res->end = ORC_END_NONE;
out:
  oiter_free(&s.idx);
  if (s.have_bi) oiter_free(&s.bi);
  return 0;
}

void oracle_scan_free(oracle_scan_result* r) {
  free(r->keys); free(r->vals); free(r->key_end); free(r->val_end);
  memset(r, 0, sizeof(*r));
}

/* ==================== full-size checker: device Writer output vs this restatement ====================
 * TEST INFRASTRUCTURE (tests/test_cfg3_oracle_gpu.py).  For every shard (an independent Writer,
 * src/writer.rs:112-149) of a device-encoded chunk:
 *  - the oracle Writer (oracle_writer_insert / _finish: the flush rule :125-130, BlockBuilder::add /
 *    finish src/block_builder.rs:49-104, write_block framing :203-237) is fed the shard's records and
 *    its data-block region is compared frame by frame with the device's framed blocks (varint64
 *    length, crc32c, content): res[0] += equal blocks, res[1] += device blocks of the shard;
 *  - every device block's content is decoded by the restated seek_to_first + next/get scan
 *    (odecode_block, src/block.rs:119-238) and each yielded record compared with the input record
 *    (key bytes, value bytes): res[2] += equal records, res[3] += records the cut assigns;
 *  - res[4] = first block that differs (UINT64_MAX if none), res[5] = shards whose cut, block count
 *    or framing does not line up with the oracle Writer's.
 * key_end / val_end: u64 END offsets from record 0; blk_rec[nblk + 1], shard_rec[nshard + 1]:
 * record cuts (int64).  Work is split over nthreads by shard. */
typedef struct {
  const uint8_t* keys; const uint64_t* key_end; const uint8_t* vals; const uint64_t* val_end;
  uint64_t r, r_end, equal, seen;
} ochk_rec;
static int ochk_cb(void* c, const uint8_t* k, uint64_t kl, const uint8_t* v, uint64_t vl) {
  ochk_rec* x = (ochk_rec*)c;
  x->seen++;
  if (x->r < x->r_end) {
    uint64_t k0 = x->r ? x->key_end[x->r - 1] : 0, v0 = x->r ? x->val_end[x->r - 1] : 0;
    uint64_t ekl = x->key_end[x->r] - k0, evl = x->val_end[x->r] - v0;
    if (ekl == kl && evl == vl && (!kl || !memcmp(k, x->keys + k0, kl)) && (!vl || !memcmp(v, x->vals + v0, vl)))
      x->equal++;
  }
  x->r++;
  return 0;
}
typedef struct {
  const uint8_t* file; uint64_t file_len; const uint64_t* blk_off; const uint32_t* blk_len; uint64_t nblk;
  const int64_t* blk_rec; const uint8_t* keys; const uint64_t* key_end; const uint8_t* vals; const uint64_t* val_end;
  const int64_t* shard_rec; uint64_t nshard; uint64_t block_size, interval;
  volatile uint64_t next_shard;
  pthread_mutex_t mu;
  uint64_t res[6];
} ochk_job;
static uint64_t ochk_lower(const int64_t* a, uint64_t n, int64_t v) {   /* first i in [0, n] with a[i] >= v */
  uint64_t lo = 0, hi = n + 1;
  while (lo < hi) { uint64_t m = (lo + hi) / 2; if (a[m] >= v) hi = m; else lo = m + 1; }
  return lo;
}
static void* ochk_run(void* a) {
  ochk_job* j = (ochk_job*)a;
  for (;;) {
    uint64_t s = __sync_fetch_and_add(&j->next_shard, 1);
    if (s >= j->nshard) break;
    uint64_t res[6] = {0, 0, 0, 0, UINT64_MAX, 0};
    int64_t r0 = j->shard_rec[s], r1 = j->shard_rec[s + 1];
    if (r1 > j->blk_rec[j->nblk]) r1 = j->blk_rec[j->nblk];
    if (r0 < r1) {
      uint64_t b0 = ochk_lower(j->blk_rec, j->nblk, r0), b1 = ochk_lower(j->blk_rec, j->nblk, r1);
      if (b0 > j->nblk || j->blk_rec[b0] != r0 || b1 > j->nblk || j->blk_rec[b1] != r1) res[5]++;
      if (b1 > j->nblk) b1 = j->nblk;
      /* the oracle Writer over the shard's records */
      oracle_writer* w = oracle_writer_new(j->block_size, j->interval, 0);
      int bad = 0;
      for (int64_t r = r0; r < r1 && !bad; r++) {
        uint64_t k0 = r ? j->key_end[r - 1] : 0, v0 = r ? j->val_end[r - 1] : 0;
        bad = oracle_writer_insert(w, j->keys + k0, j->key_end[r] - k0, j->vals + v0, j->val_end[r] - v0) != 0;
      }
      uint8_t* of = NULL;
      uint64_t olen = 0;
      if (!bad) bad = oracle_writer_finish(w, &of, &olen) != 0;
      uint64_t data_end = bad ? 0 : w->meta[M_IDX_OFF];
      oracle_writer_free(w);
      uint64_t pos = 0;
      for (uint64_t b = b0; b < b1; b++) {
        res[1]++;
        /* the device frame: varint64(len) | crc32c | content, ending at the content's end */
        uint8_t lb[10];
        uint32_t ll = oracle_varint_encode64(lb, j->blk_len[b]);
        uint64_t fl = ll + 4 + (uint64_t)j->blk_len[b];
        int eq = 0;
        if (!bad && j->blk_off[b] >= ll + 4 && j->blk_off[b] + j->blk_len[b] <= j->file_len && pos + fl <= data_end) {
          const uint8_t* dv = j->file + j->blk_off[b] - ll - 4;
          eq = memcmp(dv, of + pos, fl) == 0;
        }
        if (eq) res[0]++;
        else if (res[4] == UINT64_MAX) res[4] = b;
        pos += fl;
        /* the restated scan over the device block's content */
        ochk_rec x = {j->keys, j->key_end, j->vals, j->val_end, (uint64_t)j->blk_rec[b],
                      (uint64_t)(b + 1 <= j->nblk ? j->blk_rec[b + 1] : j->blk_rec[b]), 0, 0};
        uint64_t n = 0;
        int st = ORC_ST_CORRUPT;
        if (j->blk_off[b] + j->blk_len[b] <= j->file_len)
          st = odecode_block(j->file + j->blk_off[b], j->blk_len[b], ochk_cb, &x, &n);
        uint64_t want = x.r_end - (uint64_t)j->blk_rec[b];
        res[3] += want;
        if (st == ORC_ST_OK && x.seen == want) res[2] += x.equal;
        else if (res[4] == UINT64_MAX) res[4] = b;
      }
      if (bad || pos != data_end) res[5]++;
      free(of);
    }
    pthread_mutex_lock(&j->mu);
    for (int i = 0; i < 4; i++) j->res[i] += res[i];
    if (res[4] < j->res[4]) j->res[4] = res[4];
    j->res[5] += res[5];
    pthread_mutex_unlock(&j->mu);
  }
  return NULL;
}
int32_t oracle_check_writer_blocks(const uint8_t* file, uint64_t file_len, const uint64_t* blk_off,
                                   const uint32_t* blk_len, uint64_t nblk, const int64_t* blk_rec,
                                   const uint8_t* keys, const uint64_t* key_end, const uint8_t* vals,
                                   const uint64_t* val_end, const int64_t* shard_rec, uint64_t nshard,
                                   uint64_t block_size, uint64_t interval, int nthreads, uint64_t* res) {
  ochk_job j;
  memset(&j, 0, sizeof j);
  j.file = file; j.file_len = file_len; j.blk_off = blk_off; j.blk_len = blk_len; j.nblk = nblk;
  j.blk_rec = blk_rec; j.keys = keys; j.key_end = key_end; j.vals = vals; j.val_end = val_end;
  j.shard_rec = shard_rec; j.nshard = nshard; j.block_size = block_size; j.interval = interval;
  j.res[4] = UINT64_MAX;
  pthread_mutex_init(&j.mu, NULL);
  if (nthreads < 1) nthreads = 1;
  pthread_t* th = (pthread_t*)calloc((size_t)nthreads, sizeof(pthread_t));
  for (int i = 1; i < nthreads; i++) pthread_create(&th[i], NULL, ochk_run, &j);
  ochk_run(&j);
  for (int i = 1; i < nthreads; i++) pthread_join(th[i], NULL);
  free(th);
  pthread_mutex_destroy(&j.mu);
  memcpy(res, j.res, sizeof j.res);
  return 0;
}
