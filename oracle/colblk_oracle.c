/*
 * oracle/colblk_oracle.c — TEST INFRASTRUCTURE ONLY.
 *
 * A plain-C, sequential restatement of Pebble's columnar (colblk) data-block
 * reader for the default key schema and the CockroachDB "crdb1" key schema,
 * used as the parity checker for the HIP decoder.  Only tests/, the smoke() of
 * __graft_entry__.py and bench.py's cpu_baseline leg may load this.
 *
 * Pinned by: the whole-block hex dumps of the sstable/colblk/testdata/data_block
 * files and cockroachkvs/testdata/block_encoding, against the KVs the reference's
 * tests wrote into them (tests/golden/colblk_golden.json, tests/test_oracle_colblk.py).
 *
 * Functions restated (cockroachdb/pebble, paths relative to the repo root):
 *   header / column directory  sstable/colblk/block.go:179-201 (Header), :287-301
 *                              (DecodeColumn: type check, end == next page start),
 *                              :320-387 (BlockDecoder.Init, pageStart: last column
 *                              ends at len-1)
 *   Uint columns               sstable/colblk/unsafe_uints.go:32-72 (DecodeUnsafeUints),
 *                              :87-96 (DecodeUnsafeOffsets: no base, width != 8),
 *                              endian_little.go:21-43 (At = base + v[i])
 *   RawBytes                   sstable/colblk/raw_bytes.go:63-81 (DecodeRawBytes), At/Slice
 *   PrefixBytes                sstable/colblk/prefix_bytes.go:206-231 (DecodePrefixBytes),
 *                              :286-386 (SetAt/SetNext/SharedPrefix/RowBundlePrefix/
 *                              rowSuffixOffsets: an empty suffix repeats the nearest
 *                              non-empty one of the bundle), :1135-1170 (bundleCalc)
 *   Bitmap                     sstable/colblk/bitmap.go:43-77 (DecodeBitmap, At)
 *   DataBlockDecoder.Init      sstable/colblk/data_block.go:1096-1109 (+ panics ->
 *                              corruption, :1001-1014)
 *   DataBlockIter.Next         sstable/colblk/data_block.go:1662-1708 (K = {MaterializeUserKey,
 *                              trailers.At}, V = values.At, isValueExternal -> valuer)
 *   defaultKeySeeker           sstable/colblk/data_block.go:361-366, 428-442
 *   cockroachKeySeeker         cockroachkvs/cockroachkvs.go:782-802 (init), 1009-1071
 *                              (MaterializeUserKey)
 *   DataBlockIter.decodeMeta   sstable/colblk/data_block.go:1602-1641 (FLAG_TIERING, the
 *                              Pebblev8 tiering columns, ids :514-525): tieringSpanIDs /
 *                              tieringAttributes decoded by DecodeColumn as Uint columns;
 *                              KVMeta{} without the flag.  Pinned by the v8 block of
 *                              sstable/testdata/writer_tiering_histogram (the only
 *                              tiering bytes the reference holds).  A missing or
 *                              malformed tiering column, where Go panics in
 *                              initTieringMetadata, is CORRUPT_COLBLK_HEADER.
 *
 * Where Go would panic during metadata init the oracle reports
 * CORRUPT_COLBLK_HEADER; where Go would silently read outside a column during
 * iteration (unchecked unsafe offsets) it reports CORRUPT_BOUNDS.  A corrupt
 * block emits no rows, as on the device.
 */
#define _POSIX_C_SOURCE 200809L
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "oracle.h"

enum { DT_BOOL = 1, DT_UINT = 2, DT_BYTES = 3, DT_PREFIX = 4 };
#define DATA_BLOCK_CUSTOM_HEADER 4u /* data_block.go:607 */

static uint64_t le(const uint8_t* p, int w) {
  uint64_t v = 0;
  for (int i = w - 1; i >= 0; i--) v = v << 8 | p[i];
  return v;
}

typedef struct { uint64_t base, at; int w; } ucol;           /* UnsafeUints       */
typedef struct { ucol off; uint64_t data; uint32_t n; } rbcol; /* RawBytes (n slices) */
typedef struct { int zero; uint64_t at; } bmcol;              /* Bitmap            */
typedef struct { uint32_t shift; rbcol rb; } pbcol;           /* PrefixBytes       */

typedef struct {
  const uint8_t* b;
  uint64_t len;
  uint32_t custom, ncols, rows;
} blkdec;

static int page_start(const blkdec* d, uint32_t col, uint64_t* ps) {
  if (col >= d->ncols) { *ps = d->len - 1; return 1; }
  uint64_t h = (uint64_t)d->custom + 7 + 5ull * col;
  if (h + 5 > d->len) return 0;
  *ps = le(d->b + h + 1, 4);
  return 1;
}

static int dec_uints(const blkdec* d, uint64_t off, uint32_t rows, ucol* u, uint64_t* end) {
  u->base = 0; u->w = 0; u->at = off;
  if (rows == 0) { *end = off; return 1; }
  if (off >= d->len) return 0;
  uint8_t e = d->b[off++];
  int w = e & 0x7f, delta = (e & 0x80) != 0;
  if (!(w == 0 || w == 1 || w == 2 || w == 4 || (w == 8 && !delta))) return 0; /* IsValid */
  if (delta) {
    if (off + 8 > d->len) return 0;
    u->base = le(d->b + off, 8);
    off += 8;
  }
  if (w) off = (off + (uint64_t)w - 1) & ~((uint64_t)w - 1);
  u->w = w;
  u->at = off;
  *end = off + (uint64_t)rows * (uint64_t)w;
  return 1;
}
static uint64_t u_at(const blkdec* d, const ucol* u, uint32_t i) {
  return u->w ? u->base + le(d->b + u->at + (uint64_t)i * u->w, u->w) : u->base;
}

static int dec_rawbytes(const blkdec* d, uint64_t off, uint32_t count, rbcol* r, uint64_t* end) {
  memset(r, 0, sizeof(*r));
  r->n = count;
  if (count == 0) { *end = off; return 1; }
  uint64_t dend;
  if (!dec_uints(d, off, count + 1, &r->off, &dend)) return 0;
  if (r->off.base != 0 || r->off.w == 8) return 0; /* DecodeUnsafeOffsets */
  if (dend > d->len) return 0;
  r->data = dend;
  *end = dend + u_at(d, &r->off, count);
  return *end <= d->len;
}

static int dec_bitmap(const blkdec* d, uint64_t off, uint32_t n, bmcol* m, uint64_t* end) {
  if (off >= d->len) return 0;
  uint8_t e = d->b[off++];
  if (e == 1) { m->zero = 1; m->at = 0; *end = off; return 1; }
  m->zero = 0;
  off = (off + 7) & ~7ull;
  uint64_t nw = ((uint64_t)n + 63) >> 6, ns = (nw + 63) >> 6;
  m->at = off;
  *end = off + 8 * (nw + ns);
  return *end <= d->len;
}
static int bm_at(const blkdec* d, const bmcol* m, uint32_t i) {
  return m->zero ? 0 : (int)((le(d->b + m->at + 8ull * (i >> 6), 8) >> (i & 63)) & 1);
}

static int dec_prefix(const blkdec* d, uint64_t off, uint32_t count, pbcol* p, uint64_t* end) {
  if (count == 0 || off >= d->len) return 0; /* "empty PrefixBytes" panics */
  p->shift = d->b[off];
  if (p->shift > 16) return 0;
  uint32_t nb = 1 + ((count - 1) >> p->shift);
  return dec_rawbytes(d, off + 1, count + nb, &p->rb, end);
}

/* DecodeColumn: type check + end offset == next column's page start. */
static int column(const blkdec* d, uint32_t col, int type, uint64_t* start, uint64_t* next) {
  if (col >= d->ncols) return 0;
  uint64_t h = (uint64_t)d->custom + 7 + 5ull * col;
  if (h + 5 > d->len || d->b[h] != type) return 0;
  return page_start(d, col, start) && page_start(d, col + 1, next) && *next <= d->len && *start <= *next;
}

typedef struct {
  blkdec d;
  uint32_t schema, ncols_schema;
  pbcol keys;       /* col 0: default prefixes / crdb1 roach keys */
  rbcol suffixes;   /* default col 1                              */
  ucol wall, logical; rbcol untyped; /* crdb1 cols 1..3            */
  ucol trailers;
  bmcol prefix_changed, external, obsolete;
  rbcol values;
  ucol span, attr;  /* tiering columns (zero columns unless decoded) */
  uint32_t shared_len, data_len; /* prefix-bytes shared prefix length and data length */
} coldec;

static int init_decoder(const uint8_t* blk, uint64_t len, uint32_t schema, coldec* c) {
  memset(c, 0, sizeof(*c));
  c->schema = schema;
  c->ncols_schema = schema == FMT_COL_CRDB1 ? 4 : 2;
  uint32_t custom = DATA_BLOCK_CUSTOM_HEADER + (schema == FMT_COL_CRDB1 ? 1 : 0);
  blkdec* d = &c->d;
  d->b = blk; d->len = len; d->custom = custom;
  if (len < (uint64_t)custom + 7) return 0;
  d->ncols = (uint32_t)le(blk + custom + 1, 2);
  d->rows = (uint32_t)le(blk + custom + 3, 4);
  uint32_t S = c->ncols_schema;
  uint64_t s, nx, e;
  /* DataBlockDecoder.Init (data_block.go:1096-1109) */
  if (!column(d, S + 0, DT_UINT, &s, &nx) || !dec_uints(d, s, d->rows, &c->trailers, &e) || e != nx) return 0;
  if (!column(d, S + 1, DT_BOOL, &s, &nx) || !dec_bitmap(d, s, d->rows, &c->prefix_changed, &e) || e != nx) return 0;
  if (!column(d, S + 2, DT_BYTES, &s, &nx) || !dec_rawbytes(d, s, d->rows, &c->values, &e) || e != nx) return 0;
  if (!column(d, S + 3, DT_BOOL, &s, &nx) || !dec_bitmap(d, s, d->rows, &c->external, &e) || e != nx) return 0;
  if (!column(d, S + 4, DT_BOOL, &s, &nx) || !dec_bitmap(d, s, d->rows, &c->obsolete, &e) || e != nx) return 0;
  /* KeySchema.InitKeySeekerMetadata */
  if (!column(d, 0, DT_PREFIX, &s, &nx) || !dec_prefix(d, s, d->rows, &c->keys, &e) || e != nx) return 0;
  if (schema == FMT_COL_CRDB1) {
    if (!column(d, 1, DT_UINT, &s, &nx) || !dec_uints(d, s, d->rows, &c->wall, &e) || e != nx) return 0;
    if (!column(d, 2, DT_UINT, &s, &nx) || !dec_uints(d, s, d->rows, &c->logical, &e) || e != nx) return 0;
    if (!column(d, 3, DT_BYTES, &s, &nx) || !dec_rawbytes(d, s, d->rows, &c->untyped, &e) || e != nx) return 0;
  } else {
    if (!column(d, 1, DT_BYTES, &s, &nx) || !dec_rawbytes(d, s, d->rows, &c->suffixes, &e) || e != nx) return 0;
  }
  c->shared_len = (uint32_t)u_at(d, &c->keys.rb.off, 0);
  c->data_len = (uint32_t)u_at(d, &c->keys.rb.off, c->keys.rb.n);
  return 1;
}

/* initTieringMetadata (data_block.go:1605-1631): the two Uint columns after
 * isObsolete, by DecodeColumn (type check, end == next page start). */
static int init_tiering(coldec* c) {
  const blkdec* d = &c->d;
  uint32_t S = c->ncols_schema;
  uint64_t s, nx, e;
  if (!column(d, S + 5, DT_UINT, &s, &nx) || !dec_uints(d, s, d->rows, &c->span, &e) || e != nx) return 0;
  if (!column(d, S + 6, DT_UINT, &s, &nx) || !dec_uints(d, s, d->rows, &c->attr, &e) || e != nx) return 0;
  return 1;
}

/* RawBytes slice i, checked: [lo, hi) within the column's data. */
static int rb_slice(const coldec* c, const rbcol* r, uint32_t i, uint64_t* lo, uint64_t* hi) {
  uint64_t a = u_at(&c->d, &r->off, i), b = u_at(&c->d, &r->off, i + 1), n = u_at(&c->d, &r->off, r->n);
  if (a > b || b > n) return 0;
  *lo = r->data + a;
  *hi = r->data + b;
  return 1;
}

/* PrefixBytes key parts for `row`: shared [0,shared_len), bundle prefix, suffix. */
static int pb_parts(const coldec* c, uint32_t row, uint64_t* bp_lo, uint64_t* bp_hi, uint64_t* sf_lo,
                    uint64_t* sf_hi) {
  const pbcol* p = &c->keys;
  uint32_t s = p->shift, mask = ~((1u << s) - 1);
  uint32_t bi = (row >> s) + (row & mask);   /* bundleOffsetIndexForRow */
  uint32_t si = 1 + (row >> s) + row;        /* rowSuffixIndex          */
  if (c->shared_len > c->data_len) return 0;
  if (!rb_slice(c, &p->rb, bi, bp_lo, bp_hi)) return 0;
  uint64_t lo, hi;
  if (!rb_slice(c, &p->rb, si, &lo, &hi)) return 0;
  uint32_t first = 1 + bi;
  while (lo == hi && si > first) { /* rowSuffixOffsets: duplicate key */
    si--;
    if (!rb_slice(c, &p->rb, si, &lo, &hi)) return 0;
  }
  *sf_lo = lo;
  *sf_hi = hi;
  return 1;
}

/* MaterializeUserKey into dst (NULL = length only).  Returns length or -1. */
static int64_t materialize(const coldec* c, uint32_t row, uint8_t* dst) {
  uint64_t bl, bh, sl, sh;
  if (!pb_parts(c, row, &bl, &bh, &sl, &sh)) return -1;
  uint64_t n = 0;
  uint64_t parts[3][2] = {{c->keys.rb.data, c->keys.rb.data + c->shared_len}, {bl, bh}, {sl, sh}};
  for (int k = 0; k < 3; k++) {
    uint64_t m = parts[k][1] - parts[k][0];
    if (dst) memcpy(dst + n, c->d.b + parts[k][0], m);
    n += m;
  }
  if (c->schema == FMT_COL_CRDB1) {
    uint64_t wall = u_at(&c->d, &c->wall, row);
    uint32_t logical = (uint32_t)u_at(&c->d, &c->logical, row);
    if (wall == 0 && logical == 0) {
      uint64_t ul, uh;
      if (!rb_slice(c, &c->untyped, row, &ul, &uh)) return -1;
      if (dst) dst[n] = 0;
      n++;
      if (uh > ul) {
        if (dst) {
          memcpy(dst + n, c->d.b + ul, uh - ul);
          dst[n + (uh - ul)] = (uint8_t)(uh - ul + 1);
        }
        n += uh - ul + 1;
      }
    } else {
      if (dst) {
        dst[n] = 0;
        for (int i = 0; i < 8; i++) dst[n + 1 + i] = (uint8_t)(wall >> (56 - 8 * i));
      }
      n += 9;
      if (logical == 0) {
        if (dst) dst[n] = 9;
        n += 1;
      } else {
        if (dst) {
          for (int i = 0; i < 4; i++) dst[n + i] = (uint8_t)(logical >> (24 - 8 * i));
          dst[n + 4] = 13;
        }
        n += 5;
      }
    }
  } else {
    uint64_t ul, uh;
    if (!rb_slice(c, &c->suffixes, row, &ul, &uh)) return -1;
    if (dst) memcpy(dst + n, c->d.b + ul, uh - ul);
    n += uh - ul;
  }
  return (int64_t)n;
}

/* Two passes (count, then fill) over DataBlockIter First/Next (NextWithMeta
 * with FLAG_TIERING). */
int orc_colblk_decode_flags(const uint8_t* blk, uint64_t len, uint32_t schema, uint32_t flags, orc_block_out* o) {
  o->n_kv = o->key_bytes = o->val_bytes = o->n_restarts = 0;
  if (schema != FMT_COL_DEFAULT && schema != FMT_COL_CRDB1) return UNSUPPORTED;
  coldec c;
  if (!init_decoder(blk, len, schema, &c)) return CORRUPT_COLBLK_HEADER;
  if ((flags & FLAG_TIERING) && !init_tiering(&c)) return CORRUPT_COLBLK_HEADER;
  uint64_t kb = 0, vb = 0;
  uint32_t rows = c.d.rows;
  for (uint32_t r = 0; r < rows; r++) {
    int64_t kl = materialize(&c, r, NULL);
    uint64_t lo, hi;
    if (kl < 0 || !rb_slice(&c, &c.values, r, &lo, &hi)) return CORRUPT_BOUNDS;
    if (kb + (uint64_t)kl > 0xffffffffu || vb + (hi - lo) > 0xffffffffu) return UNSUPPORTED;
    kb += (uint64_t)kl;
    vb += hi - lo;
  }
  o->n_kv = rows;
  o->key_bytes = kb;
  o->val_bytes = vb;
  if (!o->trailer) return OK;
  kb = vb = 0;
  for (uint32_t r = 0; r < rows; r++) {
    int64_t kl = materialize(&c, r, o->keys + kb);
    uint64_t lo, hi;
    rb_slice(&c, &c.values, r, &lo, &hi);
    memcpy(o->vals + vb, blk + lo, hi - lo);
    o->trailer[r] = u_at(&c.d, &c.trailers, r);
    uint8_t fl = 0;
    if (bm_at(&c.d, &c.prefix_changed, r)) fl |= KV_PREFIX_CHANGED;
    if (bm_at(&c.d, &c.obsolete, r)) fl |= KV_OBSOLETE;
    if (bm_at(&c.d, &c.external, r)) fl |= (hi > lo && (blk[lo] & 0xC0) == 0x80) ? KV_VALBLK : KV_BLOB;
    if (o->kv_flags) o->kv_flags[r] = fl;
    if (o->entry_off) o->entry_off[r] = r;
    if (o->span) { /* decodeMeta (data_block.go:1633-1641); KVMeta{} without tiering */
      o->span[r] = u_at(&c.d, &c.span, r);
      o->attr[r] = u_at(&c.d, &c.attr, r);
    }
    o->key_off[r] = (uint32_t)kb;
    o->val_off[r] = (uint32_t)vb;
    kb += (uint64_t)kl;
    vb += hi - lo;
  }
  o->key_off[rows] = (uint32_t)kb;
  o->val_off[rows] = (uint32_t)vb;
  return OK;
}

int orc_colblk_decode(const uint8_t* blk, uint64_t len, uint32_t schema, orc_block_out* o) {
  return orc_colblk_decode_flags(blk, len, schema, 0, o);
}

/* Iterate-only CPU baseline for colblk (SURVEY.md §8(d) mode i), shaped like
 * DataBlockIter.First/Next: PrefixBytes.SetNext keeps the shared + bundle prefix
 * in a reused key buffer and copies only a row's suffix (prefix_bytes.go:303-356),
 * the version is appended per MaterializeUserKey, the value is zero-copy; all of
 * it folded into a checksum.  Typed loads of the column widths (no byte loops). */
static inline uint64_t u_fast(const uint8_t* b, const ucol* u, uint32_t i) {
  const uint8_t* p = b + u->at;
  switch (u->w) {
    case 0: return u->base;
    case 1: return u->base + p[i];
    case 2: { uint16_t v; memcpy(&v, p + 2ull * i, 2); return u->base + v; }
    case 4: { uint32_t v; memcpy(&v, p + 4ull * i, 4); return u->base + v; }
    default: { uint64_t v; memcpy(&v, p + 8ull * i, 8); return v; }
  }
}

uint64_t orc_colblk_scan_checksum(const uint8_t* blk, uint64_t len, uint32_t schema, uint64_t* n_kv) {
  coldec c;
  *n_kv = 0;
  if (!init_decoder(blk, len, schema, &c)) return 0;
  uint8_t key[4096];
  const uint8_t* pdata = blk + c.keys.rb.data;
  const uint32_t shift = c.keys.shift, rows = c.d.rows;
  if (c.shared_len > sizeof(key) / 2) return 0;
  memcpy(key, pdata, c.shared_len);
  uint32_t pre = c.shared_len;  /* shared + bundle prefix length in key[] */
  uint32_t klen = pre;          /* roach key / prefix length */
  uint64_t h = 1469598103934665603ull;
  for (uint32_t r = 0; r < rows; r++) {
    if ((r & ((1u << shift) - 1)) == 0) { /* bundle start: bundle prefix */
      uint32_t bi = (r >> shift) + r;
      uint32_t a = (uint32_t)u_fast(blk, &c.keys.rb.off, bi), z = (uint32_t)u_fast(blk, &c.keys.rb.off, bi + 1);
      if (z < a || c.shared_len + (z - a) > sizeof(key) / 2) return 0;
      memcpy(key + c.shared_len, pdata + a, z - a);
      pre = c.shared_len + (z - a);
      klen = pre;
    }
    uint32_t si = 1 + (r >> shift) + r;
    uint32_t lo = (uint32_t)u_fast(blk, &c.keys.rb.off, si), hi = (uint32_t)u_fast(blk, &c.keys.rb.off, si + 1);
    if (hi > lo) { /* SetNext: an empty suffix keeps the previous key */
      if (pre + (hi - lo) > sizeof(key) / 2) return 0;
      memcpy(key + pre, pdata + lo, hi - lo);
      klen = pre + (hi - lo);
    }
    uint32_t n = klen;
    if (schema == FMT_COL_CRDB1) {
      uint64_t wall = u_fast(blk, &c.wall, r);
      uint32_t logical = (uint32_t)u_fast(blk, &c.logical, r);
      key[n++] = 0;
      if (wall == 0 && logical == 0) {
        uint32_t x = (uint32_t)u_fast(blk, &c.untyped.off, r), y = (uint32_t)u_fast(blk, &c.untyped.off, r + 1);
        if (y > x) {
          if (n + (y - x) + 1 > sizeof(key)) return 0;
          memcpy(key + n, blk + c.untyped.data + x, y - x);
          n += y - x;
          key[n++] = (uint8_t)(y - x + 1);
        }
      } else {
        uint64_t be = __builtin_bswap64(wall);
        memcpy(key + n, &be, 8);
        n += 8;
        if (logical == 0) key[n++] = 9;
        else { uint32_t bl = __builtin_bswap32(logical); memcpy(key + n, &bl, 4); n += 4; key[n++] = 13; }
      }
    } else {
      uint32_t x = (uint32_t)u_fast(blk, &c.suffixes.off, r), y = (uint32_t)u_fast(blk, &c.suffixes.off, r + 1);
      if (y < x || n + (y - x) > sizeof(key)) return 0;
      memcpy(key + n, blk + c.suffixes.data + x, y - x);
      n += y - x;
    }
    uint32_t vlo = (uint32_t)u_fast(blk, &c.values.off, r), vhi = (uint32_t)u_fast(blk, &c.values.off, r + 1);
    uint64_t tr = u_fast(blk, &c.trailers, r);
    h = (h ^ tr ^ key[n ? n - 1 : 0] ^ (vhi > vlo ? blk[c.values.data + vlo] : 0) ^ (vhi - vlo)) * 1099511628211ull;
  }
  *n_kv = rows;
  return h;
}

/* DataBlockIter under blockiter.Transforms{HideObsoletePoints}
 * (sstable/colblk/data_block.go:1680-1697): rows whose isObsolete bit is set
 * (data_block.go:519) are skipped; the block is checked and decoded whole
 * first, so a block that fails without the transform fails with it. */
static int colblk_decode_hide(const uint8_t* blk, uint64_t len, uint32_t fmt, uint32_t flags, orc_block_out* o) {
  orc_block_out t;
  memset(&t, 0, sizeof(t));
  int st = orc_colblk_decode_flags(blk, len, fmt, flags, &t);
  if (st != OK) {
    o->n_kv = o->key_bytes = o->val_bytes = o->n_restarts = 0;
    return st;
  }
  const uint64_t n = t.n_kv;
  uint64_t* tr = calloc(n + 1, 8);
  uint8_t* fl = calloc(n + 1, 1);
  uint32_t* eo = calloc(n + 1, 4);
  uint32_t* ko = calloc(n + 1, 4);
  uint32_t* vo = calloc(n + 1, 4);
  uint8_t* kb = calloc(t.key_bytes + 1, 1);
  uint8_t* vb = calloc(t.val_bytes + 1, 1);
  uint64_t* sp = calloc(n + 1, 8);
  uint64_t* at = calloc(n + 1, 8);
  orc_block_out f = {0, 0, 0, 0, tr, fl, eo, ko, vo, kb, vb, NULL, sp, at};
  st = orc_colblk_decode_flags(blk, len, fmt, flags, &f);
  uint64_t m = 0, kn = 0, vn = 0;
  for (uint64_t i = 0; st == OK && i < n; i++) {
    if (fl[i] & KV_OBSOLETE) continue;
    const uint32_t kl = ko[i + 1] - ko[i], vl = vo[i + 1] - vo[i];
    if (o->trailer) {
      o->trailer[m] = tr[i];
      if (o->kv_flags) o->kv_flags[m] = fl[i];
      if (o->entry_off) o->entry_off[m] = eo[i];
      if (o->span) {
        o->span[m] = sp[i];
        o->attr[m] = at[i];
      }
      o->key_off[m] = (uint32_t)kn;
      o->val_off[m] = (uint32_t)vn;
      memcpy(o->keys + kn, kb + ko[i], kl);
      memcpy(o->vals + vn, vb + vo[i], vl);
    }
    m++;
    kn += kl;
    vn += vl;
  }
  if (o->trailer && st == OK) {
    o->key_off[m] = (uint32_t)kn;
    o->val_off[m] = (uint32_t)vn;
  }
  free(tr); free(fl); free(eo); free(ko); free(vo); free(kb); free(vb); free(sp); free(at);
  o->n_kv = st == OK ? m : 0;
  o->key_bytes = st == OK ? kn : 0;
  o->val_bytes = st == OK ? vn : 0;
  o->n_restarts = 0;
  return st;
}

static int decode_block(const uint8_t* blk, uint64_t len, uint32_t fmt, uint32_t flags, orc_block_out* o) {
  if (fmt != FMT_ROW && (flags & FLAG_HIDE_OBSOLETE)) return colblk_decode_hide(blk, len, fmt, flags, o);
  if (fmt == FMT_ROW && o->span) { /* rowblk.Iter: no meta columns, KVMeta{} */
    uint64_t* sp = o->span;
    uint64_t* at = o->attr;
    o->span = o->attr = NULL;
    int st = decode_block(blk, len, fmt, flags, o);
    if (st == OK && o->trailer)
      for (uint64_t i = 0; i < o->n_kv; i++) sp[i] = at[i] = 0;
    o->span = sp;
    o->attr = at;
    return st;
  }
  if (fmt == FMT_ROW && (flags & FLAG_HIDE_OBSOLETE) && !(flags & FLAG_RAW_KEYS)) {
    /* HideObsoletePoints: rowblk.Iter under blockiter.Transforms{HideObsoletePoints} */
    const orc_transforms t = {0, 1, 0, NULL, 0, NULL, 0};
    return orc_rowblk_decode_tf(blk, len, flags & ~FLAG_HIDE_OBSOLETE, &t, o);
  }
  if (fmt == FMT_ROW) return orc_rowblk_decode(blk, len, flags, o);
  return orc_colblk_decode_flags(blk, len, fmt, flags, o);
}

/* Batch decode of a (possibly mixed) batch in the device layout; block b has
 * format block_fmt[b] when block_fmt is non-NULL, else `fmt`. */
int orc_decode_batch(const uint8_t* blocks, const uint64_t* off, const uint32_t* len, uint32_t n_blocks,
                     uint32_t fmt, const uint8_t* block_fmt, uint32_t flags, orc_batch_out* bo) {
  uint64_t kvb = 0, kb = 0, vb = 0, rb = 0;
  bo->status_mask = 0;
  bo->n_bad_blocks = 0;
  for (uint32_t b = 0; b < n_blocks; b++) {
    orc_block_out o;
    memset(&o, 0, sizeof(o));
    int fill = bo->trailer != NULL;
    if (fill) {
      o.trailer = bo->trailer + kvb;
      o.kv_flags = bo->kv_flags ? bo->kv_flags + kvb : NULL;
      o.entry_off = bo->entry_off ? bo->entry_off + kvb : NULL;
      o.key_off = bo->key_off + kvb + b;
      o.val_off = bo->val_off + kvb + b;
      o.keys = bo->key_bytes + kb;
      o.vals = bo->val_bytes + vb;
      o.restarts = bo->restarts ? bo->restarts + rb : NULL;
      o.span = bo->tiering_span_id ? bo->tiering_span_id + kvb : NULL;
      o.attr = bo->tiering_attr ? bo->tiering_attr + kvb : NULL;
    }
    int st = decode_block(blocks + off[b], len[b], block_fmt ? block_fmt[b] : fmt, flags, &o);
    if (fill && st != OK) {
      bo->key_off[kvb + b] = 0;
      bo->val_off[kvb + b] = 0;
    }
    if (bo->blk_status) bo->blk_status[b] = (uint32_t)st;
    if (bo->blk_kv_base) {
      bo->blk_kv_base[b] = kvb;
      bo->blk_key_base[b] = kb;
      bo->blk_val_base[b] = vb;
      if (bo->blk_rst_base) bo->blk_rst_base[b] = rb;
    }
    if (st != OK) {
      bo->status_mask |= 1u << st;
      bo->n_bad_blocks++;
    }
    kvb += o.n_kv;
    kb += o.key_bytes;
    vb += o.val_bytes;
    rb += o.n_restarts;
  }
  if (bo->blk_kv_base) {
    bo->blk_kv_base[n_blocks] = kvb;
    bo->blk_key_base[n_blocks] = kb;
    bo->blk_val_base[n_blocks] = vb;
    if (bo->blk_rst_base) bo->blk_rst_base[n_blocks] = rb;
  }
  bo->n_kv = kvb;
  bo->key_bytes_total = kb;
  bo->val_bytes_total = vb;
  bo->n_restarts = rb;
  return 0;
}

/* CPU baseline timing for either format (bench.py cpu_baseline leg): mode 0
 * iterate-only, mode 1 materialize into per-thread flat arrays. */
typedef struct {
  const uint8_t* blocks;
  const uint64_t* off;
  const uint32_t* len;
  uint32_t n, fmt, flags;
  int mode, reps, tid, nth;
  uint64_t sum;
} bench_task;

static void* bench_worker(void* arg) {
  bench_task* t = (bench_task*)arg;
  uint64_t s = 0, nkv = 0;
  uint64_t* tr = NULL; uint8_t* fl = NULL; uint32_t *eo = NULL, *ko = NULL, *vo = NULL, *rs = NULL;
  uint8_t *keys = NULL, *vals = NULL;
  if (t->mode == 1) {
    tr = malloc(16384 * 8); fl = malloc(16384); eo = malloc(16384 * 4);
    ko = malloc(16385 * 4); vo = malloc(16385 * 4); rs = malloc(16384 * 4);
    keys = malloc(1 << 20); vals = malloc(1 << 20);
  }
  for (int r = 0; r < t->reps; r++) {
    for (uint32_t b = (uint32_t)t->tid; b < t->n; b += (uint32_t)t->nth) {
      const uint8_t* blk = t->blocks + t->off[b];
      if (t->mode == 0) {
        s ^= t->fmt == FMT_ROW ? orc_rowblk_scan_checksum(blk, t->len[b], t->flags, &nkv)
                               : orc_colblk_scan_checksum(blk, t->len[b], t->fmt, &nkv);
      } else {
        orc_block_out o = {0, 0, 0, 0, tr, fl, eo, ko, vo, keys, vals, rs};
        if (t->len[b] <= 65536) decode_block(blk, t->len[b], t->fmt, t->flags, &o);
        s += o.n_kv + (o.key_bytes ? keys[0] : 0) + (o.val_bytes ? vals[o.val_bytes - 1] : 0);
      }
    }
  }
  free(tr); free(fl); free(eo); free(ko); free(vo); free(rs); free(keys); free(vals);
  t->sum = s;
  return NULL;
}

uint64_t orc_bench(const uint8_t* blocks, const uint64_t* off, const uint32_t* len, uint32_t n, uint32_t fmt,
                   uint32_t flags, int n_threads, int mode, int reps, double* seconds) {
  if (n_threads < 1) n_threads = 1;
  if (n_threads > 256) n_threads = 256;
  bench_task tasks[256];
  pthread_t th[256];
  struct timespec a, b;
  clock_gettime(CLOCK_MONOTONIC, &a);
  for (int i = 0; i < n_threads; i++) {
    tasks[i] = (bench_task){blocks, off, len, n, fmt, flags, mode, reps, i, n_threads, 0};
    pthread_create(&th[i], NULL, bench_worker, &tasks[i]);
  }
  uint64_t s = 0;
  for (int i = 0; i < n_threads; i++) { pthread_join(th[i], NULL); s ^= tasks[i].sum; }
  clock_gettime(CLOCK_MONOTONIC, &b);
  *seconds = (double)(b.tv_sec - a.tv_sec) + 1e-9 * (double)(b.tv_nsec - a.tv_nsec);
  return s;
}

/* Single-column decode for the per-codec known-answer tests
 * (tests/test_oracle_codecs.py), over the column bytes the reference's own
 * codec tests print (sstable/colblk/testdata/{uints,raw_bytes,bitmap,
 * prefix_bytes}): `off` is the column's start in `buf` (the tests' `offset=`
 * argument), `rows` its row count.
 *   kind 0  UnsafeUints.At (uints.go:41-67)            out[i] = value
 *   kind 1  RawBytes.At (raw_bytes.go:127-141)         out[2i], out[2i+1] = slice [lo, hi) in buf
 *   kind 2  Bitmap.At (bitmap.go:29-127)               out[i] = bit
 *   kind 3  PrefixBytes.At (prefix_bytes.go:286-386)   keys[] = the rows' keys back to back,
 *                                                      out[i] = end offset of key i in keys[]
 * Returns the column's end offset (the decoder's), or -1 when the decoder
 * rejects the bytes. */
int64_t orc_col_decode(const uint8_t* buf, uint64_t len, uint64_t off, uint32_t rows, int kind, uint64_t* out,
                       uint8_t* keys, uint64_t keys_cap) {
  coldec c;
  memset(&c, 0, sizeof(c));
  c.d.b = buf;
  c.d.len = len;
  c.d.rows = rows;
  uint64_t end = 0;
  if (kind == 0) {
    ucol u;
    if (!dec_uints(&c.d, off, rows, &u, &end) || end > len) return -1;
    for (uint32_t i = 0; i < rows; i++) out[i] = u_at(&c.d, &u, i);
  } else if (kind == 1) {
    rbcol r;
    if (!dec_rawbytes(&c.d, off, rows, &r, &end)) return -1;
    for (uint32_t i = 0; i < rows; i++)
      if (!rb_slice(&c, &r, i, &out[2 * i], &out[2 * i + 1])) return -1;
  } else if (kind == 2) {
    bmcol m;
    if (!dec_bitmap(&c.d, off, rows, &m, &end)) return -1;
    for (uint32_t i = 0; i < rows; i++) out[i] = (uint64_t)bm_at(&c.d, &m, i);
  } else if (kind == 3) {
    c.schema = FMT_COL_DEFAULT;
    if (!dec_prefix(&c.d, off, rows, &c.keys, &end)) return -1;
    c.shared_len = (uint32_t)u_at(&c.d, &c.keys.rb.off, 0);
    c.data_len = (uint32_t)u_at(&c.d, &c.keys.rb.off, c.keys.rb.n);
    uint64_t n = 0;
    for (uint32_t i = 0; i < rows; i++) {
      uint64_t bl, bh, sl, sh;
      if (!pb_parts(&c, i, &bl, &bh, &sl, &sh)) return -1;
      const uint64_t parts[3][2] = {{c.keys.rb.data, c.keys.rb.data + c.shared_len}, {bl, bh}, {sl, sh}};
      for (int k = 0; k < 3; k++) {
        const uint64_t m = parts[k][1] - parts[k][0];
        if (n + m > keys_cap) return -1;
        memcpy(keys + n, buf + parts[k][0], m);
        n += m;
      }
      out[i] = n;
    }
  } else {
    return -1;
  }
  return (int64_t)end;
}
