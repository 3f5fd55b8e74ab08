/*
 * oracle/rowblk_oracle.c — TEST INFRASTRUCTURE ONLY.
 *
 * A plain-C, sequential restatement of Pebble's row-oriented data-block reader,
 * used as the parity checker for the HIP decoder.  Only tests/, the smoke() of
 * __graft_entry__.py and bench.py's cpu_baseline leg may load this; the product
 * path (pebble_amd/) never does.
 *
 * Pinned by: the golden block bytes of sstable/rowblk/rowblk_writer_test.go:51-55,
 * 104-114; the data blocks of sstable/testdata/h-no-compression-sst/000012.sst
 * checked against sstable/testdata/h.txt; sstable/rowblk/testdata/rowblk_iter;
 * the varint KAT of sstable/rowblk/unsafe_test.go:21-42 (tests/test_oracle_rowblk.py).
 *
 * Functions restated (cockroachdb/pebble, paths relative to the repo root):
 *   orc_decode_varint   sstable/rowblk/rowblk_iter.go:2020-2038 (uint32 arithmetic:
 *                       a 5th byte contributes uint32(e)<<28, high bits dropped)
 *   orc_rowblk_decode   Iter.Init :241-276, readFirstKey :418-485, readEntry :333-416,
 *                       First :1061-1087, Next :1145-1201, decodeInternalKey :487-504,
 *                       Valid :1666-1668, decodeRestart :1092-1096,
 *                       value classification :1192-1199 with block.ValuePrefix
 *                       (sstable/block/kv.go:14-41), TrailerObsoleteMask
 *                       (sstable/rowblk/rowblk_writer.go:30-42)
 *
 * Where Go would read outside the block (unsafe pointer arithmetic) or panic,
 * the oracle reports a corruption status and emits no KVs for the block; the
 * device decoder does the same.
 */
#define _POSIX_C_SOURCE 200809L
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "oracle.h"

static const uint64_t TRAILER_OBSOLETE_MASK = (((uint64_t)1 << 56) - 1) << 8 | 191u;
static const uint64_t TRAILER_OBSOLETE_BIT = 64u;
static const uint64_t KIND_INVALID = 191u;
static const uint64_t KIND_SET = 1u;

static uint32_t le32(const uint8_t* p) {
  return (uint32_t)p[0] | (uint32_t)p[1] << 8 | (uint32_t)p[2] << 16 | (uint32_t)p[3] << 24;
}
static uint64_t le64(const uint8_t* p) { return (uint64_t)le32(p) | (uint64_t)le32(p + 4) << 32; }

/* rowblk_iter.go:2020-2038.  Returns bytes consumed (1..5); 0 if it would read
 * past `end`. */
int orc_decode_varint(const uint8_t* p, const uint8_t* end, uint32_t* v) {
  uint32_t r = 0;
  for (int i = 0; i < 5; i++) {
    if (p + i >= end) return 0;
    uint8_t b = p[i];
    if (i == 4) { r |= (uint32_t)b << 28; *v = r; return 5; }
    if (b < 128) { r |= (uint32_t)b << (7 * i); *v = r; return i + 1; }
    r |= (uint32_t)(b & 0x7f) << (7 * i);
  }
  return 0;
}


/* Comparer.Split for the synthetic-suffix transform (PBL_SPLIT_*):
 * base.DefaultSplit (whole key), testkeys (before the last '@',
 * internal/testkeys/testkeys.go:144-150), cockroachkvs.Split (last byte = version
 * length, cockroachkvs/cockroachkvs.go:298-309; a length past the key is taken as
 * 0 where Go would panic). */
uint64_t orc_split(const uint8_t* k, uint64_t n, int split) {
  if (split == 1) {
    for (uint64_t i = n; i > 0; i--)
      if (k[i - 1] == '@') return i - 1;
    return n;
  }
  if (split == 2) {
    if (n == 0) return 0;
    uint64_t v = k[n - 1];
    return v <= n ? n - v : 0;
  }
  return n;
}

/*
 * Sequential decode of one row block exactly as rowblk.Iter First/Next sees it,
 * under blockiter.Transforms `t` (NULL = NoTransforms):
 *   Init :259-263           fullKey starts as the synthetic prefix
 *   readEntry :400-403      shared += PrefixLen(); fullKey = fullKey[:shared] ++ unshared
 *   Next :1168-1191         the internal key is decoded from prefix ++ key: the
 *                           len >= 8 test, the trailer and the obsolete bit all see
 *                           the prefixed key; hidden points are skipped before the
 *                           value is looked at; SyntheticSeqNum via SetSeqNum; the
 *                           synthetic suffix replaces key[Split(prefix ++ key):]
 *   Next :1192-1199         value classification by the (possibly new) kind
 * RawIter (FLAG_RAW_KEYS) takes no transforms.
 */
static int rowblk_decode_impl(const uint8_t* blk, uint64_t len, uint32_t flags, const orc_transforms* t,
                              orc_block_out* o) {
  o->n_kv = o->key_bytes = o->val_bytes = o->n_restarts = 0;
  if (flags & FLAG_RAW_KEYS) t = NULL;
  const uint64_t P = t ? t->prefix_len : 0;
  if (len < 4) return CORRUPT_BOUNDS;
  const uint8_t* end = blk + len;
  int32_t num_restarts = (int32_t)le32(blk + len - 4);       /* :248 */
  if (num_restarts == 0) return CORRUPT_NO_RESTARTS;         /* :249-251 */
  if (num_restarts < 0) return CORRUPT_BOUNDS;
  int64_t restarts = (int64_t)len - 4 * (1 + (int64_t)num_restarts); /* :256 */
  if (restarts < 0) return CORRUPT_BOUNDS; /* Go: Valid() never true, table unreadable */
  if (restarts > 0 && !(flags & FLAG_RAW_KEYS)) {            /* readFirstKey :418-485 */
    if (blk[0] != 0) return CORRUPT_FIRST_KEY;                /* :429-434 */
    uint32_t unshared, vl;
    int n1 = orc_decode_varint(blk + 1, end, &unshared);
    if (!n1) return CORRUPT_BOUNDS;
    int n2 = orc_decode_varint(blk + 1 + n1, end, &vl);
    if (!n2) return CORRUPT_BOUNDS;
    if (unshared < 8) return CORRUPT_FIRST_KEY;               /* :471-476 (before the prefix) */
  }
  const uint8_t* rtab = blk + restarts;

  /* First pass validates and counts; second pass writes.  Corrupt => no KVs. */
  uint8_t* full = NULL;
  uint64_t full_cap = 0, full_len = 0;
  int status = OK;
  for (int pass = 0; pass < 2 && status == OK; pass++) {
    int write = pass == 1;
    uint64_t nkv = 0, kb = 0, vb = 0;
    full_len = P;
    int64_t offset = 0;
    uint32_t ri = 0; /* restart cursor for the restart flag */
    while (offset >= 0 && offset < restarts) {                /* Valid :1666 */
      const uint8_t* p = blk + offset;
      uint32_t shared, unshared, vlen;
      int a = orc_decode_varint(p, end, &shared);
      if (!a) { status = CORRUPT_BOUNDS; break; }
      int b = orc_decode_varint(p + a, end, &unshared);
      if (!b) { status = CORRUPT_BOUNDS; break; }
      int c = orc_decode_varint(p + a + b, end, &vlen);
      if (!c) { status = CORRUPT_BOUNDS; break; }
      const uint8_t* kp = p + a + b + c;
      if ((uint64_t)(end - kp) < (uint64_t)unshared) { status = CORRUPT_BOUNDS; break; }
      const uint8_t* vp = kp + unshared;
      if ((uint64_t)(end - vp) < (uint64_t)vlen) { status = CORRUPT_BOUNDS; break; }
      /* fullKey = append(fullKey[:shared + P], unshared...) :400-403 */
      if ((uint64_t)shared + P > full_len) { status = CORRUPT_BOUNDS; break; }
      uint64_t klen = P + (uint64_t)shared + unshared;
      if (klen > full_cap) {
        uint64_t nc = full_cap ? full_cap : 64;
        while (nc < klen) nc *= 2;
        uint8_t* nf = (uint8_t*)realloc(full, nc);
        if (!nf) { status = CORRUPT_BOUNDS; break; }
        full = nf; full_cap = nc;
      }
      if (P) memcpy(full, t->prefix, P); /* full[:P] is always the prefix (Init :259-263) */
      memcpy(full + P + shared, kp, unshared);
      full_len = klen;
      const int64_t this_off = offset;
      offset = (int64_t)(vp - blk) + vlen;                     /* nextOffset :415 */
      /* decodeInternalKey :487-504 on prefix ++ key */
      uint64_t trailer, ukl, kout_len = 0;
      uint8_t fl = 0;
      if (flags & FLAG_RAW_KEYS) {                             /* RawIter.readEntry :1784-1794 */
        trailer = 0;
        ukl = klen;
      } else if (klen >= 8) {
        uint64_t raw = le64(full + klen - 8);
        if (raw & TRAILER_OBSOLETE_BIT) fl |= KV_OBSOLETE;
        trailer = raw & TRAILER_OBSOLETE_MASK;
        ukl = klen - 8;
        if (t && t->hide && (raw & TRAILER_OBSOLETE_BIT)) continue;   /* hiddenPoint: goto start */
        if (t && t->seq) trailer = t->seq << 8 | (trailer & 0xff);   /* SetSeqNum */
      } else {
        trailer = KIND_INVALID;
        ukl = 0;
        fl |= KV_INVALID_KEY;
      }
      uint64_t split_at = ukl; /* user key = full[:split_at] ++ (suffix | full[split_at:ukl]) */
      kout_len = ukl;
      if (t && t->suffix_len && klen >= 8) {
        split_at = orc_split(full, ukl, t->split);
        kout_len = split_at + t->suffix_len;
      }
      /* value classification :1192-1199 */
      const uint8_t* v = vp;
      uint64_t vl = vlen;
      if ((flags & FLAG_VALUE_PREFIX) && !(flags & FLAG_RAW_KEYS) && (trailer & 0xff) == KIND_SET) {
        if (vl == 0) { status = CORRUPT_BOUNDS; break; } /* Go: i.val[0] panics */
        uint8_t prefix = v[0];
        if ((prefix & 0xC0) == 0 || (flags & FLAG_NO_VALUER)) {
          v++; vl--;
        } else if ((prefix & 0xC0) == 0x80) {
          fl |= KV_VALBLK;
        } else {
          fl |= KV_BLOB; /* 0x40; 0xC0 is undefined and routed to the valuer too */
        }
      }
      /* restart flag: entry offset equals a (masked) restart offset */
      while (ri < (uint32_t)num_restarts && (int64_t)(le32(rtab + 4 * ri) & 0x7fffffffu) < this_off) ri++;
      if (ri < (uint32_t)num_restarts && (int64_t)(le32(rtab + 4 * ri) & 0x7fffffffu) == this_off) {
        fl |= KV_RESTART;
        if (le32(rtab + 4 * ri) & 0x80000000u) fl |= KV_RESTART_SAMEPFX;
      }
      if (write) {
        if (o->trailer) o->trailer[nkv] = trailer;
        if (o->kv_flags) o->kv_flags[nkv] = fl;
        if (o->entry_off) o->entry_off[nkv] = (uint32_t)this_off;
        if (o->key_off) o->key_off[nkv] = (uint32_t)kb;
        if (o->val_off) o->val_off[nkv] = (uint32_t)vb;
        if (o->keys && split_at) memcpy(o->keys + kb, full, split_at);
        if (o->keys && kout_len > split_at) {
          if (t && t->suffix_len && klen >= 8) memcpy(o->keys + kb + split_at, t->suffix, t->suffix_len);
          else memcpy(o->keys + kb + split_at, full + split_at, kout_len - split_at);
        }
        if (o->vals && vl) memcpy(o->vals + vb, v, vl);
      }
      nkv++;
      kb += kout_len;
      vb += vl;
    }
    if (status != OK) break;
    if (write) {
      if (o->key_off) o->key_off[nkv] = (uint32_t)kb;
      if (o->val_off) o->val_off[nkv] = (uint32_t)vb;
      if (o->restarts)
        for (int32_t r = 0; r < num_restarts; r++) o->restarts[r] = le32(rtab + 4 * r);
    }
    o->n_kv = nkv;
    o->key_bytes = kb;
    o->val_bytes = vb;
    o->n_restarts = (uint64_t)num_restarts;
  }
  free(full);
  if (status != OK) o->n_kv = o->key_bytes = o->val_bytes = o->n_restarts = 0;
  return status;
}

int orc_rowblk_decode(const uint8_t* blk, uint64_t len, uint32_t flags, orc_block_out* o) {
  return rowblk_decode_impl(blk, len, flags, NULL, o);
}

int orc_rowblk_decode_tf(const uint8_t* blk, uint64_t len, uint32_t flags, const orc_transforms* t,
                         orc_block_out* o) {
  return rowblk_decode_impl(blk, len, flags, t, o);
}

/*
 * Batch form in exactly the device layout of include/pebble_amd.h
 * (pbl_decode_out): pass NULL output arrays to size, then call again with
 * arrays.  blk_*_base have n_blocks+1 entries.
 */

int orc_rowblk_decode_batch(const uint8_t* blocks, const uint64_t* off, const uint32_t* len,
                            uint32_t n_blocks, uint32_t flags, orc_batch_out* bo) {
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
    }
    int st = orc_rowblk_decode(blocks + off[b], len[b], flags, &o);
    if (fill && st != OK) { /* corrupt block: zero KVs, offset array [0] */
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

/*
 * "Iterate-only" CPU baseline (SURVEY.md §8(d) mode i): what a Go scan does per
 * block — key materialised into a reused buffer, value zero-copy — folded into a
 * checksum so nothing is dead code.  Returns the checksum; *n_kv gets the count.
 */
uint64_t orc_rowblk_scan_checksum(const uint8_t* blk, uint64_t len, uint32_t flags, uint64_t* n_kv) {
  orc_block_out o;
  memset(&o, 0, sizeof(o));
  /* a single pass with a reused key buffer */
  uint64_t h = 1469598103934665603ull, n = 0;
  if (len < 4) return 0;
  int32_t nr = (int32_t)le32(blk + len - 4);
  if (nr <= 0) return 0;
  int64_t restarts = (int64_t)len - 4 * (1 + (int64_t)nr);
  uint8_t keybuf[4096];
  uint64_t klen_prev = 0;
  const uint8_t* end = blk + len;
  int64_t offset = 0;
  while (offset >= 0 && offset < restarts) {
    const uint8_t* p = blk + offset;
    uint32_t s, u, v;
    int a = orc_decode_varint(p, end, &s);
    int b = orc_decode_varint(p + a, end, &u);
    int c = orc_decode_varint(p + a + b, end, &v);
    if (!a || !b || !c || s > klen_prev || (uint64_t)s + u > sizeof(keybuf)) return 0;
    const uint8_t* kp = p + a + b + c;
    memcpy(keybuf + s, kp, u);
    uint64_t klen = (uint64_t)s + u;
    klen_prev = klen;
    uint64_t tr = klen >= 8 ? (le64(keybuf + klen - 8) & TRAILER_OBSOLETE_MASK) : KIND_INVALID;
    const uint8_t* vp = kp + u;
    uint64_t vl = v;
    if ((flags & FLAG_VALUE_PREFIX) && (tr & 0xff) == KIND_SET && vl) { vp++; vl--; }
    h = (h ^ tr ^ (klen >= 8 ? keybuf[0] : 0) ^ (vl ? vp[0] : 0) ^ vl) * 1099511628211ull;
    n++;
    offset = (int64_t)(kp + u - blk) + v;
  }
  (void)o;
  *n_kv = n;
  return h;
}

/*
 * CPU baseline timing (bench.py cpu_baseline leg): decode blocks [0, n) `reps`
 * times on `n_threads` pthreads, one block per task.  mode 0 = iterate-only
 * (Go semantics: key into a reused buffer, value zero-copy, checksum to keep it
 * live); mode 1 = materialize into per-thread flat arrays (the GPU contract).
 * Returns the checksum; *seconds gets the wall time.
 */
#include <pthread.h>
#include <time.h>

typedef struct {
  const uint8_t* blocks;
  const uint64_t* off;
  const uint32_t* len;
  uint32_t n, flags;
  int mode, reps, tid, nth;
  uint64_t sum;
} orc_bench_task;

static void* orc_bench_worker(void* arg) {
  orc_bench_task* t = (orc_bench_task*)arg;
  uint64_t s = 0, nkv = 0;
  /* materialize scratch: generous per-block bounds */
  uint64_t* tr = NULL; uint8_t* fl = NULL; uint32_t *eo = NULL, *ko = NULL, *vo = NULL, *rs = NULL;
  uint8_t *keys = NULL, *vals = NULL;
  if (t->mode == 1) {
    tr = malloc(16384 * 8); fl = malloc(16384); eo = malloc(16384 * 4);
    ko = malloc(16385 * 4); vo = malloc(16385 * 4); rs = malloc(16384 * 4);
    keys = malloc(1 << 20); vals = malloc(1 << 20);
  }
  for (int r = 0; r < t->reps; r++) {
    for (uint32_t b = (uint32_t)t->tid; b < t->n; b += (uint32_t)t->nth) {
      if (t->mode == 0) {
        s ^= orc_rowblk_scan_checksum(t->blocks + t->off[b], t->len[b], t->flags, &nkv);
      } else {
        orc_block_out o = {0, 0, 0, 0, tr, fl, eo, ko, vo, keys, vals, rs};
        if (t->len[b] <= 65536) orc_rowblk_decode(t->blocks + t->off[b], t->len[b], t->flags, &o);
        s += o.n_kv + (o.key_bytes ? keys[0] : 0) + (o.val_bytes ? vals[o.val_bytes - 1] : 0);
      }
    }
  }
  free(tr); free(fl); free(eo); free(ko); free(vo); free(rs); free(keys); free(vals);
  t->sum = s;
  return NULL;
}

uint64_t orc_rowblk_bench(const uint8_t* blocks, const uint64_t* off, const uint32_t* len, uint32_t n,
                          uint32_t flags, int n_threads, int mode, int reps, double* seconds) {
  if (n_threads < 1) n_threads = 1;
  if (n_threads > 256) n_threads = 256;
  orc_bench_task tasks[256];
  pthread_t th[256];
  struct timespec a, b;
  clock_gettime(CLOCK_MONOTONIC, &a);
  for (int i = 0; i < n_threads; i++) {
    tasks[i] = (orc_bench_task){blocks, off, len, n, flags, mode, reps, i, n_threads, 0};
    pthread_create(&th[i], NULL, orc_bench_worker, &tasks[i]);
  }
  uint64_t s = 0;
  for (int i = 0; i < n_threads; i++) { pthread_join(th[i], NULL); s ^= tasks[i].sum; }
  clock_gettime(CLOCK_MONOTONIC, &b);
  *seconds = (double)(b.tv_sec - a.tv_sec) + 1e-9 * (double)(b.tv_nsec - a.tv_nsec);
  return s;
}
