/*
 * zstd_oracle.c — TEST INFRASTRUCTURE ONLY (the parity checker for the device
 * zstd decoder; never linked into the product).
 *
 * Pebble decompresses zstd blocks through github.com/DataDog/zstd v1.5.7 (a cgo
 * wrapper of facebook/zstd 1.5.7; /root/reference/go.mod:4), absent here:
 *   zstdDecompressor.DecompressInto (internal/compression/zstd_cgo.go:86-108):
 *     skip the uvarint decoded length Pebble prefixes (Compress, :45-66),
 *     ZSTD_decompressDCtx into a buffer of exactly that length, and require the
 *     decoded size to equal it.
 * This file restates the published Zstandard format (RFC 8878) that library
 * decodes: frames (§3.1.1: header, blocks, content checksum), skippable frames,
 * raw / RLE / compressed blocks (§3.1.1.2), the literals section with its
 * Huffman tables and 1 or 4 streams (§3.1.1.3.1, §4.2), the sequences section
 * with predefined / RLE / FSE / repeat tables (§3.1.1.3.2, §4.1), repeat
 * offsets (§3.1.2.5) and sequence execution (§3.1.1.4).  Dictionaries are out
 * of scope (Pebble uses none): a frame naming a dictionary is unsupported.
 *
 * Parity pinning: tests/test_oracle_zstd.py checks this restatement against
 * the reference's zstd table (sstable/testdata/h-zstd-compression-sst/000004.sst
 * decodes to h.txt) and against frames made by the zstd library in pyarrow
 * (facebook/zstd) at several levels, and its XXH64 against the xxhash package.
 */
#include <stdint.h>
#include <string.h>

#define ZE_CORRUPT (-1)
#define ZE_UNSUPPORTED (-2)
#define ZE_DST_SMALL (-3)

/* ---- XXH64 (content checksum, RFC 8878 §3.1.1: low 32 bits, seed 0) ---- */
static const uint64_t P1 = 11400714785074694791ull, P2 = 14029467366897019727ull, P3 = 1609587929392839161ull,
                      P4 = 9650029242287828579ull, P5 = 2870177450012600261ull;
static uint64_t rotl(uint64_t x, int r) { return (x << r) | (x >> (64 - r)); }
static uint64_t rd64(const uint8_t* p) {
  uint64_t v = 0;
  for (int i = 0; i < 8; i++) v |= (uint64_t)p[i] << (8 * i);
  return v;
}
static uint32_t rd32(const uint8_t* p) { return p[0] | (uint32_t)p[1] << 8 | (uint32_t)p[2] << 16 | (uint32_t)p[3] << 24; }
static uint64_t xround(uint64_t acc, uint64_t in) { return rotl(acc + in * P2, 31) * P1; }
static uint64_t xmerge(uint64_t acc, uint64_t v) { return (acc ^ xround(0, v)) * P1 + P4; }

uint64_t orc_xxh64(const uint8_t* p, uint64_t n, uint64_t seed) {
  const uint8_t* end = p + n;
  uint64_t h;
  if (n >= 32) {
    uint64_t v1 = seed + P1 + P2, v2 = seed + P2, v3 = seed, v4 = seed - P1;
    while (p + 32 <= end) {
      v1 = xround(v1, rd64(p));
      v2 = xround(v2, rd64(p + 8));
      v3 = xround(v3, rd64(p + 16));
      v4 = xround(v4, rd64(p + 24));
      p += 32;
    }
    h = rotl(v1, 1) + rotl(v2, 7) + rotl(v3, 12) + rotl(v4, 18);
    h = xmerge(h, v1);
    h = xmerge(h, v2);
    h = xmerge(h, v3);
    h = xmerge(h, v4);
  } else {
    h = seed + P5;
  }
  h += n;
  while (p + 8 <= end) {
    h ^= xround(0, rd64(p));
    h = rotl(h, 27) * P1 + P4;
    p += 8;
  }
  if (p + 4 <= end) {
    h ^= (uint64_t)rd32(p) * P1;
    h = rotl(h, 23) * P2 + P3;
    p += 4;
  }
  while (p < end) {
    h ^= (*p) * P5;
    h = rotl(h, 11) * P1;
    p++;
  }
  h ^= h >> 33;
  h *= P2;
  h ^= h >> 29;
  h *= P3;
  h ^= h >> 32;
  return h;
}

static int highbit32(uint32_t v) { return 31 - __builtin_clz(v); }

/* ---- backward bitstream (§4.1: read from the end, marker bit first) ---- */
typedef struct {
  const uint8_t* p;
  int64_t pos; /* unread bits are [0, pos); reads past 0 yield zeros */
} BitR;

static int br_init(BitR* b, const uint8_t* p, uint64_t n) {
  if (n == 0 || p[n - 1] == 0) return -1;
  b->p = p;
  b->pos = (int64_t)(8 * n) - 8 + highbit32(p[n - 1]);
  return 0;
}
static uint64_t br_peek(const BitR* b, int k) { /* bits [pos-k, pos), MSB = bit pos-1 */
  uint64_t v = 0;
  for (int i = 0; i < k; i++) {
    const int64_t bit = b->pos - k + i;
    if (bit >= 0) v |= (uint64_t)((b->p[bit >> 3] >> (bit & 7)) & 1) << i;
  }
  return v;
}
static uint64_t br_read(BitR* b, int k) {
  const uint64_t v = br_peek(b, k);
  b->pos -= k;
  return v;
}

/* ---- FSE tables (§4.1.1) ---- */
typedef struct {
  uint8_t sym, nb;
  uint16_t base;
} FseEnt;
typedef struct {
  int al; /* accuracy log */
  FseEnt t[1 << 9];
} FseTab;

static int fse_build(FseTab* T, const int16_t* norm, int nsym, int al) {
  const int size = 1 << al;
  int high = size - 1;
  uint16_t next[256];
  T->al = al;
  for (int s = 0; s < nsym; s++) {
    if (norm[s] == -1) {
      T->t[high--].sym = (uint8_t)s;
      next[s] = 1;
    } else {
      next[s] = (uint16_t)norm[s];
    }
  }
  int pos = 0;
  const int step = (size >> 1) + (size >> 3) + 3, mask = size - 1;
  for (int s = 0; s < nsym; s++)
    for (int i = 0; i < norm[s]; i++) {
      T->t[pos].sym = (uint8_t)s;
      do pos = (pos + step) & mask;
      while (pos > high);
    }
  if (pos != 0) return -1;
  for (int u = 0; u < size; u++) {
    const int s = T->t[u].sym;
    const uint32_t x = next[s]++;
    const int nb = al - highbit32(x);
    T->t[u].nb = (uint8_t)nb;
    T->t[u].base = (uint16_t)((x << nb) - size);
  }
  return 0;
}

/* bits [bit, bit+k) of a forward little-endian bitstream; zeros past its end */
static uint64_t fwd_peek(const uint8_t* p, uint64_t n, uint64_t bit, int k) {
  uint64_t v = 0;
  for (int i = 0; i < k; i++) {
    const uint64_t q = bit + i;
    if (q < 8 * n) v |= (uint64_t)((p[q >> 3] >> (q & 7)) & 1) << i;
  }
  return v;
}

/* FSE_readNCount (§4.1.1): the table description, bits read forward.  Returns
   bytes used, or -1. */
static int64_t fse_read_desc(FseTab* T, const uint8_t* src, uint64_t n, int max_al, int max_sym) {
  uint64_t bit = 0;
  int16_t norm[256];
  int al = (int)fwd_peek(src, n, bit, 4) + 5;
  bit += 4;
  if (al > max_al) return -1;
  int remaining = (1 << al) + 1, threshold = 1 << al, nbits = al + 1, s = 0;
  while (remaining > 1 && s <= max_sym) {
    const int max = (2 * threshold - 1) - remaining;
    int v;
    const int low = (int)fwd_peek(src, n, bit, nbits - 1);
    if (low < max) {
      v = low;
      bit += nbits - 1;
    } else {
      v = (int)fwd_peek(src, n, bit, nbits);
      if (v >= threshold) v -= max;
      bit += nbits;
    }
    const int prob = v - 1;
    remaining -= prob < 0 ? -prob : prob;
    norm[s++] = (int16_t)prob;
    if (prob == 0) {
      for (;;) {
        const int r = (int)fwd_peek(src, n, bit, 2);
        bit += 2;
        for (int i = 0; i < r && s <= max_sym; i++) norm[s++] = 0;
        if (r != 3) break;
      }
    }
    while (remaining < threshold && nbits > 1) {
      nbits--;
      threshold >>= 1;
    }
  }
  if (remaining != 1 || bit > 8 * n || s > max_sym + 1) return -1;
  if (fse_build(T, norm, s, al)) return -1;
  return (int64_t)((bit + 7) / 8);
}

/* ---- predefined distributions and code tables (§3.1.1.3.2.2) ---- */
static const int16_t kLLDef[36] = {4, 3, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 1, 1, 1, 2, 2,
                                   2, 2, 2, 2, 2, 2, 2, 3, 2, 1, 1, 1, 1, 1, -1, -1, -1, -1};
static const int16_t kMLDef[53] = {1, 4, 3, 2, 2, 2, 2, 2, 2, 1, 1, 1, 1, 1, 1, 1, 1, 1,
                                   1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1,
                                   1, 1, 1, 1, 1, 1, 1, 1, 1, 1, -1, -1, -1, -1, -1, -1, -1};
static const int16_t kOFDef[29] = {1, 1, 1, 1, 1, 1, 2, 2, 2, 1, 1, 1, 1, 1, 1,
                                   1, 1, 1, 1, 1, 1, 1, 1, 1, -1, -1, -1, -1, -1};
static const uint32_t kLLBase[36] = {0,  1,  2,  3,  4,  5,  6,   7,   8,   9,   10,   11,   12,   13,    14,    15,   16, 18,
                                     20, 22, 24, 28, 32, 40, 48, 64, 128, 256, 512, 1024, 2048, 4096, 8192, 16384, 32768, 65536};
static const uint8_t kLLBits[36] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0,  0,  1,  1,
                                    1, 1, 2, 2, 3, 3, 4, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16};
static const uint32_t kMLBase[53] = {3,  4,  5,  6,  7,  8,  9,  10, 11,  12,  13,  14,  15,   16,   17,   18,    19,    20,
                                     21, 22, 23, 24, 25, 26, 27, 28, 29,  30,  31,  32,  33,   34,   35,   37,    39,    41,
                                     43, 47, 51, 59, 67, 83, 99, 131, 259, 515, 1027, 2051, 4099, 8195, 16387, 32771, 65539};
static const uint8_t kMLBits[53] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0,  0,  0,  0,  0,  0,  0,  0, 0,
                                    0, 0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 3, 3, 4, 4, 5, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16};

/* ---- Huffman (§4.2) ---- */
typedef struct {
  int log; /* 0 = no table yet */
  uint8_t sym[1 << 11], nb[1 << 11];
} HufTab;

/* The tree description at src; returns bytes used or -1. */
static int64_t huf_read(HufTab* H, const uint8_t* src, uint64_t n) {
  if (n < 1) return -1;
  uint8_t w[256];
  int nw = 0;
  int64_t used;
  const int hb = src[0];
  if (hb >= 128) {
    nw = hb - 127;
    used = 1 + (nw + 1) / 2;
    if ((uint64_t)used > n) return -1;
    for (int i = 0; i < nw; i++) w[i] = (i & 1) ? (src[1 + i / 2] & 15) : (src[1 + i / 2] >> 4);
  } else {
    used = 1 + hb;
    if ((uint64_t)used > n || hb == 0) return -1;
    FseTab T;
    const int64_t d = fse_read_desc(&T, src + 1, hb, 6, 255);
    if (d < 0 || d >= hb) return -1;
    BitR b;
    if (br_init(&b, src + 1 + d, hb - d)) return -1;
    uint32_t s1 = (uint32_t)br_read(&b, T.al), s2 = (uint32_t)br_read(&b, T.al);
    for (;;) {
      if (nw > 253) return -1;
      w[nw++] = T.t[s1].sym;
      s1 = T.t[s1].base + (uint32_t)br_read(&b, T.t[s1].nb);
      if (b.pos < 0) {
        w[nw++] = T.t[s2].sym;
        break;
      }
      w[nw++] = T.t[s2].sym;
      s2 = T.t[s2].base + (uint32_t)br_read(&b, T.t[s2].nb);
      if (b.pos < 0) {
        w[nw++] = T.t[s1].sym;
        break;
      }
    }
  }
  uint32_t sum = 0;
  for (int i = 0; i < nw; i++) {
    if (w[i] > 11) return -1;
    if (w[i]) sum += 1u << (w[i] - 1);
  }
  if (sum == 0) return -1;
  const int log = highbit32(sum) + 1;
  if (log > 11) return -1;
  const uint32_t rest = (1u << log) - sum;
  if (rest & (rest - 1)) return -1;
  w[nw++] = (uint8_t)(highbit32(rest) + 1);
  /* table: weight 1 first, symbols in order within a weight (HUF_readDTableX1) */
  uint32_t start[13] = {0}, cnt[13] = {0};
  for (int i = 0; i < nw; i++) cnt[w[i]]++;
  uint32_t acc = 0;
  for (int k = 1; k <= log; k++) {
    start[k] = acc;
    acc += cnt[k] << (k - 1);
  }
  for (int i = 0; i < nw; i++) {
    const int k = w[i];
    if (!k) continue;
    const uint32_t len = 1u << (k - 1);
    for (uint32_t u = 0; u < len; u++) {
      H->sym[start[k] + u] = (uint8_t)i;
      H->nb[start[k] + u] = (uint8_t)(log + 1 - k);
    }
    start[k] += len;
  }
  H->log = log;
  return used;
}

static int huf_stream(const HufTab* H, const uint8_t* src, uint64_t n, uint8_t* out, uint64_t cnt) {
  BitR b;
  if (br_init(&b, src, n)) return -1;
  for (uint64_t i = 0; i < cnt; i++) {
    const uint32_t idx = (uint32_t)br_peek(&b, H->log);
    out[i] = H->sym[idx];
    b.pos -= H->nb[idx];
  }
  return b.pos == 0 ? 0 : -1;
}

/* ---- decoder state across the blocks of a frame ---- */
typedef struct {
  HufTab huf;
  FseTab ll, of, ml;
  int have_ll, have_of, have_ml;
  uint32_t rep[3];
  uint8_t lit[1 << 17];
} ZCtx;

static int64_t seq_table(FseTab* T, int* have, int mode, const int16_t* def, int ndef, int def_al, int max_al,
                         int max_sym, const uint8_t* src, uint64_t n) {
  if (mode == 0) {
    fse_build(T, def, ndef, def_al);
    *have = 1;
    return 0;
  }
  if (mode == 1) {
    if (n < 1 || src[0] > max_sym) return -1;
    T->al = 0;
    T->t[0].sym = src[0];
    T->t[0].nb = 0;
    T->t[0].base = 0;
    *have = 1;
    return 1;
  }
  if (mode == 2) {
    const int64_t d = fse_read_desc(T, src, n, max_al, max_sym);
    if (d < 0) return -1;
    *have = 1;
    return d;
  }
  return *have ? 0 : -1;
}

/* One compressed block (§3.1.1.3) appended at dst[*pos]; matches reach back
   no further than the frame's first byte, dst[start]. */
static int comp_block(ZCtx* Z, const uint8_t* src, uint64_t n, uint8_t* dst, uint64_t cap, uint64_t start,
                      uint64_t* pos) {
  if (n < 1) return ZE_CORRUPT;
  const uint32_t b0 = src[0], ltype = b0 & 3, sf = (b0 >> 2) & 3;
  uint64_t h, regen, csize = 0;
  int streams = 1;
  if (ltype < 2) {
    if (sf == 0 || sf == 2) {
      h = 1;
      regen = b0 >> 3;
    } else if (sf == 1) {
      h = 2;
      if (n < 2) return ZE_CORRUPT;
      regen = (b0 >> 4) + ((uint64_t)src[1] << 4);
    } else {
      h = 3;
      if (n < 3) return ZE_CORRUPT;
      regen = (b0 >> 4) + ((uint64_t)src[1] << 4) + ((uint64_t)src[2] << 12);
    }
  } else {
    if (sf < 2) {
      h = 3;
      if (n < 3) return ZE_CORRUPT;
      regen = (b0 >> 4) + ((uint64_t)(src[1] & 0x3f) << 4);
      csize = (src[1] >> 6) + ((uint64_t)src[2] << 2);
      streams = sf == 0 ? 1 : 4;
    } else if (sf == 2) {
      h = 4;
      if (n < 4) return ZE_CORRUPT;
      regen = (b0 >> 4) + ((uint64_t)src[1] << 4) + ((uint64_t)(src[2] & 3) << 12);
      csize = (src[2] >> 2) + ((uint64_t)src[3] << 6);
      streams = 4;
    } else {
      h = 5;
      if (n < 5) return ZE_CORRUPT;
      regen = (b0 >> 4) + ((uint64_t)src[1] << 4) + ((uint64_t)(src[2] & 0x3f) << 12);
      csize = (src[2] >> 6) + ((uint64_t)src[3] << 2) + ((uint64_t)src[4] << 10);
      streams = 4;
    }
  }
  if (regen > (1u << 17)) return ZE_CORRUPT;
  uint64_t s = h;
  if (ltype == 0) {
    if (s + regen > n) return ZE_CORRUPT;
    memcpy(Z->lit, src + s, regen);
    s += regen;
  } else if (ltype == 1) {
    if (s + 1 > n) return ZE_CORRUPT;
    memset(Z->lit, src[s], regen);
    s += 1;
  } else {
    if (s + csize > n) return ZE_CORRUPT;
    const uint8_t* c = src + s;
    uint64_t cn = csize;
    if (ltype == 2) {
      const int64_t t = huf_read(&Z->huf, c, cn);
      if (t < 0) return ZE_CORRUPT;
      c += t;
      cn -= t;
    } else if (!Z->huf.log) {
      return ZE_CORRUPT;
    }
    if (streams == 1) {
      if (huf_stream(&Z->huf, c, cn, Z->lit, regen)) return ZE_CORRUPT;
    } else {
      if (cn < 6) return ZE_CORRUPT;
      const uint64_t l1 = c[0] | (uint32_t)c[1] << 8, l2 = c[2] | (uint32_t)c[3] << 8, l3 = c[4] | (uint32_t)c[5] << 8;
      if (6 + l1 + l2 + l3 > cn) return ZE_CORRUPT;
      const uint64_t l4 = cn - 6 - l1 - l2 - l3, seg = (regen + 3) / 4;
      if (3 * seg > regen) return ZE_CORRUPT;
      const uint8_t* q = c + 6;
      const uint64_t ls[4] = {l1, l2, l3, l4};
      for (int i = 0; i < 4; i++) {
        const uint64_t cnt = i < 3 ? seg : regen - 3 * seg;
        if (huf_stream(&Z->huf, q, ls[i], Z->lit + i * seg, cnt)) return ZE_CORRUPT;
        q += ls[i];
      }
    }
    s += csize;
  }
  /* sequences section */
  if (s >= n) return ZE_CORRUPT;
  uint64_t nseq = src[s];
  if (nseq < 128) {
    s += 1;
  } else if (nseq < 255) {
    if (s + 2 > n) return ZE_CORRUPT;
    nseq = ((nseq - 128) << 8) + src[s + 1];
    s += 2;
  } else {
    if (s + 3 > n) return ZE_CORRUPT;
    nseq = src[s + 1] + ((uint64_t)src[s + 2] << 8) + 0x7F00;
    s += 3;
  }
  uint64_t lp = 0, d = *pos;
  if (nseq > 0) {
    if (s >= n) return ZE_CORRUPT;
    const uint32_t modes = src[s++];
    if (modes & 3) return ZE_CORRUPT;
    int64_t u;
    if ((u = seq_table(&Z->ll, &Z->have_ll, modes >> 6, kLLDef, 36, 6, 9, 35, src + s, n - s)) < 0) return ZE_CORRUPT;
    s += u;
    if ((u = seq_table(&Z->of, &Z->have_of, (modes >> 4) & 3, kOFDef, 29, 5, 8, 31, src + s, n - s)) < 0)
      return ZE_CORRUPT;
    s += u;
    if ((u = seq_table(&Z->ml, &Z->have_ml, (modes >> 2) & 3, kMLDef, 53, 6, 9, 52, src + s, n - s)) < 0)
      return ZE_CORRUPT;
    s += u;
    BitR b;
    if (br_init(&b, src + s, n - s)) return ZE_CORRUPT;
    uint32_t sl = (uint32_t)br_read(&b, Z->ll.al), so = (uint32_t)br_read(&b, Z->of.al),
             sm = (uint32_t)br_read(&b, Z->ml.al);
    for (uint64_t i = 0; i < nseq; i++) {
      const uint32_t oc = Z->of.t[so].sym, mc = Z->ml.t[sm].sym, lc = Z->ll.t[sl].sym;
      if (oc > 31) return ZE_CORRUPT;
      const uint64_t ofv = (1ull << oc) + br_read(&b, oc);
      const uint64_t ml = kMLBase[mc] + br_read(&b, kMLBits[mc]);
      const uint64_t ll = kLLBase[lc] + br_read(&b, kLLBits[lc]);
      if (i + 1 < nseq) {
        sl = Z->ll.t[sl].base + (uint32_t)br_read(&b, Z->ll.t[sl].nb);
        sm = Z->ml.t[sm].base + (uint32_t)br_read(&b, Z->ml.t[sm].nb);
        so = Z->of.t[so].base + (uint32_t)br_read(&b, Z->of.t[so].nb);
      }
      uint64_t off;
      if (ofv > 3) {
        off = ofv - 3;
        Z->rep[2] = Z->rep[1];
        Z->rep[1] = Z->rep[0];
        Z->rep[0] = (uint32_t)off;
      } else {
        const uint32_t k = (uint32_t)ofv - 1 + (ll == 0);
        if (k == 0) {
          off = Z->rep[0];
        } else {
          off = k == 3 ? Z->rep[0] - 1u : Z->rep[k];
          if (k != 1) Z->rep[2] = Z->rep[1];
          Z->rep[1] = Z->rep[0];
          Z->rep[0] = (uint32_t)off;
        }
      }
      if (ll > regen - lp || d + ll + ml > cap) return ll > regen - lp ? ZE_CORRUPT : ZE_DST_SMALL;
      memcpy(dst + d, Z->lit + lp, ll);
      lp += ll;
      d += ll;
      if (off == 0 || off > d - start) return ZE_CORRUPT;
      for (uint64_t j = 0; j < ml; j++) dst[d + j] = dst[d - off + j];
      d += ml;
    }
    if (b.pos != 0) return ZE_CORRUPT;
  } else if (s != n) {
    return ZE_CORRUPT;
  }
  if (d + (regen - lp) > cap) return ZE_DST_SMALL;
  memcpy(dst + d, Z->lit + lp, regen - lp);
  *pos = d + (regen - lp);
  return 0;
}

/* ZSTD_decompressDCtx over src (frames and skippable frames back to back).
   Returns the decoded size, or ZE_*. */
int64_t orc_zstd_decompress(const uint8_t* src, uint64_t n, uint8_t* dst, uint64_t cap) {
  static __thread ZCtx Z;
  uint64_t s = 0, pos = 0;
  if (n == 0) return ZE_CORRUPT;
  while (s < n) {
    if (n - s < 4) return ZE_CORRUPT;
    const uint32_t magic = rd32(src + s);
    if ((magic & 0xFFFFFFF0u) == 0x184D2A50u) { /* skippable frame */
      if (n - s < 8) return ZE_CORRUPT;
      const uint64_t sz = rd32(src + s + 4);
      if (sz > n - s - 8) return ZE_CORRUPT;
      s += 8 + sz;
      continue;
    }
    if (magic != 0xFD2FB528u) return ZE_CORRUPT;
    s += 4;
    if (s >= n) return ZE_CORRUPT;
    const uint32_t fhd = src[s++];
    const uint32_t fcs_flag = fhd >> 6, single = (fhd >> 5) & 1, cksum = (fhd >> 2) & 1, did = fhd & 3;
    if (fhd & 8) return ZE_CORRUPT; /* reserved bit */
    uint64_t window = 0;
    if (!single) {
      if (s >= n) return ZE_CORRUPT;
      const uint32_t wd = src[s++], e = wd >> 3, m = wd & 7;
      window = (1ull << (10 + e));
      window += (window / 8) * m;
    }
    const int dl = did == 0 ? 0 : did == 1 ? 1 : did == 2 ? 2 : 4;
    if (n - s < (uint64_t)dl) return ZE_CORRUPT;
    uint64_t dict = 0;
    for (int i = 0; i < dl; i++) dict |= (uint64_t)src[s + i] << (8 * i);
    s += dl;
    if (dict) return ZE_UNSUPPORTED;
    const int fl = fcs_flag == 0 ? (single ? 1 : 0) : fcs_flag == 1 ? 2 : fcs_flag == 2 ? 4 : 8;
    if (n - s < (uint64_t)fl) return ZE_CORRUPT;
    uint64_t fcs = 0;
    for (int i = 0; i < fl; i++) fcs |= (uint64_t)src[s + i] << (8 * i);
    if (fl == 2) fcs += 256;
    s += fl;
    (void)window;
    Z.huf.log = 0;
    Z.have_ll = Z.have_of = Z.have_ml = 0;
    Z.rep[0] = 1;
    Z.rep[1] = 4;
    Z.rep[2] = 8;
    const uint64_t start = pos;
    for (;;) {
      if (n - s < 3) return ZE_CORRUPT;
      const uint32_t bh = src[s] | (uint32_t)src[s + 1] << 8 | (uint32_t)src[s + 2] << 16;
      s += 3;
      const uint32_t last = bh & 1, type = (bh >> 1) & 3, bs = bh >> 3;
      if (type == 3) return ZE_CORRUPT;
      if (type == 1) {
        if (s + 1 > n) return ZE_CORRUPT;
        if (bs > cap - pos) return ZE_DST_SMALL;
        memset(dst + pos, src[s], bs);
        pos += bs;
        s += 1;
      } else {
        if (bs > n - s) return ZE_CORRUPT;
        if (bs > (1u << 17)) return ZE_CORRUPT;
        if (type == 0) {
          if (bs > cap - pos) return ZE_DST_SMALL;
          memcpy(dst + pos, src + s, bs);
          pos += bs;
        } else {
          const int r = comp_block(&Z, src + s, bs, dst, cap, start, &pos);
          if (r) return r;
        }
        s += bs;
      }
      if (last) break;
    }
    if (fl && pos - start != fcs) return ZE_CORRUPT;
    if (cksum) {
      if (n - s < 4) return ZE_CORRUPT;
      if ((uint32_t)orc_xxh64(dst + start, pos - start, 0) != rd32(src + s)) return ZE_CORRUPT;
      s += 4;
    }
  }
  return (int64_t)pos;
}
