/*
 * minlz_oracle.c — TEST INFRASTRUCTURE ONLY (the parity checker, never the
 * product).  CPU restatement of the MinLZ block format that Pebble's
 * compression indicator 8 names (sstable/block/compression.go:192,229-230;
 * internal/compression/minlz.go:52-72 calls minlz.Decode / minlz.DecodedLen).
 *
 * The codec is a third-party dependency absent from /root/reference:
 * github.com/minio/minlz v1.0.2-0.20260119185444-845e64f85661 (go.mod:23).
 * This file restates its published block format from the project's format
 * specification as the builder recalls it; NO MinLZ-encoded bytes exist in the
 * reference to pin it, so every native MinLZ encoding here is PARITY UNPINNED.
 * The one property the reference does pin (internal/compression/
 * minlz_test.go:31-36: a MinLZ decompressor always decodes what the Snappy
 * fallback of minlzCompressor.Compress wrote, minlz.go:21-27) is pinned: a
 * block whose first byte is not 0 is a Snappy block (orc_snappy_decode).
 *
 * Block:  0x00, uvarint n (decoded length, <= 8 MiB = minlz.MaxBlockSize);
 *         n == 0 with bytes after the header: those bytes ARE the block
 *         (stored); a lone 0x00 is the empty block; a compressed block is
 *         never longer than its output (n < remaining -> corrupt).
 * Ops (tag = first byte, low 2 bits):
 *   00  literal (bit 2 = 0) / repeat (bit 2 = 1): x = tag >> 3;
 *       x < 29: len = x + 1; 29: len = 30 + b1; 30: len = 30 + LE16;
 *       31: len = 30 + LE24.  A literal copies len input bytes; a repeat
 *       copies len bytes from the last offset (initially 1).
 *   01  copy1: 2 bytes; len = ((tag >> 2) & 15) + 4, 15 -> 18 + next byte;
 *       offset = (LE16 >> 6) + 1 (1..1024).
 *   10  copy2: 3 bytes; l = tag >> 2: l <= 60 -> len = l + 4; 61 -> 64 + b;
 *       62 -> 64 + LE16; 63 -> 64 + LE24; offset = LE16(bytes 1-2) + 64.
 *   11  fused ops, v = LE32 of the 4 bytes at the tag:
 *       bit 2 = 0: copy2 with literals: 3 bytes; lits = ((v >> 3) & 3) + 1,
 *         len = ((v >> 5) & 7) + 4, offset = ((v >> 8) & 0xffff) + 64;
 *       bit 2 = 1: copy3: 4 bytes; lits = (v >> 3) & 3, l = (v >> 5) & 63
 *         (l <= 60 -> len = l + 4; 61/62/63 -> 64 + 1/2/3 extra LE bytes),
 *         offset = (v >> 11) + 65536;
 *       the literals follow the op's bytes and are emitted BEFORE the copy.
 * Every copy must have offset <= bytes decoded so far and fit the output;
 * the output must end exactly at n.  Anything else is ErrCorrupt.
 */
#include <stddef.h>
#include <stdint.h>
#include <string.h>

int64_t orc_snappy_decode(const uint8_t* src, uint64_t n, uint8_t* dst, uint64_t cap);
int64_t orc_snappy_decoded_len(const uint8_t* src, uint64_t n);

#define MINLZ_MAX_BLOCK (8u << 20)

static int mz_uvarint(const uint8_t* p, uint64_t n, uint64_t* v, uint64_t* used) {
  uint64_t x = 0;
  for (uint64_t i = 0; i < n && i < 10; i++) {
    x |= (uint64_t)(p[i] & 0x7f) << (7 * i);
    if (p[i] < 0x80) {
      *v = x;
      *used = i + 1;
      return 1;
    }
  }
  return 0;
}

/* Header of a MinLZ-form block (src[0] == 0): sets *dlen, *hdr (bytes before
 * the first op) and *stored.  0 on a corrupt header. */
static int mz_header(const uint8_t* src, uint64_t n, uint64_t* dlen, uint64_t* hdr, int* stored) {
  *stored = 0;
  if (n == 1) {  /* the empty block */
    *dlen = 0;
    *hdr = 1;
    return 1;
  }
  uint64_t v, u;
  if (!mz_uvarint(src + 1, n - 1, &v, &u) || v > MINLZ_MAX_BLOCK) return 0;
  const uint64_t rest = n - 1 - u;
  if (rest == 0) return 0;
  *hdr = 1 + u;
  if (v == 0) {
    *stored = 1;
    *dlen = rest;
    return 1;
  }
  if (v < rest) return 0;
  *dlen = v;
  return 1;
}

/* minlz.DecodedLen: -1 on a corrupt header. */
int64_t orc_minlz_decoded_len(const uint8_t* src, uint64_t n) {
  if (n == 0) return -1;
  if (src[0] != 0) return orc_snappy_decoded_len(src, n);
  uint64_t dlen, hdr;
  int stored;
  if (!mz_header(src, n, &dlen, &hdr, &stored)) return -1;
  return (int64_t)dlen;
}

/* minlz.Decode into dst (cap bytes): the decoded length or -1. */
int64_t orc_minlz_decode(const uint8_t* src, uint64_t n, uint8_t* dst, uint64_t cap) {
  if (n == 0) return -1;
  if (src[0] != 0) return orc_snappy_decode(src, n, dst, cap);
  uint64_t dlen, s;
  int stored;
  if (!mz_header(src, n, &dlen, &s, &stored) || dlen > cap) return -1;
  if (stored) {
    memcpy(dst, src + s, dlen);
    return (int64_t)dlen;
  }
  uint64_t d = 0, last = 1;
  while (s < n) {
    const uint32_t t = src[s];
    uint64_t lits = 0, lit_at = 0, len = 0, off = 0;
    switch (t & 3) {
      case 0: {
        const uint32_t x = t >> 3;
        uint64_t l;
        if (x < 29) {
          l = x + 1;
          s += 1;
        } else {
          const uint64_t nb = x - 28; /* 1..3 length bytes */
          if (s + 1 + nb > n) return -1;
          l = 0;
          for (uint64_t i = 0; i < nb; i++) l |= (uint64_t)src[s + 1 + i] << (8 * i);
          l += 30;
          s += 1 + nb;
        }
        if (t & 4) { /* repeat */
          len = l;
          off = last;
        } else {
          if (l > n - s || l > dlen - d) return -1;
          memcpy(dst + d, src + s, l);
          d += l;
          s += l;
          continue;
        }
        break;
      }
      case 1: {
        if (s + 2 > n) return -1;
        const uint32_t v = (uint32_t)src[s] | (uint32_t)src[s + 1] << 8;
        off = (v >> 6) + 1;
        len = (t >> 2) & 15;
        s += 2;
        if (len == 15) {
          if (s + 1 > n) return -1;
          len = 18 + src[s];
          s += 1;
        } else {
          len += 4;
        }
        break;
      }
      case 2: {
        if (s + 3 > n) return -1;
        const uint32_t l = t >> 2;
        off = ((uint64_t)src[s + 1] | (uint64_t)src[s + 2] << 8) + 64;
        s += 3;
        if (l <= 60) {
          len = l + 4;
        } else {
          const uint64_t nb = l - 60;
          if (s + nb > n) return -1;
          len = 0;
          for (uint64_t i = 0; i < nb; i++) len |= (uint64_t)src[s + i] << (8 * i);
          len += 64;
          s += nb;
        }
        break;
      }
      default: {
        if (t & 4) { /* copy3 */
          if (s + 4 > n) return -1;
          const uint32_t v = (uint32_t)src[s] | (uint32_t)src[s + 1] << 8 | (uint32_t)src[s + 2] << 16 |
                             (uint32_t)src[s + 3] << 24;
          lits = (v >> 3) & 3;
          const uint32_t l = (v >> 5) & 63;
          off = (uint64_t)(v >> 11) + 65536;
          s += 4;
          if (l <= 60) {
            len = l + 4;
          } else {
            const uint64_t nb = l - 60;
            if (s + nb > n) return -1;
            len = 0;
            for (uint64_t i = 0; i < nb; i++) len |= (uint64_t)src[s + i] << (8 * i);
            len += 64;
            s += nb;
          }
        } else { /* copy2 with 1..4 literals */
          if (s + 3 > n) return -1;
          const uint32_t v = (uint32_t)src[s] | (uint32_t)src[s + 1] << 8 | (uint32_t)src[s + 2] << 16;
          lits = ((v >> 3) & 3) + 1;
          len = ((v >> 5) & 7) + 4;
          off = ((v >> 8) & 0xffff) + 64;
          s += 3;
        }
        lit_at = s;
        if (lits > n - s || lits > dlen - d) return -1;
        memcpy(dst + d, src + lit_at, lits);
        d += lits;
        s += lits;
        break;
      }
    }
    if (off == 0 || off > d || len > dlen - d) return -1;
    for (uint64_t i = 0; i < len; i++) dst[d + i] = dst[d - off + i]; /* overlapping copies repeat */
    d += len;
    last = off;
  }
  return d == dlen ? (int64_t)d : -1;
}

/* ---- a test encoder (produces every op form; not minlz.Encode) --------------
 * Greedy LZ77 over a 4-byte hash chain.  `style` bits steer the choice of op
 * forms so the tests reach each decoder branch:
 *   1  prefer repeats when the match offset equals the last offset
 *   2  fuse up to 4 (copy2) / 3 (copy3) pending literals into the copy
 *   4  split long copies into chunks (exercises the short forms only)
 *   8  store (n == 0 form) when the encoding is not shorter
 * Returns the encoded length, or 0 when dst (cap bytes) is too small. */
static uint64_t put_len_lit(uint8_t* o, uint32_t kind_bits, uint64_t l) {
  /* l >= 1: the literal/repeat length header */
  if (l <= 29) {
    o[0] = (uint8_t)(((l - 1) << 3) | kind_bits);
    return 1;
  }
  uint64_t x = l - 30;
  if (x < 256) {
    o[0] = (uint8_t)((29u << 3) | kind_bits);
    o[1] = (uint8_t)x;
    return 2;
  }
  if (x < 65536) {
    o[0] = (uint8_t)((30u << 3) | kind_bits);
    o[1] = (uint8_t)x;
    o[2] = (uint8_t)(x >> 8);
    return 3;
  }
  o[0] = (uint8_t)((31u << 3) | kind_bits);
  o[1] = (uint8_t)x;
  o[2] = (uint8_t)(x >> 8);
  o[3] = (uint8_t)(x >> 16);
  return 4;
}

static uint64_t put_ext_len(uint8_t* o, uint64_t l) { /* l >= 64: 1-3 extra bytes, returns count */
  const uint64_t x = l - 64;
  o[0] = (uint8_t)x;
  if (x < 256) return 1;
  o[1] = (uint8_t)(x >> 8);
  if (x < 65536) return 2;
  o[2] = (uint8_t)(x >> 16);
  return 3;
}

static uint64_t emit_lits(uint8_t* o, const uint8_t* p, uint64_t l) {
  uint64_t w = 0;
  while (l) {
    uint64_t c = l > (30 + 0xffffffu) ? (30 + 0xffffffu) : l;
    w += put_len_lit(o + w, 0, c);
    memcpy(o + w, p, c);
    w += c;
    p += c;
    l -= c;
  }
  return w;
}

/* one copy of length len (>= 4 unless a repeat) at offset off; `pl` pending
 * literals at lp may be fused.  Returns bytes written; *fused = literals used. */
static uint64_t emit_copy(uint8_t* o, uint64_t off, uint64_t len, const uint8_t* lp, uint64_t pl, int style,
                          uint64_t* fused) {
  *fused = 0;
  if (off <= 1024 && len <= 273 && !(pl && (style & 2) && off >= 64 && off < 65600 && len <= 11)) {
    const uint64_t v = (off - 1) << 6;
    if (len <= 18) {
      o[0] = (uint8_t)(1 | ((len - 4) << 2) | (v & 0xc0));
      o[1] = (uint8_t)(v >> 8);
      return 2;
    }
    o[0] = (uint8_t)(1 | (15 << 2) | (v & 0xc0));
    o[1] = (uint8_t)(v >> 8);
    o[2] = (uint8_t)(len - 18);
    return 3;
  }
  if (off >= 64 && off < 65600) {
    const uint64_t ov = off - 64;
    if (pl && (style & 2) && len <= 11) { /* fused copy2 */
      const uint64_t fl = pl;
      const uint32_t v = 3u | (uint32_t)((fl - 1) << 3) | (uint32_t)((len - 4) << 5) | (uint32_t)(ov << 8);
      o[0] = (uint8_t)v;
      o[1] = (uint8_t)(v >> 8);
      o[2] = (uint8_t)(v >> 16);
      memcpy(o + 3, lp, fl);
      *fused = fl;
      return 3 + fl;
    }
    uint64_t w;
    if (len <= 64) {
      o[0] = (uint8_t)(2 | ((len - 4) << 2));
      w = 3;
      o[1] = (uint8_t)ov;
      o[2] = (uint8_t)(ov >> 8);
    } else {
      uint8_t ext[3];
      const uint64_t nb = put_ext_len(ext, len);
      o[0] = (uint8_t)(2 | ((60 + nb) << 2));
      o[1] = (uint8_t)ov;
      o[2] = (uint8_t)(ov >> 8);
      memcpy(o + 3, ext, nb);
      w = 3 + nb;
    }
    return w;
  }
  /* copy3 (offset >= 65536, or >= 1025 and < 64 cannot happen) */
  const uint64_t ov = off - 65536;
  const uint64_t fl = pl;
  uint8_t ext[3];
  uint64_t nb = 0, lf;
  if (len <= 64) lf = len - 4;
  else {
    nb = put_ext_len(ext, len);
    lf = 60 + nb;
  }
  const uint32_t v = 7u | (uint32_t)(fl << 3) | (uint32_t)(lf << 5) | (uint32_t)(ov << 11);
  o[0] = (uint8_t)v;
  o[1] = (uint8_t)(v >> 8);
  o[2] = (uint8_t)(v >> 16);
  o[3] = (uint8_t)(v >> 24);
  memcpy(o + 4, ext, nb);
  memcpy(o + 4 + nb, lp, fl);
  *fused = fl;
  return 4 + nb + fl;
}

uint64_t orc_minlz_encode(const uint8_t* src, uint64_t n, uint8_t* dst, uint64_t cap, int style) {
  /* worst case: header 11 + literal headers; callers give cap >= n + n/16 + 64 */
  if (n > MINLZ_MAX_BLOCK || cap < n + n / 16 + 64) return 0;
  uint64_t w = 0;
  dst[w++] = 0;
  if (n == 0) return w;
  uint64_t v = n;
  do {
    dst[w++] = (uint8_t)((v & 0x7f) | (v >= 0x80 ? 0x80 : 0));
    v >>= 7;
  } while (v);
  const uint64_t hdr = w;
  enum { HB = 15 };
  static int64_t head[1 << HB];
  for (int i = 0; i < (1 << HB); i++) head[i] = -1;
  uint64_t i = 0, lit0 = 0, last = 1;
  while (i + 4 <= n) {
    const uint32_t k = (uint32_t)src[i] | (uint32_t)src[i + 1] << 8 | (uint32_t)src[i + 2] << 16 |
                       (uint32_t)src[i + 3] << 24;
    const uint32_t h = (k * 2654435761u) >> (32 - HB);
    const int64_t c = head[h];
    head[h] = (int64_t)i;
    uint64_t off = 0, len = 0;
    /* the repeat offset first (style 1), then the hash candidate */
    if ((style & 1) && i >= last && memcmp(src + i, src + i - last, 4) == 0) off = last;
    else if (c >= 0 && i - (uint64_t)c <= (65536ull + (1u << 21) - 1) && memcmp(src + c, src + i, 4) == 0)
      off = i - (uint64_t)c;
    if (!off) {
      i++;
      continue;
    }
    while (i + len < n && src[i + len] == src[i + len - off]) len++;
    if (style & 4 && len > 40) len = 40;
    /* pending literals [lit0, i) */
    uint64_t pl = i - lit0, used = 0;
    if (off == last && (style & 1)) {
      w += emit_lits(dst + w, src + lit0, pl);
      w += put_len_lit(dst + w, 4, len);
    } else {
      /* the first chunk, then whether a fused form takes the LAST pending
       * literals (copy3: up to 3; copy2 of length <= 11: up to 4) */
      uint64_t c2 = len;
      if (off <= 1024 && c2 > 273) c2 = 273;
      if (c2 > 64 + 0xffffffu) c2 = 64 + 0xffffffu;
      if (len - c2 != 0 && len - c2 < 4) c2 = len - 4;
      uint64_t keep = 0;
      if ((style & 2) && pl) {
        if (off >= 65600) keep = pl > 3 ? 3 : pl;
        else if (off >= 64 && c2 <= 11) keep = pl > 4 ? 4 : pl;
      }
      w += emit_lits(dst + w, src + lit0, pl - keep);
      uint64_t rem = len;
      while (rem) {
        w += emit_copy(dst + w, off, c2, src + i - keep, keep, style, &used);
        keep = 0;
        rem -= c2;
        c2 = rem;
        if (off <= 1024 && c2 > 273) c2 = 273;
        if (c2 > 64 + 0xffffffu) c2 = 64 + 0xffffffu;
        if (rem - c2 != 0 && rem - c2 < 4) c2 = rem - 4;
      }
    }
    last = off;
    i += len;
    lit0 = i;
    if (w + (n - i) + 16 > cap) return 0;
  }
  w += emit_lits(dst + w, src + lit0, n - lit0);
  if (w - hdr > n || ((style & 8) && w - hdr == n)) { /* stored (a compressed block is never longer than its output) */
    w = 0;
    dst[w++] = 0;
    dst[w++] = 0;
    memcpy(dst + w, src, n);
    w += n;
  }
  return w;
}
