/*
 * physical_oracle.c — TEST INFRASTRUCTURE ONLY (the parity checker, never the
 * product).  CPU restatement of the physical-block step that precedes data-block
 * decode in Pebble's block reader (sstable/block/block.go:539-571):
 *
 *   orc_crc32c        internal/crc/crc.go:21-40: CRC-32 with the Castagnoli
 *                     polynomial (Go hash/crc32.Update) over the block bytes and
 *                     the compression-indicator byte, then Value()'s rotation
 *                     and delta: (c>>15 | c<<17) + 0xa282ead8
 *                     (ValidateChecksum, block.go:164-176)
 *   orc_snappy_*      golang/snappy (go.mod: github.com/golang/snappy), the
 *                     published Snappy block format: uvarint decoded length,
 *                     then literal / copy-1 / copy-2 / copy-4 elements; any
 *                     malformed input is an error, as snappy.Decode's
 *                     ErrCorrupt (internal/compression/snappy.go:30-46)
 *
 * xxhash64 (ChecksumTypeXXHash64, cespare/xxhash/v2) is checked in the tests with
 * the `xxhash` Python package (the XXH64 reference library) and its published
 * vectors.  Pinned by tests/test_oracle_physical.py against the stored checksums
 * of the reference's test SSTs and their KVs in h.txt.
 */
#include <stddef.h>
#include <stdint.h>
#include <string.h>

static uint32_t crc_table[256];
static int crc_ready;

static void crc_init(void) {
  for (uint32_t i = 0; i < 256; i++) {
    uint32_t c = i;
    for (int k = 0; k < 8; k++) c = (c & 1) ? (c >> 1) ^ 0x82F63B78u : c >> 1;
    crc_table[i] = c;
  }
  crc_ready = 1;
}

/* Go: crc32.Update(crc, castagnoli, p) = ^update(^crc, p) */
uint32_t orc_crc32c_update(uint32_t crc, const uint8_t* p, uint64_t n) {
  if (!crc_ready) crc_init();
  uint32_t c = ~crc;
  for (uint64_t i = 0; i < n; i++) c = crc_table[(c ^ p[i]) & 0xff] ^ (c >> 8);
  return ~c;
}

/* crc.New(b).Value() */
uint32_t orc_crc32c(const uint8_t* p, uint64_t n) {
  const uint32_t c = orc_crc32c_update(0, p, n);
  return ((c >> 15) | (c << 17)) + 0xa282ead8u;
}

static int uvarint(const uint8_t* p, uint64_t n, uint64_t* v, uint64_t* used) {
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

/* snappy.DecodedLen: -1 on a corrupt header. */
int64_t orc_snappy_decoded_len(const uint8_t* src, uint64_t n) {
  uint64_t v, u;
  if (!uvarint(src, n, &v, &u) || v > 0xffffffffu) return -1;
  return (int64_t)v;
}

/* snappy.Decode into dst (cap bytes): returns the decoded length or -1. */
int64_t orc_snappy_decode(const uint8_t* src, uint64_t n, uint8_t* dst, uint64_t cap) {
  uint64_t dlen, u;
  if (!uvarint(src, n, &dlen, &u) || dlen > cap) return -1;
  uint64_t s = u, d = 0;
  while (s < n) {
    const uint8_t t = src[s];
    uint64_t len, off;
    switch (t & 3) {
      case 0: { /* literal */
        uint64_t x = t >> 2;
        if (x < 60) {
          s += 1;
        } else {
          const uint64_t nb = x - 59; /* 1..4 length bytes */
          if (s + 1 + nb > n) return -1;
          x = 0;
          for (uint64_t i = 0; i < nb; i++) x |= (uint64_t)src[s + 1 + i] << (8 * i);
          s += 1 + nb;
        }
        len = x + 1;
        if (len > n - s || len > dlen - d) return -1;
        memcpy(dst + d, src + s, len);
        d += len;
        s += len;
        continue;
      }
      case 1:
        if (s + 2 > n) return -1;
        len = 4 + ((t >> 2) & 7);
        off = ((uint64_t)(t & 0xe0) << 3) | src[s + 1];
        s += 2;
        break;
      case 2:
        if (s + 3 > n) return -1;
        len = 1 + (t >> 2);
        off = (uint64_t)src[s + 1] | (uint64_t)src[s + 2] << 8;
        s += 3;
        break;
      default:
        if (s + 5 > n) return -1;
        len = 1 + (t >> 2);
        off = (uint64_t)src[s + 1] | (uint64_t)src[s + 2] << 8 | (uint64_t)src[s + 3] << 16 |
              (uint64_t)src[s + 4] << 24;
        s += 5;
        break;
    }
    if (off == 0 || off > d || len > dlen - d) return -1;
    for (uint64_t i = 0; i < len; i++) dst[d + i] = dst[d - off + i]; /* overlapping copies repeat */
    d += len;
  }
  return d == dlen ? (int64_t)d : -1;
}
