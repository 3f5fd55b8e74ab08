// colblk_writer.cpp — native restatement of Pebble's columnar data-block
// ENCODER (the format producer; host code), for the default key schema and the
// CockroachDB "crdb1" key schema, plus the seeded synthetic config-3 generator.
//
// The builders are restated INCREMENTALLY (row by row, with the same running
// statistics) because the reference's byte output depends on that history: e.g.
// UintBuilder keeps the delta base of a row later excluded by Finish(rows-1),
// and the data-block header keeps the maximum key length of that row.  The
// golden fixtures in tests/golden/colblk_golden.json pin the output bytes.
//
// Follows (cockroachdb/pebble, paths relative to the repo root):
//   UintBuilder          sstable/colblk/uints.go:94-141 (DetermineUintEncoding),
//                        :194-430 (Init/Reset/Set/Size/determineEncoding/Finish),
//                        :444-466 (reduceUints)
//   RawBytesBuilder      sstable/colblk/raw_bytes.go:150-240
//   PrefixBytesBuilder   sstable/colblk/prefix_bytes.go:700-1120 (Put, writePrefixCompressed,
//                        Finish, Size)
//   BitmapBuilder        sstable/colblk/bitmap.go:280-423 (Set/Size/InvertedSize/Invert/Finish)
//   BlockEncoder         sstable/colblk/block.go:205-262
//   DataBlockEncoder     sstable/colblk/data_block.go:600-790 (Init/Reset/Add/Size/Finish),
//                        with the Pebblev8 tiering columns (WithTieringColumns :594-601;
//                        internalAdd :753-761, Size :782-786, Finish :840-844): span and
//                        attribute UintBuilders InitWithDefault, the secondary blob
//                        handles a RawBytesBuilder
//   defaultKeyWriter     sstable/colblk/data_block.go:230-345
//   cockroachKeyWriter   cockroachkvs/cockroachkvs.go:575-766 (ComparePrev/WriteKey/FinishHeader)
//   KeyGenConfig         cockroachkvs/test_utils.go (RandomKVs, randRoachKey, randTimestamp)
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "../../include/pebble_amd.h"

namespace {

constexpr int kUintRowThreshold = 8;  // UintEncodingRowThreshold (uints.go:87)

inline uint8_t byte_width(uint64_t v) {  // byteWidthTable[bits.Len64(v)]
  int n = v ? 64 - __builtin_clzll(v) : 0;
  return n == 0 ? 0 : n <= 8 ? 1 : n <= 16 ? 2 : n <= 32 ? 4 : 8;
}
inline uint8_t uint_encoding(uint64_t mn, uint64_t mx, int rows) {  // DetermineUintEncoding
  uint8_t b = byte_width(mx - mn);
  if (b == 8) return 8;
  bool delta = mx >= (1ull << (b * 8));
  if (delta && rows < kUintRowThreshold) {
    uint8_t bn = byte_width(mx);
    if (rows * int(bn - b) < 8) { b = bn; delta = false; }
  }
  return uint8_t(b | (delta ? 0x80 : 0));
}
inline uint32_t align_up(uint32_t off, uint32_t a) { return (off + a - 1) & ~(a - 1); }
inline uint32_t align_zero(uint8_t* buf, uint32_t off, uint32_t a) {
  uint32_t x = align_up(off, a);
  for (uint32_t i = off; i < x; i++) buf[i] = 0;
  return x;
}
inline uint32_t uint_col_size(uint32_t rows, uint32_t off, uint8_t e) {  // uintColumnSize
  off++;
  if (e & 0x80) off += 8;
  uint32_t w = e & 0x7f;
  if (w) off = align_up(off, w);
  return off + rows * w;
}
inline void put_le(uint8_t* p, uint64_t v, int w) {
  for (int i = 0; i < w; i++) p[i] = uint8_t(v >> (8 * i));
}
inline size_t common_prefix(const uint8_t* a, size_t al, const uint8_t* b, size_t bl) {
  size_t n = std::min(al, bl), i = 0;
  while (i < n && a[i] == b[i]) i++;
  return i;
}

struct UintB {
  bool use_default = false;
  std::vector<uint64_t> elems;
  uint64_t mn = 0, mx = 0;
  uint8_t enc = 0;
  int enc_row = 0;

  void init(bool d) { use_default = d; reset(); }
  void reset() {
    if (use_default) { mn = mx = 0; std::fill(elems.begin(), elems.end(), 0); }
    else { mn = ~0ull; mx = 0; }
    enc = 0;  // uintEncodingAllZero
    enc_row = 0;
  }
  uint64_t get(int row) const { return size_t(row) < elems.size() ? elems[row] : 0; }
  void set(int row, uint64_t v) {
    if (elems.size() <= size_t(row)) {
      size_t n2 = std::max<size_t>(elems.size() << 1, 32);
      while (n2 <= size_t(row)) n2 <<= 1;
      elems.resize(n2, 0);
    }
    if (mn > v || mx < v || row < kUintRowThreshold) {
      mn = std::min(v, mn);
      mx = std::max(v, mx);
      uint8_t e = uint_encoding(mn, mx, row + 1);
      if (e != enc) { enc = e; enc_row = row; }
    }
    elems[row] = v;
  }
  void determine(int rows, uint8_t* e, uint64_t* base) const {
    if (enc_row < rows) { *e = enc; *base = mn; return; }
    size_t n = std::min<size_t>(rows, elems.size());
    uint64_t a = ~0ull, b = 0;
    for (size_t i = 0; i < n; i++) { a = std::min(a, elems[i]); b = std::max(b, elems[i]); }
    if (n == 0) a = 0;
    if (use_default) a = 0;
    *e = uint_encoding(a, b, rows);
    *base = a;
  }
  uint32_t size(int rows, uint32_t off) const {
    if (rows == 0) return off;
    uint8_t e; uint64_t b;
    determine(rows, &e, &b);
    return uint_col_size(rows, off, e);
  }
  uint32_t finish(int rows, uint32_t off, uint8_t* buf) const {
    if (rows == 0) return off;
    uint8_t e; uint64_t mnv;
    determine(rows, &e, &mnv);
    buf[off++] = e;
    uint64_t base = 0;
    if (e & 0x80) { base = mnv; put_le(buf + off, mnv, 8); off += 8; }
    uint32_t w = e & 0x7f;
    if (w == 0) return off;
    off = align_zero(buf, off, w);
    size_t n = std::min<size_t>(rows, elems.size());
    for (int i = 0; i < rows; i++) put_le(buf + off + size_t(i) * w, size_t(i) < n ? elems[i] - base : 0, w);
    return off + uint32_t(rows) * w;
  }
};

struct BitmapB {
  std::vector<uint64_t> words;
  int min_nz = 0;
  bool is_zero(int rows) const { return min_nz == 0 || rows < min_nz; }
  void set(int i) {
    if (is_zero(i + 1)) min_nz = i + 1;
    size_t w = size_t(i) >> 6;
    if (words.size() <= w) words.resize(w + 1, 0);
    words[w] |= 1ull << (i & 63);
  }
  void reset() { words.clear(); min_nz = 0; }
  static uint32_t required(int total) {
    int nw = (total + 63) >> 6, ns = (nw + 63) >> 6;
    return uint32_t(nw + ns) << 3;
  }
  uint32_t size(int rows, uint32_t off) const {
    off++;
    if (is_zero(rows)) return off;
    return align_up(off, 8) + required(rows);
  }
  uint32_t inverted_size(int rows, uint32_t off) const { return align_up(off + 1, 8) + required(rows); }
  void invert(int n) {
    min_nz = 1;
    size_t nw = size_t(n + 63) >> 6;
    words.resize(nw, 0);
    for (auto& w : words) w = ~w;
  }
  uint32_t finish(int n, uint32_t off, uint8_t* buf) {
    if (is_zero(n)) { buf[off] = 1; return off + 1; }
    buf[off++] = 0;
    off = align_zero(buf, off, 8);
    size_t nw = size_t(n + 63) >> 6;
    if (words.size() > nw) words.resize(nw);
    if (int i = n % 64; words.size() >= nw && i != 0) words[nw - 1] &= (1ull << i) - 1;
    size_t ns = (nw + 63) >> 6;
    for (size_t i = 0; i < nw; i++) put_le(buf + off + 8 * i, i < words.size() ? words[i] : 0, 8);
    off += uint32_t(nw) * 8;
    for (size_t i = 0; i < ns; i++) {
      size_t wo = i << 6;
      size_t cnt = words.size() > wo ? std::min<size_t>(64, words.size() - wo) : 0;
      uint64_t s = 0;
      for (size_t j = 0; j < cnt; j++)
        if (words[wo + j]) s |= 1ull << j;
      put_le(buf + off + 8 * i, s, 8);
    }
    return off + uint32_t(ns) * 8;
  }
};

struct RawBytesB {
  int rows = 0;
  std::vector<uint8_t> data;
  UintB offsets;
  void init() { offsets.init(false); reset(); }
  void reset() { rows = 0; data.clear(); offsets.reset(); offsets.set(0, 0); }
  void put(const uint8_t* s, size_t n) {
    data.insert(data.end(), s, s + n);
    rows++;
    offsets.set(rows, data.size());
  }
  void put_concat(const uint8_t* a, size_t an, const uint8_t* b, size_t bn) {
    data.insert(data.end(), a, a + an);
    data.insert(data.end(), b, b + bn);
    rows++;
    offsets.set(rows, data.size());
  }
  uint32_t size(int r, uint32_t off) const {
    if (r == 0) return off;
    return offsets.size(r + 1, off) + uint32_t(offsets.get(r));
  }
  uint32_t finish(int r, uint32_t off, uint8_t* buf) const {
    if (r == 0) return off;
    uint64_t dl = offsets.get(r);
    off = offsets.finish(r + 1, off, buf);
    std::memcpy(buf + off, data.data(), dl);
    return off + uint32_t(dl);
  }
  size_t len_at(int i) const { return offsets.get(i + 1) - offsets.get(i); }
};

struct PrefixSizing {
  int last_key_off = 0, offset_count = 0, block_prefix_len = 0;
  int cur_bundle_distinct_len = 0, cur_bundle_distinct_keys = 0, cur_bundle_prefix_len = 0;
  int cur_bundle_prefix_offset = 0, compressed_len = 0;
  uint8_t offset_enc = 0;
};

struct PrefixBytesB {
  int bundle_size = 16, bundle_shift = 4, n_keys = 0, completed_bundle_len = 0;
  int max_shared = (1 << 16) - 1;
  std::vector<uint8_t> data;
  std::vector<uint32_t> off;  // offsets.elems[:count]
  PrefixSizing sz[2];
  std::string last_key;

  void init(int bs) {
    bundle_size = bs;
    bundle_shift = __builtin_ctz(unsigned(bs));
    reset();
  }
  void reset() {
    n_keys = completed_bundle_len = 0;
    data.clear();
    off.clear();
    sz[0] = sz[1] = PrefixSizing{};
    last_key.clear();
  }
  int bundle_count(int rows) const { return 1 + ((rows - 1) >> bundle_shift); }
  void put(const uint8_t* key, int kl, int shared) {
    int ci = n_keys & 1;
    PrefixSizing& cur = sz[ci];
    PrefixSizing& prev = sz[ci ^ 1];
    last_key.assign(reinterpret_cast<const char*>(key), kl);
    if ((n_keys & (bundle_size - 1)) == 0) {
      if (n_keys == 0) {
        off.push_back(0);
        off.push_back(0);
        n_keys++;
        data.insert(data.end(), key, key + kl);
        off.push_back(uint32_t(data.size()));
        cur = PrefixSizing{};
        cur.last_key_off = 0;
        cur.offset_count = int(off.size());
        cur.block_prefix_len = std::min(kl, max_shared);
        cur.cur_bundle_distinct_len = kl;
        cur.cur_bundle_distinct_keys = 1;
        cur.cur_bundle_prefix_len = std::min(kl, max_shared);
        cur.cur_bundle_prefix_offset = 1;
        cur.compressed_len = kl;
        cur.offset_enc = byte_width(uint64_t(kl));  // DetermineUintEncodingNoDelta
        return;
      }
      off[prev.cur_bundle_prefix_offset] = off[prev.cur_bundle_prefix_offset - 1] + uint32_t(prev.cur_bundle_prefix_len);
      int just = prev.cur_bundle_distinct_len - (prev.cur_bundle_distinct_keys - 1) * prev.cur_bundle_prefix_len;
      completed_bundle_len += just;
      int blp = std::min(prev.block_prefix_len, shared);
      n_keys++;
      cur = PrefixSizing{};
      cur.last_key_off = int(data.size());
      cur.offset_count = int(off.size()) + 2;
      cur.block_prefix_len = blp;
      cur.cur_bundle_prefix_offset = int(off.size());
      cur.cur_bundle_prefix_len = std::min(kl, max_shared);
      cur.cur_bundle_distinct_len = kl;
      cur.cur_bundle_distinct_keys = 1;
      cur.compressed_len = completed_bundle_len + kl - (bundle_count(n_keys) - 1) * blp;
      cur.offset_enc = byte_width(uint64_t(cur.compressed_len));
      data.insert(data.end(), key, key + kl);
      off.push_back(0);  // bundle prefix placeholder
      off.push_back(uint32_t(data.size()));
      return;
    }
    n_keys++;
    if (shared == kl) {
      cur = prev;
      cur.offset_count++;
      off.push_back(off.back());
      return;
    }
    PrefixSizing c{};
    c.last_key_off = int(data.size());
    c.offset_count = prev.offset_count + 1;
    c.block_prefix_len = std::min(prev.block_prefix_len, shared);
    c.cur_bundle_distinct_len = prev.cur_bundle_distinct_len + kl;
    c.cur_bundle_distinct_keys = prev.cur_bundle_distinct_keys + 1;
    c.cur_bundle_prefix_len = std::min(prev.cur_bundle_prefix_len, shared);
    c.cur_bundle_prefix_offset = prev.cur_bundle_prefix_offset;
    c.compressed_len = completed_bundle_len + c.cur_bundle_distinct_len -
                       (c.cur_bundle_distinct_keys - 1) * c.cur_bundle_prefix_len;
    c.compressed_len -= (bundle_count(n_keys) - 1) * c.block_prefix_len;
    c.offset_enc = byte_width(uint64_t(c.compressed_len));
    cur = c;
    data.insert(data.end(), key, key + kl);
    off.push_back(uint32_t(data.size()));
  }
  uint32_t size(int rows, uint32_t o) const {
    if (rows == 0) return o;
    const PrefixSizing& s = sz[(rows & 1) ^ 1];
    o++;
    o = uint_col_size(uint32_t(s.offset_count), o, s.offset_enc);
    return o + uint32_t(s.compressed_len);
  }
  uint32_t finish(int rows, uint32_t o, uint8_t* buf) const {
    if (rows == 0) return o;
    buf[o++] = uint8_t(bundle_shift);
    const PrefixSizing& s = sz[(rows & 1) ^ 1];
    uint32_t str_off = uint_col_size(uint32_t(s.offset_count), o, s.offset_enc);
    uint32_t w = s.offset_enc;
    buf[o++] = uint8_t(s.offset_enc);
    o = align_zero(buf, o, w);
    uint8_t* dst = buf + str_off;
    auto set_off = [&](int i, uint32_t v) { put_le(buf + o + size_t(i) * w, v, int(w)); };
    if (rows <= 1) {
      uint32_t e = off[2];
      set_off(0, e); set_off(1, e); set_off(2, e);
      std::memcpy(dst, data.data(), e);
      return str_off + uint32_t(s.compressed_len);
    }
    std::memcpy(dst, data.data(), size_t(s.block_prefix_len));
    uint32_t dest = uint32_t(s.block_prefix_len);
    set_off(0, dest);
    uint32_t last_row = 0;
    int shared = 0;
    for (int i = 1; i < s.offset_count; i++) {
      uint32_t of = off[i];
      const uint8_t* sp;
      size_t sl;
      if ((i - 1) % (bundle_size + 1) == 0) {
        uint32_t a = last_row + uint32_t(s.block_prefix_len);
        uint32_t b = i == s.cur_bundle_prefix_offset ? last_row + uint32_t(s.cur_bundle_prefix_len) : of;
        sp = data.data() + a;
        sl = b - a;
        shared = s.block_prefix_len + int(sl);
      } else {
        if (of == last_row) { set_off(i, dest); continue; }
        sp = data.data() + last_row + shared;
        sl = of - (last_row + uint32_t(shared));
        last_row = of;
      }
      std::memmove(dst + dest, sp, sl);
      dest += uint32_t(sl);
      set_off(i, dest);
    }
    return str_off + uint32_t(s.compressed_len);
  }
};

struct KCmp { int prefix_len, common_prefix_len; bool prefix_equal() const { return prefix_len == common_prefix_len; } };

// ---- key writers --------------------------------------------------------------
struct KeyWriter {
  virtual ~KeyWriter() {}
  virtual int ncols() const = 0;
  virtual uint8_t col_type(int c) const = 0;
  virtual int header_size() const = 0;
  virtual KCmp compare_prev(const uint8_t* k, int kl, int prefix_len) const = 0;
  virtual void write_key(int row, const uint8_t* k, int kl, int prefix_len, int shared) = 0;
  virtual uint32_t size(int rows, uint32_t off) const = 0;
  virtual uint32_t finish(int col, int rows, uint32_t off, uint8_t* buf) = 0;
  virtual void finish_header(uint8_t* buf) const = 0;
  virtual void reset() = 0;
};

enum { kTypeBool = 1, kTypeUint = 2, kTypeBytes = 3, kTypePrefixBytes = 4 };

struct DefaultKeyWriter : KeyWriter {  // data_block.go:230-345 (comparer Split = first '@', testkeys)
  PrefixBytesB prefixes;
  RawBytesB suffixes;
  explicit DefaultKeyWriter(int bundle) { prefixes.init(bundle); suffixes.init(); }
  int ncols() const override { return 2; }
  uint8_t col_type(int c) const override { return c == 0 ? kTypePrefixBytes : kTypeBytes; }
  int header_size() const override { return 0; }
  static int split(const uint8_t* k, int kl) {
    const void* p = std::memchr(k, '@', size_t(kl));
    return p ? int(static_cast<const uint8_t*>(p) - k) : kl;
  }
  KCmp compare_prev(const uint8_t* k, int kl, int prefix_len) const override {
    KCmp c{prefix_len >= 0 ? prefix_len : split(k, kl), 0};
    if (prefixes.n_keys == 0) return c;
    const std::string& lp = prefixes.last_key;
    c.common_prefix_len = int(common_prefix(reinterpret_cast<const uint8_t*>(lp.data()), lp.size(), k,
                                            size_t(c.prefix_len)));
    return c;
  }
  void write_key(int, const uint8_t* k, int kl, int pl, int shared) override {
    prefixes.put(k, pl, shared);
    suffixes.put(k + pl, size_t(kl - pl));
  }
  uint32_t size(int rows, uint32_t off) const override { return suffixes.size(rows, prefixes.size(rows, off)); }
  uint32_t finish(int col, int rows, uint32_t off, uint8_t* buf) override {
    return col == 0 ? prefixes.finish(rows, off, buf) : suffixes.finish(rows, off, buf);
  }
  void finish_header(uint8_t*) const override {}
  void reset() override { prefixes.reset(); suffixes.reset(); }
};

struct CrdbKeyWriter : KeyWriter {  // cockroachkvs.go:575-766
  PrefixBytesB roach;
  UintB wall, logical;
  RawBytesB untyped;
  uint8_t suffix_types = 0;
  int prev_roach_len = 0;
  std::vector<uint8_t> prev_suffix;
  CrdbKeyWriter() { roach.init(16); wall.init(false); logical.init(true); untyped.init(); }
  int ncols() const override { return 4; }
  uint8_t col_type(int c) const override {
    return c == 0 ? kTypePrefixBytes : c == 3 ? kTypeBytes : kTypeUint;
  }
  int header_size() const override { return 1; }
  static int split(const uint8_t* k, int kl) { return kl == 0 ? 0 : kl - int(k[kl - 1]); }  // cockroachkvs.go:298-310
  KCmp compare_prev(const uint8_t* k, int kl, int prefix_len) const override {
    int pl = prefix_len >= 0 ? prefix_len : split(k, kl);
    KCmp c{pl, 0};
    if (roach.n_keys == 0) return c;
    const std::string& lr = roach.last_key;
    int cp = int(common_prefix(reinterpret_cast<const uint8_t*>(lr.data()), lr.size(), k, size_t(pl - 1)));
    if (int(lr.size()) == cp && k[cp] == 0x00) cp++;
    c.common_prefix_len = cp;
    return c;
  }
  void write_key(int row, const uint8_t* k, int kl, int pl, int shared) override {
    int vlen = k[kl - 1];
    prev_suffix.assign(k + pl, k + kl);
    roach.put(k, pl - 1, std::min(shared, prev_roach_len));
    prev_roach_len = pl - 1;
    uint64_t wt = 0;
    const uint8_t* uv = nullptr;
    size_t uvl = 0;
    auto be64 = [](const uint8_t* p) { uint64_t v = 0; for (int i = 0; i < 8; i++) v = v << 8 | p[i]; return v; };
    switch (vlen) {
      case 0: suffix_types |= 2; break;  // hasEmptySuffixes
      case 9: suffix_types |= 1; wt = be64(k + pl); break;
      case 13:
      case 14: {
        suffix_types |= 1;
        wt = be64(k + pl);
        uint32_t lg = uint32_t(k[pl + 8]) << 24 | uint32_t(k[pl + 9]) << 16 | uint32_t(k[pl + 10]) << 8 | k[pl + 11];
        logical.set(row, lg);
        break;
      }
      default: suffix_types |= 4; uv = k + pl; uvl = size_t(kl - 1 - pl); break;
    }
    wall.set(row, wt);
    untyped.put(uv, uvl);
  }
  uint32_t size(int rows, uint32_t off) const override {
    off = roach.size(rows, off);
    off = wall.size(rows, off);
    off = logical.size(rows, off);
    return untyped.size(rows, off);
  }
  uint32_t finish(int col, int rows, uint32_t off, uint8_t* buf) override {
    switch (col) {
      case 0: return roach.finish(rows, off, buf);
      case 1: return wall.finish(rows, off, buf);
      case 2: return logical.finish(rows, off, buf);
      default: return untyped.finish(rows, off, buf);
    }
  }
  void finish_header(uint8_t* buf) const override { buf[0] = suffix_types; }
  void reset() override {
    roach.reset(); wall.reset(); logical.reset(); untyped.reset();
    suffix_types = 0;
    prev_roach_len = 0;
  }
};

constexpr uint32_t kDataBlockCustomHeaderSize = 4;  // data_block.go:607
constexpr int kFormatCols = 5;     // trailer, prefixChanged, values, isValueExternal, isObsolete (dataBlockColumnMaxV1)
constexpr int kFormatColsV2 = 8;   // + tieringSpanID, tieringAttribute, secondaryBlobHandle (dataBlockColumnMaxV2)

}  // namespace

struct pbl_colblk_writer {
  KeyWriter* kw = nullptr;
  UintB trailers;
  BitmapB prefix_same, is_value_external, is_obsolete;
  RawBytesB values;
  // Pebblev8 tiering columns (OptionalColumnConfig.SupportsTiering)
  bool tiering = false;
  UintB tiering_span, tiering_attr;
  RawBytesB secondary_handles;
  int rows = 0;
  uint32_t max_key_len = 0;
  uint32_t schema = 0;

  pbl_colblk_writer(uint32_t sch, int bundle) : schema(sch) {
    if (sch == PBL_FMT_COL_CRDB1) kw = new CrdbKeyWriter();
    else kw = new DefaultKeyWriter(bundle);
    trailers.init(false);
    values.init();
    tiering_span.init(true);
    tiering_attr.init(true);
    secondary_handles.init();
  }
  ~pbl_colblk_writer() { delete kw; }
  void reset() {
    kw->reset();
    trailers.reset();
    prefix_same.reset();
    values.reset();
    is_value_external.reset();
    is_obsolete.reset();
    tiering_span.reset();
    tiering_attr.reset();
    secondary_handles.reset();
    rows = 0;
    max_key_len = 0;
  }
  int format_cols() const { return tiering ? kFormatColsV2 : kFormatCols; }  // numFormatColumns
  uint32_t header_size() const {
    return uint32_t(7 + 5 * (kw->ncols() + format_cols())) + kDataBlockCustomHeaderSize + uint32_t(kw->header_size());
  }
  uint32_t size_for(int r) const {  // DataBlockEncoder.Size at `r` rows
    uint32_t off = header_size();
    off = kw->size(r, off);
    off = trailers.size(r, off);
    off = prefix_same.inverted_size(r, off);
    off = values.size(r, off);
    off = is_value_external.size(r, off);
    off = is_obsolete.size(r, off);
    if (tiering) {
      off = tiering_span.size(r, off);
      off = tiering_attr.size(r, off);
      off = secondary_handles.size(r, off);
    }
    return off + 1;
  }
};

extern "C" {

pbl_colblk_writer* pbl_colblk_writer_new(uint32_t schema, int bundle_size) {
  if (schema != PBL_FMT_COL_DEFAULT && schema != PBL_FMT_COL_CRDB1) return nullptr;
  if (bundle_size <= 0 || (bundle_size & (bundle_size - 1))) return nullptr;
  return new pbl_colblk_writer(schema, bundle_size);
}
void pbl_colblk_writer_free(pbl_colblk_writer* w) { delete w; }
void pbl_colblk_writer_reset(pbl_colblk_writer* w) { w->reset(); }

void pbl_colblk_writer_set_tiering(pbl_colblk_writer* w, int tiering) { w->tiering = tiering != 0; }

}  // extern "C"

namespace {
// DataBlockEncoder.internalAdd (data_block.go:730-765)
int add_row(pbl_colblk_writer* w, const uint8_t* key, size_t key_len, int64_t prefix_len, uint64_t trailer,
            const uint8_t* value, size_t value_len, int value_kind, int is_obsolete, uint64_t span, uint64_t attr,
            const uint8_t* handle, size_t handle_len) {
  if (key_len == 0) return PBL_INVALID_ARG;
  int kl = int(key_len);
  KCmp c = w->kw->compare_prev(key, kl, int(prefix_len));
  if (c.prefix_len < 1 || c.prefix_len > kl) return PBL_INVALID_ARG;
  if (w->schema == PBL_FMT_COL_CRDB1 && key[c.prefix_len - 1] != 0) return PBL_INVALID_ARG;
  w->kw->write_key(w->rows, key, kl, c.prefix_len, c.common_prefix_len);
  if (c.prefix_equal()) w->prefix_same.set(w->rows);
  if (is_obsolete) w->is_obsolete.set(w->rows);
  w->trailers.set(w->rows, trailer);
  if (value_kind != 0) {  // block.ValueBlockHandlePrefix / BlobValueHandlePrefix (sstable/block/kv.go:65-90)
    uint8_t vp = uint8_t(value_kind == 1 ? 0x80 : 0x40) | uint8_t(c.prefix_equal() ? 0x20 : 0);
    w->is_value_external.set(w->rows);
    w->values.put_concat(&vp, 1, value, value_len);
  } else {
    w->values.put(value, value_len);
  }
  if (w->tiering) {
    if (attr != 0) {  // meta.IsSet() (internal/base/internal.go:700-702)
      w->tiering_span.set(w->rows, span);
      w->tiering_attr.set(w->rows, attr);
    }
    w->secondary_handles.put(handle, handle ? handle_len : 0);
  }
  if (key_len > w->max_key_len) w->max_key_len = uint32_t(key_len);
  w->rows++;
  return c.prefix_equal() ? 1 : 0;
}
}  // namespace

extern "C" {

int pbl_colblk_writer_add(pbl_colblk_writer* w, const uint8_t* key, size_t key_len, int64_t prefix_len,
                          uint64_t trailer, const uint8_t* value, size_t value_len, int value_kind,
                          int is_obsolete) {
  return add_row(w, key, key_len, prefix_len, trailer, value, value_len, value_kind, is_obsolete, 0, 0, nullptr, 0);
}

int pbl_colblk_writer_add_meta(pbl_colblk_writer* w, const uint8_t* key, size_t key_len, int64_t prefix_len,
                               uint64_t trailer, const uint8_t* value, size_t value_len, int value_kind,
                               int is_obsolete, uint64_t tiering_span_id, uint64_t tiering_attr,
                               const uint8_t* secondary_handle, size_t secondary_handle_len) {
  return add_row(w, key, key_len, prefix_len, trailer, value, value_len, value_kind, is_obsolete, tiering_span_id,
                 tiering_attr, secondary_handle, secondary_handle_len);
}

uint32_t pbl_colblk_writer_rows(const pbl_colblk_writer* w) { return uint32_t(w->rows); }
size_t pbl_colblk_writer_size(const pbl_colblk_writer* w, uint32_t rows) { return w->size_for(int(rows)); }

/* Finish `rows` (== rows() or rows()-1) rows; returns the block size, writing
 * it to dst when dst_cap suffices.  The writer must be reset before reuse. */
size_t pbl_colblk_writer_finish(pbl_colblk_writer* w, uint32_t rows, uint8_t* dst, size_t dst_cap) {
  int r = int(rows);
  if (r != w->rows && r != w->rows - 1) return 0;
  size_t size = w->size_for(r);
  if (!dst || dst_cap < size) return size;
  std::vector<uint8_t> buf(size, 0);
  uint8_t* b = buf.data();
  int cols = w->kw->ncols() + w->format_cols();
  w->prefix_same.invert(r);
  uint32_t custom = kDataBlockCustomHeaderSize + uint32_t(w->kw->header_size());
  b[custom] = 1;  // Version1
  put_le(b + custom + 1, uint64_t(cols), 2);
  put_le(b + custom + 3, uint64_t(r), 4);
  w->kw->finish_header(b);
  put_le(b + w->kw->header_size(), w->max_key_len, 4);
  uint32_t hoff = custom + 7, poff = w->header_size();
  auto col = [&](uint8_t type) {
    b[hoff] = type;
    put_le(b + hoff + 1, poff, 4);
    hoff += 5;
  };
  for (int c = 0; c < w->kw->ncols(); c++) {
    col(w->kw->col_type(c));
    poff = w->kw->finish(c, r, poff, b);
  }
  col(kTypeUint);  poff = w->trailers.finish(r, poff, b);
  col(kTypeBool);  poff = w->prefix_same.finish(r, poff, b);
  col(kTypeBytes); poff = w->values.finish(r, poff, b);
  col(kTypeBool);  poff = w->is_value_external.finish(r, poff, b);
  col(kTypeBool);  poff = w->is_obsolete.finish(r, poff, b);
  if (w->tiering) {
    col(kTypeUint);  poff = w->tiering_span.finish(r, poff, b);
    col(kTypeUint);  poff = w->tiering_attr.finish(r, poff, b);
    col(kTypeBytes); poff = w->secondary_handles.finish(r, poff, b);
  }
  b[poff++] = 0;  // block padding byte
  if (poff != size) return 0;
  std::memcpy(dst, b, size);
  return size;
}

}  // extern "C"

// ---- synthetic config-3 generator --------------------------------------------
namespace {

inline uint64_t sm64(uint64_t& s) {
  uint64_t x = (s += 0x9E3779B97F4A7C15ull);
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}
inline uint64_t rnd_n(uint64_t& s, uint64_t n) { return sm64(s) % n; }

// One block's KVs per cockroachkvs.RandomKVs (test_utils.go): roach keys share
// `shared` letters, the rest random from the alphabet; ~Exp(avg) versions per
// roach key; wall = base + U[0, 1h); logical nonzero with pct_logical%.
void gen_block_keys(uint64_t seed, uint32_t count, const pbl_colgen_config& cfg, uint32_t schema,
                    std::vector<std::string>& keys) {
  uint64_t s = seed;
  std::string shared(cfg.prefix_len_shared, 'a');
  uint64_t s0 = cfg.seed;  // batch-wide shared prefix
  for (auto& c : shared) c = char('a' + rnd_n(s0, cfg.alphabet_len));
  keys.clear();
  while (keys.size() < count) {
    std::string roach = shared;
    while (roach.size() < cfg.roach_key_len) roach.push_back(char('a' + rnd_n(s, cfg.alphabet_len)));
    double u = (double(sm64(s) >> 11) + 0.5) * (1.0 / 9007199254740992.0);
    int n = std::max(1, int(-std::log(u) * double(cfg.avg_keys_per_prefix)));
    for (int i = 0; i < n && keys.size() < count; i++) {
      uint64_t wall = cfg.base_wall_time + rnd_n(s, 3600ull * 1000000000ull);
      uint32_t logical = 0;
      if (cfg.pct_logical > 0 && rnd_n(s, 100) < cfg.pct_logical) logical = uint32_t(sm64(s));
      std::string k = roach;
      if (schema == PBL_FMT_COL_CRDB1) {  // EncodeTimestamp (cockroachkvs.go:175-197)
        k.push_back(0);
        for (int b = 7; b >= 0; b--) k.push_back(char(wall >> (8 * b)));
        if (logical) {
          for (int b = 3; b >= 0; b--) k.push_back(char(logical >> (8 * b)));
          k.push_back(13);
        } else {
          k.push_back(9);
        }
      } else {  // default schema: prefix '@' decimal wall time (testkeys-style suffix)
        k += "@" + std::to_string(wall % 1000000007ull);
      }
      keys.push_back(std::move(k));
    }
  }
  std::sort(keys.begin(), keys.end());
}

}  // namespace

extern "C" uint64_t pbl_gen_col_blocks(const pbl_colgen_config* cfgp, uint32_t schema, uint32_t n_blocks,
                                       uint32_t block_size, uint8_t* dst, uint64_t* block_off,
                                       uint32_t* block_len, int n_threads) {
  const pbl_colgen_config cfg = *cfgp;
  if (n_threads < 1) n_threads = 1;
  std::vector<uint64_t> counts(n_threads, 0);
  auto work = [&](int t) {
    pbl_colblk_writer w(schema, 16);
    w.tiering = cfg.tiering != 0;
    std::vector<std::string> keys;
    std::vector<uint8_t> val(cfg.value_len);
    for (uint32_t bl = t; bl < n_blocks; bl += n_threads) {
      const uint32_t b = cfg.first_block + bl;  // the block's global index: its content
      uint64_t s = cfg.seed ^ (0xC01B10C5ull * (b + 1));
      // Per-row estimate sizes the candidate set; refill if it runs out.
      uint32_t est = block_size / std::max<uint32_t>(1, cfg.value_len + cfg.roach_key_len / 2 + 12) + 64;
      gen_block_keys(s, est * 2, cfg, schema, keys);
      w.reset();
      uint32_t rows = 0;
      size_t k = 0;
      const std::string* prev = nullptr;
      for (; k < keys.size(); k++) {
        for (auto& x : val) x = uint8_t(sm64(s));
        uint64_t seq = (uint64_t(b) << 20) + k;
        bool obs = (prev && *prev == keys[k]) || (cfg.obsolete_every && k % cfg.obsolete_every == cfg.obsolete_every - 1);
        uint64_t span = 0, attr = 0;
        if (cfg.tiering) {
          const uint64_t r = sm64(s);
          span = 1 + r % cfg.tiering;
          attr = (r >> 32) % 10 == 0 ? 0 : cfg.base_wall_time / 1000000000ull + (r >> 8) % 3600;
        }
        add_row(&w, reinterpret_cast<const uint8_t*>(keys[k].data()), keys[k].size(), -1, (seq << 8) | 1, val.data(),
                val.size(), 0, obs, span, attr, nullptr, 0);
        prev = &keys[k];
        if (w.size_for(w.rows) > block_size) break;
      }
      rows = uint32_t(w.rows);
      if (w.size_for(w.rows) > block_size) rows--;
      size_t n = pbl_colblk_writer_finish(&w, rows, dst + uint64_t(bl) * block_size, block_size);
      block_off[bl] = uint64_t(bl) * block_size;
      block_len[bl] = uint32_t(n);
      counts[t] += rows;
    }
  };
  std::vector<std::thread> th;
  for (int t = 0; t < n_threads; t++) th.emplace_back(work, t);
  for (auto& x : th) x.join();
  uint64_t tot = 0;
  for (auto c : counts) tot += c;
  return tot;
}
