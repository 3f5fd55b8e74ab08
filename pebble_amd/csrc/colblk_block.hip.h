// colblk_block.hip.h — gfx950 decode of ONE columnar (colblk) data block per
// 256-thread workgroup, for colblk.DefaultKeySchema and cockroachkvs.KeySchema
// ("crdb1").  Shared by the pure-colblk kernel (colblk_decode.hip) and the
// mixed row+colblk kernel (rowblk_decode.hip).
//
// Restates (cockroachdb/pebble, paths relative to the repo root):
//   header / directory / DecodeColumn   sstable/colblk/block.go:179-201, 287-301, 320-387
//   Uint / offsets                      sstable/colblk/unsafe_uints.go:32-96, endian_little.go:21-43
//   RawBytes                            sstable/colblk/raw_bytes.go:63-81
//   PrefixBytes                         sstable/colblk/prefix_bytes.go:206-231, 286-386, 1135-1170
//   Bitmap                              sstable/colblk/bitmap.go:43-77
//   DataBlockDecoder.Init / Iter.Next   sstable/colblk/data_block.go:1096-1109, 1662-1708
//   default / crdb1 MaterializeUserKey  data_block.go:428-442, cockroachkvs/cockroachkvs.go:1009-1071
// Status semantics match oracle/colblk_oracle.c.
//
// HBM layout / data flow per block:
//   * the head of the block (header, key columns, trailers, prefixChanged: the
//     bytes before the values column, <= kStage) and its last kTail bytes
//     (isValueExternal / isObsolete bitmaps) are staged in LDS with 16-B loads;
//   * one thread per row computes the key's parts and length from LDS; a block
//     scan places keys; keys are built in an LDS buffer while wave 0 resolves the
//     cross-block look-back, then leave as aligned 16-B stores;
//   * the values column's data is ONE contiguous byte range: it is copied
//     global -> global with aligned 16-B loads and a funnel shift, never staged.
#pragma once

namespace pbl {
namespace col {

constexpr uint32_t kStage = 12288;  // head bytes staged in LDS
constexpr uint32_t kTail = 512;     // tail bytes staged in LDS
constexpr uint32_t kKeyBuf = 8192;  // key build buffer (one chunk of rows)
constexpr uint32_t kKeyPad = 16;
constexpr uint32_t kChunk = kTPB;   // rows per chunk (one per thread)

enum { kDtBool = 1, kDtUint = 2, kDtBytes = 3, kDtPrefix = 4 };

// Address-space-typed pointers: LDS and global reads must never merge into one
// flat access (the head/tail/global reader selects between them per byte).
using lds_cu8 = __attribute__((address_space(3))) const uint8_t*;
using lds_u8 = __attribute__((address_space(3))) uint8_t*;
using lds_cu32 = __attribute__((address_space(3))) const uint32_t*;
using lds_u4 = __attribute__((address_space(3))) u32x4*;
using glb_cu8 = __attribute__((address_space(1))) const uint8_t*;
template <class T>
__device__ __forceinline__ __attribute__((address_space(3))) T* to_lds(T* p) {
  return (__attribute__((address_space(3))) T*)p;
}

struct UCol {
  uint64_t base;
  uint32_t at, w;
};

struct Desc {
  uint32_t status, rows;
  uint32_t pb_shift, pb_data, shared_len, data_len;
  UCol pb_off;
  UCol rb_off;  // default: suffixes / crdb1: untyped versions
  uint32_t rb_data;
  UCol wall, logical, trailers;
  uint32_t pc_at, ext_at, obs_at;  // bitmap word arrays (0 = zero encoding)
  UCol v_off;
  uint32_t v_data, v_lo, v_hi;    // values data start and [off[0], off[rows])
  uint32_t key_end;               // page start of the values column
  UCol span, attr;                // Pebblev8 tiering columns (PBL_COL_TIERING; else width 0, base 0)
};

struct Lds {
  uint4 head4[kStage / 16];
  uint4 tail4[kTail / 16 + 1];
  uint4 key4[(kKeyBuf + 2 * kKeyPad) / 16];
  Desc d;
  uint64_t red[4];
  uint64_t bases[kNumComp];
  uint32_t scratch[16];
  uint32_t status, bad, nhead, tail_lo;
};

// ---- byte sources ------------------------------------------------------------
__device__ __forceinline__ uint64_t lds_le(lds_cu8 p, uint32_t w) {  // p aligned to w
  switch (w) {
    case 1: return *p;
    case 2: return *(__attribute__((address_space(3))) const uint16_t*)p;
    case 4: return *(__attribute__((address_space(3))) const uint32_t*)p;
    default: return *(__attribute__((address_space(3))) const uint64_t*)p;
  }
}
__device__ __forceinline__ uint64_t g_le(glb_cu8 p, uint32_t w) {
  if ((reinterpret_cast<uintptr_t>(p) & (w - 1)) == 0) {
    switch (w) {
      case 1: return *p;
      case 2: return *(__attribute__((address_space(1))) const uint16_t*)p;
      case 4: return *(__attribute__((address_space(1))) const uint32_t*)p;
      default: return *(__attribute__((address_space(1))) const uint64_t*)p;
    }
  }
  uint64_t v = 0;
  for (int i = int(w) - 1; i >= 0; i--) v = v << 8 | p[i];
  return v;
}

// Head (LDS) / tail (LDS) / rest (global) reader, block-relative offsets.
struct Src {
  lds_cu8 head;
  lds_cu8 tail;
  glb_cu8 g;
  uint32_t nhead, tail_lo, len;
  __device__ __forceinline__ uint32_t byte(uint32_t o) const {
    if (o < nhead) return head[o];
    if (o >= tail_lo) return tail[o - tail_lo];
    return g[o];
  }
  // LE value of width w at block offset o (o aligned to w within the block)
  __device__ __forceinline__ uint64_t le(uint32_t o, uint32_t w) const {
    if (o + w <= nhead) return lds_le(head + o, w);
    if (o >= tail_lo) return lds_le(tail + (o - tail_lo), w);
    return g_le(g + o, w);
  }
  __device__ __forceinline__ uint64_t le_u(uint32_t o, uint32_t w) const {  // unaligned, header fields
    if (o + 8 <= nhead) {
      // one round trip: three aligned LDS dwords around [o, o+8) and a funnel
      // shift (the staged head has 8 readable bytes past nhead)
      const uint32_t a = uint32_t(reinterpret_cast<uintptr_t>(head)) + o;
      lds_cu32 W = (lds_cu32)(uintptr_t)(a & ~3u);
      const uint32_t r = a & 3;
      const uint32_t x0 = W[0], x1 = W[1], x2 = W[2];
      const uint64_t v = uint64_t(__builtin_amdgcn_alignbyte(x2, x1, r)) << 32 | __builtin_amdgcn_alignbyte(x1, x0, r);
      return w >= 8 ? v : (v & ((1ull << (8 * w)) - 1));
    }
    uint64_t v = 0;
    for (int i = int(w) - 1; i >= 0; i--) v = v << 8 | byte(o + i);
    return v;
  }
};

// Column reads: F = the key region is staged (read LDS directly).
template <bool F>
__device__ __forceinline__ uint64_t u_at(const Src& S, const UCol& u, uint32_t i) {
  if (u.w == 0) return u.base;
  const uint32_t o = u.at + i * u.w;
  return u.base + (F ? lds_le(S.head + o, u.w) : S.le(o, u.w));
}
// A Uint column past the staged head (the tiering columns follow the values):
// through the head / tail / global reader.
__device__ __forceinline__ uint64_t u_at_any(const Src& S, const UCol& u, uint32_t i) {
  return u.w == 0 ? u.base : u.base + S.le(u.at + i * u.w, u.w);
}
template <bool F>
__device__ __forceinline__ uint32_t key_byte(const Src& S, uint32_t o) {
  return F ? S.head[o] : S.byte(o);
}

// ---- metadata init (lane 0): DataBlockDecoder.Init + KeySeeker init ----------
__device__ __forceinline__ bool dec_uints(const Src& S, uint64_t off, uint32_t rows, UCol* u, uint64_t* end) {
  u->base = 0; u->w = 0; u->at = uint32_t(off);
  if (rows == 0) { *end = off; return true; }
  if (off >= S.len) return false;
  const uint32_t e = S.byte(uint32_t(off++));
  const uint32_t w = e & 0x7f;
  const bool delta = (e & 0x80) != 0;
  if (!(w == 0 || w == 1 || w == 2 || w == 4 || (w == 8 && !delta))) return false;  // IsValid
  if (delta) {
    if (off + 8 > S.len) return false;
    u->base = S.le_u(uint32_t(off), 8);
    off += 8;
  }
  if (w) off = (off + w - 1) & ~uint64_t(w - 1);
  u->w = w;
  u->at = uint32_t(off);
  *end = off + uint64_t(rows) * w;
  return true;
}
__device__ __forceinline__ bool dec_rawbytes(const Src& S, uint64_t off, uint32_t count, UCol* o, uint32_t* data,
                                    uint64_t* end) {
  *data = 0;
  if (count == 0) { o->base = 0; o->w = 0; o->at = uint32_t(off); *end = off; return true; }
  uint64_t dend;
  if (!dec_uints(S, off, count + 1, o, &dend)) return false;
  if (o->base != 0 || o->w == 8 || dend > S.len) return false;  // DecodeUnsafeOffsets
  *data = uint32_t(dend);
  const uint64_t last = o->w ? S.le_u(o->at + count * o->w, o->w) : 0;
  *end = dend + last;
  return *end <= S.len;
}
__device__ __forceinline__ bool dec_bitmap(const Src& S, uint64_t off, uint32_t n, uint32_t* at, uint64_t* end) {
  if (off >= S.len) return false;
  const uint32_t e = S.byte(uint32_t(off++));
  if (e == 1) { *at = 0; *end = off; return true; }
  off = (off + 7) & ~uint64_t(7);
  const uint64_t nw = (uint64_t(n) + 63) >> 6, ns = (nw + 63) >> 6;
  *at = uint32_t(off);
  *end = off + 8 * (nw + ns);
  return *end <= S.len;
}

struct Dir {
  uint32_t custom, ncols;
  __device__ __forceinline__ bool column(const Src& S, uint32_t col, uint32_t type, uint64_t* start, uint64_t* next) const {
    if (col >= ncols) return false;
    const uint64_t h = uint64_t(custom) + 7 + 5ull * col;
    if (h + 5 > S.len || S.byte(uint32_t(h)) != type) return false;
    *start = S.le_u(uint32_t(h + 1), 4);
    if (col + 1 >= ncols) *next = S.len - 1;
    else {
      const uint64_t h2 = h + 5;
      if (h2 + 5 > S.len) return false;
      *next = S.le_u(uint32_t(h2 + 1), 4);
    }
    return *next <= S.len && *start <= *next;
  }
};

// DataBlockDecoder.Init + the KeySeeker init (data_block.go:1096-1109;
// block.go:287-301 DecodeColumn), one lane per column (wave 0, all 64 lanes call it), in uniform
// stages so that every lane issues the same reads: (1) its directory entry
// (Dir::column), (2) the encoding bytes at its column's start, (3) per-kind
// arithmetic restating dec_uints / dec_bitmap / dec_rawbytes, (4) the first and
// last offsets of offset-bearing columns.  Every read is bounds-guarded; the
// statuses combine by ballot exactly as the serial order would (every header
// failure is PBL_CORRUPT_COLBLK_HEADER; the final bounds check is
// PBL_CORRUPT_BOUNDS).  Lane 0 writes the shared fields; each column lane its own.
// `tiering` (PBL_COL_TIERING): the Pebblev8 tieringSpanID / tieringAttribute
// Uint columns (data_block.go:514-525) are decoded as initTieringMetadata does
// (:1605-1631) by two more lanes; otherwise their descriptors are zero columns.
__device__ __forceinline__ uint32_t sbyte(const Src& S, uint64_t o) { return o < S.len ? S.byte(uint32_t(o)) : 0u; }
__device__ __forceinline__ uint64_t sle(const Src& S, uint64_t o, uint32_t w) {
  return (w && o + w <= S.len) ? S.le_u(uint32_t(o), w) : 0ull;
}
__device__ __forceinline__ bool uint_width_ok(uint32_t w, bool delta) {
  return w == 0 || w == 1 || w == 2 || w == 4 || (w == 8 && !delta);
}

__device__ __forceinline__ uint32_t parse_block_wave(const Src& S, uint32_t schema, bool tiering, Desc* D) {
  const int l = lane_id();
  if (schema != PBL_FMT_COL_DEFAULT && schema != PBL_FMT_COL_CRDB1) return PBL_UNSUPPORTED;
  const uint32_t nsc = schema == PBL_FMT_COL_CRDB1 ? 4 : 2;
  const uint32_t custom = 4 + (schema == PBL_FMT_COL_CRDB1 ? 1 : 0);
  if (S.len < custom + 7) return PBL_CORRUPT_COLBLK_HEADER;
  const uint32_t ncols = uint32_t(S.le_u(custom + 1, 2));
  const uint32_t rows = uint32_t(S.le_u(custom + 3, 4));
  if (l == 0) D->rows = rows;
  const uint32_t c = uint32_t(l);
  const bool active = c < nsc + (tiering ? 7u : 5u);
  // column kinds: 0 Uint, 1 Bool, 2 Bytes, 3 PrefixBytes
  const bool crdb = schema == PBL_FMT_COL_CRDB1;
  const bool tier_col = c == nsc + 5 || c == nsc + 6;
  if (tier_col && !tiering) {  // KVMeta{}: zero columns
    UCol z;
    z.base = 0;
    z.w = 0;
    z.at = 0;
    if (c == nsc + 5) D->span = z;
    else D->attr = z;
  }
  const uint32_t kind = c == 0 ? 3u
                        : (c == nsc || tier_col || (crdb && (c == 1 || c == 2))) ? 0u
                        : (c == nsc + 1 || c == nsc + 3 || c == nsc + 4) ? 1u
                        : 2u;
  const uint32_t want = kind == 0 ? uint32_t(kDtUint) : kind == 1 ? uint32_t(kDtBool)
                        : kind == 2 ? uint32_t(kDtBytes) : uint32_t(kDtPrefix);
  // (1) directory entry: Dir::column
  const uint64_t h = uint64_t(custom) + 7 + 5ull * c;
  const uint32_t typ = sbyte(S, h);
  const uint64_t start = sle(S, h + 1, 4);
  const uint64_t nxt_raw = sle(S, h + 6, 4);
  const bool last_col = c + 1 >= ncols;
  const uint64_t nx = last_col ? uint64_t(S.len) - 1 : nxt_raw;
  bool ok = c < ncols && h + 5 <= S.len && typ == want && (last_col || h + 10 <= S.len) && nx <= S.len &&
            start <= nx;
  // (2) encoding bytes at the column start (PrefixBytes: its shift byte, then
  // the offsets' Uint encoding one byte later)
  const uint64_t u0 = kind == 3 ? start + 1 : start;   // Uint encoding byte of this column
  const uint32_t b_shift = sbyte(S, start);
  const uint32_t enc = sbyte(S, u0);
  const uint64_t base8 = sle(S, u0 + 1, 8);
  // (3) per kind
  uint32_t cnt = rows;  // value count (Uint) / slice count (Bytes, Prefix)
  uint32_t shift = 0, nbund = 0;
  if (kind == 3) {
    ok = ok && rows != 0 && start < S.len;
    shift = b_shift;
    ok = ok && shift <= 16;
    nbund = ok ? 1 + ((rows - 1) >> shift) : 0;
    cnt = rows + nbund;
  }
  uint64_t at = 0, end = 0, base = 0;
  uint32_t w = 0;
  if (kind == 1) {  // dec_bitmap
    ok = ok && start < S.len;
    if (enc == 1) {
      at = 0;
      end = start + 1;
    } else {
      const uint64_t off = (start + 1 + 7) & ~uint64_t(7);
      const uint64_t nw = (uint64_t(rows) + 63) >> 6, ns = (nw + 63) >> 6;
      at = off;
      end = off + 8 * (nw + ns);
      ok = ok && end <= S.len;
    }
  } else {  // dec_uints over cnt (+1 for offset columns) values at u0
    const uint32_t nvals = kind == 0 ? cnt : cnt + 1;
    if (nvals == 0) {
      at = u0;
      end = u0;
    } else {
      ok = ok && u0 < S.len;
      w = enc & 0x7f;
      const bool delta = (enc & 0x80) != 0;
      ok = ok && uint_width_ok(w, delta);
      uint64_t off = u0 + 1;
      if (delta) {
        ok = ok && off + 8 <= S.len;
        base = base8;
        off += 8;
      }
      if (w) off = (off + w - 1) & ~uint64_t(w - 1);
      at = off;
      end = off + uint64_t(nvals) * w;
      if (kind != 0) ok = ok && base == 0 && w != 8 && end <= S.len;  // DecodeUnsafeOffsets
    }
  }
  // (4) first and last offsets of offset-bearing columns
  const uint64_t first = (kind >= 2 && w) ? sle(S, at, w) : 0;
  const uint64_t lastv = (kind >= 2 && w) ? sle(S, at + uint64_t(cnt) * w, w) : 0;
  uint64_t data = 0;
  if (kind >= 2) {
    data = end;            // RawBytes data start
    end = end + lastv;     // RawBytes end
    ok = ok && end <= S.len;
  }
  ok = ok && end == nx;
  if (active && ok) {
    UCol u;
    u.base = base;
    u.w = w;
    u.at = uint32_t(at);
    if (kind == 3) {
      D->pb_shift = shift;
      D->pb_off = u;
      D->pb_data = uint32_t(data);
      D->shared_len = uint32_t(first);
      D->data_len = uint32_t(lastv);
    } else if (kind == 0) {
      if (c == nsc) D->trailers = u;
      else if (c == nsc + 5) D->span = u;
      else if (c == nsc + 6) D->attr = u;
      else if (c == 1) D->wall = u;
      else D->logical = u;
    } else if (kind == 1) {
      const uint32_t a32 = uint32_t(at);
      if (c == nsc + 1) D->pc_at = a32;
      else if (c == nsc + 3) D->ext_at = a32;
      else D->obs_at = a32;
    } else if (c == nsc + 2) {
      D->v_off = u;
      D->v_data = uint32_t(data);
      D->key_end = uint32_t(start);
      D->v_lo = uint32_t(first);
      D->v_hi = uint32_t(lastv);
    } else {
      D->rb_off = u;
      D->rb_data = uint32_t(data);
    }
  }
  if (__ballot(active && !ok)) return PBL_CORRUPT_COLBLK_HEADER;
  wave_sync();
  if (D->shared_len > D->data_len || D->v_lo > D->v_hi) return PBL_CORRUPT_BOUNDS;
  return PBL_OK;
}

// ---- per row ------------------------------------------------------------------
struct RowParts {
  uint32_t bl, bh, sl, sh, ul, uh;  // block offsets of bundle prefix / suffix / untyped-or-suffix bytes
  uint64_t wall;
  uint32_t logical, klen;
  bool ok;
};

template <bool F>
__device__ __forceinline__ RowParts row_parts(const Src& S, const Desc& d, uint32_t schema, uint32_t r) {
  RowParts p;
  p.ok = true;
  const uint32_t s = d.pb_shift, mask = ~((1u << s) - 1);
  const uint32_t bi = (r >> s) + (r & mask);  // bundleOffsetIndexForRow
  uint32_t si = 1 + (r >> s) + r;             // rowSuffixIndex
  const uint32_t n = d.data_len;
  const uint32_t a = uint32_t(u_at<F>(S, d.pb_off, bi)), b = uint32_t(u_at<F>(S, d.pb_off, bi + 1));
  uint32_t lo = uint32_t(u_at<F>(S, d.pb_off, si)), hi = uint32_t(u_at<F>(S, d.pb_off, si + 1));
  p.ok = a <= b && b <= n && lo <= hi && hi <= n;
  while (p.ok && lo == hi && si > bi + 1) {  // rowSuffixOffsets: duplicate of the previous key
    si--;
    hi = lo;
    lo = uint32_t(u_at<F>(S, d.pb_off, si));
    p.ok = lo <= hi;
  }
  p.bl = d.pb_data + a;
  p.bh = d.pb_data + b;
  p.sl = d.pb_data + lo;
  p.sh = d.pb_data + hi;
  uint32_t klen = d.shared_len + (b - a) + (hi - lo);
  p.wall = 0;
  p.logical = 0;
  bool need_rb = true;
  if (schema == PBL_FMT_COL_CRDB1) {
    p.wall = u_at<F>(S, d.wall, r);
    p.logical = uint32_t(u_at<F>(S, d.logical, r));
    need_rb = p.wall == 0 && p.logical == 0;
    if (!need_rb) klen += p.logical ? 14 : 10;
  }
  p.ul = p.uh = 0;
  if (need_rb) {
    const uint32_t rn = uint32_t(u_at<F>(S, d.rb_off, d.rows));
    const uint32_t x = uint32_t(u_at<F>(S, d.rb_off, r)), y = uint32_t(u_at<F>(S, d.rb_off, r + 1));
    p.ok = p.ok && x <= y && y <= rn;
    p.ul = d.rb_data + x;
    p.uh = d.rb_data + y;
    if (schema == PBL_FMT_COL_CRDB1) klen += 1 + (y > x ? y - x + 1 : 0);
    else klen += y - x;
  }
  p.klen = klen;
  return p;
}

// value slice check (values offsets are read through the general source)
__device__ __forceinline__ bool value_ok(const Src& S, const Desc& d, uint32_t r) {
  const UCol& v = d.v_off;
  if (v.w == 0) return true;
  const uint32_t lo = uint32_t(S.le(v.at + r * v.w, v.w)), hi = uint32_t(S.le(v.at + (r + 1) * v.w, v.w));
  return lo <= hi && hi <= d.v_hi;
}

// n LDS bytes src[0, n) to kb[dst, dst + n): 16 bytes per unaligned
// ds_read_b128 / ds_write_b128 (gfx950 runs in unaligned mode), the tail by
// the fewest narrower writes, nothing written past dst + n (the next key is
// another lane's); reads may run up to 15 bytes past the source, inside the
// workgroup's LDS.  Returns dst + n.
__device__ __forceinline__ uint32_t lds_copy(lds_u8 kb, uint32_t dst, lds_cu8 src, uint32_t n) {
  typedef u32x4 u32x4_l __attribute__((aligned(1)));
  typedef uint64_t u64_l __attribute__((aligned(1)));
  typedef uint32_t u32_l __attribute__((aligned(1)));
  typedef uint16_t u16_l __attribute__((aligned(1)));
  uint32_t c = 0;
  for (; c + 16 <= n; c += 16)
    *(__attribute__((address_space(3))) u32x4_l*)(kb + dst + c) =
        *(__attribute__((address_space(3))) const u32x4_l*)(src + c);
  if (c < n) {
    const u32x4 w = *(__attribute__((address_space(3))) const u32x4_l*)(src + c);
    uint64_t lo = uint64_t(w.x) | uint64_t(w.y) << 32;
    const uint64_t hi = uint64_t(w.z) | uint64_t(w.w) << 32;
    const uint32_t r = n - c;
    lds_u8 o = kb + dst + c;
    if (r & 8) { *(__attribute__((address_space(3))) u64_l*)o = lo; lo = hi; o += 8; }
    if (r & 4) { *(__attribute__((address_space(3))) u32_l*)o = uint32_t(lo); lo >>= 32; o += 4; }
    if (r & 2) { *(__attribute__((address_space(3))) u16_l*)o = uint16_t(lo); lo >>= 16; o += 2; }
    if (r & 1) *o = uint8_t(lo);
  }
  return dst + n;
}

#ifndef PBL_COL_KEYCOPY16
#define PBL_COL_KEYCOPY16 1  // staged keys: segment copies 16 B at a time (else byte by byte)
#endif

// MaterializeUserKey of row r into LDS bytes kb[dst ..).
template <bool F>
__device__ __forceinline__ void build_key(const Src& S, const Desc& d, uint32_t schema, const RowParts& p,
                                          lds_u8 kb, uint32_t dst) {
  if (F && PBL_COL_KEYCOPY16) {  // every key byte is in the staged head
    const lds_cu8 H = S.head;
    dst = lds_copy(kb, dst, H + d.pb_data, d.shared_len);
    dst = lds_copy(kb, dst, H + p.bl, p.bh - p.bl);
    dst = lds_copy(kb, dst, H + p.sl, p.sh - p.sl);
    if (schema == PBL_FMT_COL_CRDB1) {
      kb[dst++] = 0;
      if (p.wall == 0 && p.logical == 0) {
        if (p.uh > p.ul) {
          dst = lds_copy(kb, dst, H + p.ul, p.uh - p.ul);
          kb[dst++] = uint8_t(p.uh - p.ul + 1);
        }
      } else {
#pragma unroll
        for (int i = 0; i < 8; i++) kb[dst++] = uint8_t(p.wall >> (56 - 8 * i));
        if (p.logical == 0) {
          kb[dst++] = 9;
        } else {
#pragma unroll
          for (int i = 0; i < 4; i++) kb[dst++] = uint8_t(p.logical >> (24 - 8 * i));
          kb[dst++] = 13;
        }
      }
    } else {
      lds_copy(kb, dst, H + p.ul, p.uh - p.ul);
    }
    return;
  }
  for (uint32_t i = 0; i < d.shared_len; i++) kb[dst++] = uint8_t(key_byte<F>(S, d.pb_data + i));
  for (uint32_t o = p.bl; o < p.bh; o++) kb[dst++] = uint8_t(key_byte<F>(S, o));
  for (uint32_t o = p.sl; o < p.sh; o++) kb[dst++] = uint8_t(key_byte<F>(S, o));
  if (schema == PBL_FMT_COL_CRDB1) {
    kb[dst++] = 0;
    if (p.wall == 0 && p.logical == 0) {
      if (p.uh > p.ul) {
        for (uint32_t o = p.ul; o < p.uh; o++) kb[dst++] = uint8_t(key_byte<F>(S, o));
        kb[dst++] = uint8_t(p.uh - p.ul + 1);
      }
    } else {
#pragma unroll
      for (int i = 0; i < 8; i++) kb[dst++] = uint8_t(p.wall >> (56 - 8 * i));
      if (p.logical == 0) {
        kb[dst++] = 9;
      } else {
#pragma unroll
        for (int i = 0; i < 4; i++) kb[dst++] = uint8_t(p.logical >> (24 - 8 * i));
        kb[dst++] = 13;
      }
    }
  } else {
    for (uint32_t o = p.ul; o < p.uh; o++) kb[dst++] = uint8_t(key_byte<F>(S, o));
  }
}

// Same key, straight to global memory (chunks whose keys exceed the LDS buffer).
template <bool F>
__device__ __forceinline__ void build_key_global(const Src& S, const Desc& d, uint32_t schema, const RowParts& p,
                                                 uint8_t* out) {
  uint32_t n = 0;
  for (uint32_t i = 0; i < d.shared_len; i++) out[n++] = uint8_t(key_byte<F>(S, d.pb_data + i));
  for (uint32_t o = p.bl; o < p.bh; o++) out[n++] = uint8_t(key_byte<F>(S, o));
  for (uint32_t o = p.sl; o < p.sh; o++) out[n++] = uint8_t(key_byte<F>(S, o));
  if (schema == PBL_FMT_COL_CRDB1) {
    out[n++] = 0;
    if (p.wall == 0 && p.logical == 0) {
      if (p.uh > p.ul) {
        for (uint32_t o = p.ul; o < p.uh; o++) out[n++] = uint8_t(key_byte<F>(S, o));
        out[n++] = uint8_t(p.uh - p.ul + 1);
      }
    } else {
      for (int i = 0; i < 8; i++) out[n++] = uint8_t(p.wall >> (56 - 8 * i));
      if (p.logical == 0) {
        out[n++] = 9;
      } else {
        for (int i = 0; i < 4; i++) out[n++] = uint8_t(p.logical >> (24 - 8 * i));
        out[n++] = 13;
      }
    }
  } else {
    for (uint32_t o = p.ul; o < p.uh; o++) out[n++] = uint8_t(key_byte<F>(S, o));
  }
}

// bytes [a, a+16) of an LDS word array (a may be unaligned)
__device__ __forceinline__ uint4 lds_bytes16(lds_cu32 W, uint32_t a) {
  const uint32_t k = a >> 2, s = a & 3;
  const uint32_t w0 = W[k], w1 = W[k + 1], w2 = W[k + 2], w3 = W[k + 3], w4 = W[k + 4];
  return make_uint4(__builtin_amdgcn_alignbyte(w1, w0, s), __builtin_amdgcn_alignbyte(w2, w1, s),
                    __builtin_amdgcn_alignbyte(w3, w2, s), __builtin_amdgcn_alignbyte(w4, w3, s));
}

// 16 bytes starting `sh` bytes into the 32-byte pair (x, y)
__device__ __forceinline__ uint4 funnel16(const uint4& x, const uint4& y, uint32_t sh) {
  const uint32_t s = sh & 3;
  uint32_t d0, d1, d2, d3, d4;
  switch (sh >> 2) {
    case 0: d0 = x.x; d1 = x.y; d2 = x.z; d3 = x.w; d4 = y.x; break;
    case 1: d0 = x.y; d1 = x.z; d2 = x.w; d3 = y.x; d4 = y.y; break;
    case 2: d0 = x.z; d1 = x.w; d2 = y.x; d3 = y.y; d4 = y.z; break;
    default: d0 = x.w; d1 = y.x; d2 = y.y; d3 = y.z; d4 = y.w; break;
  }
  return make_uint4(__builtin_amdgcn_alignbyte(d1, d0, s), __builtin_amdgcn_alignbyte(d2, d1, s),
                    __builtin_amdgcn_alignbyte(d3, d2, s), __builtin_amdgcn_alignbyte(d4, d3, s));
}

// Stage block bytes [lo, lo + n) (lo a multiple of 16) into LDS granules.
__device__ __forceinline__ void stage(lds_u4 dst, const uint8_t* blocks, uint64_t boff, uint64_t a1, uint32_t lo,
                                      uint32_t n) {
  const uint64_t start = boff + lo;
  const uint32_t ph = uint32_t(start & 15);
  const uint4* G = reinterpret_cast<const uint4*>(blocks + (start & ~uint64_t(15)));
  const uint32_t n16 = (n + 15) >> 4;
  for (uint32_t g = threadIdx.x; g < n16; g += kTPB) {
    const uint4 x = G[g];
    if (ph == 0) { dst[g] = u32x4{x.x, x.y, x.z, x.w}; continue; }
    const uint64_t ynext = (start & ~uint64_t(15)) + 16ull * (g + 1);
    const uint4 y = ynext < a1 ? G[g + 1] : make_uint4(0, 0, 0, 0);
    const uint4 z = funnel16(x, y, ph);
    dst[g] = u32x4{z.x, z.y, z.z, z.w};
  }
}

__device__ __forceinline__ uint64_t block_sum_u64(uint64_t v, uint64_t* red) {
  v = wave_sum(v);
  if (lane_id() == 0) red[wave_id()] = v;
  __syncthreads();
  const uint64_t t = red[0] + red[1] + red[2] + red[3];
  __syncthreads();
  return t;
}

// Decode block b (format `schema`); the caller has taken ticket b.
template <bool F>
__device__ __forceinline__ void col_rows(Lds& s, const Args& A, uint32_t b, uint32_t schema, const Src& S);

__device__ __forceinline__ void col_block(Lds& s, const Args& A, uint32_t b, uint32_t schema) {
  const int t = threadIdx.x;
  const uint64_t boff = A.in.block_off[b];
  const uint32_t blen = A.in.block_len[b];
  const uint64_t a1 = (boff + blen + 15) & ~uint64_t(15);  // readable end (ABI: 16-B slack)
  const uint32_t nhead = blen < kStage ? blen : kStage;
  const uint32_t tail_lo = blen > kTail ? ((blen - kTail) & ~15u) : 0;
  stage((lds_u4)to_lds(s.head4), A.in.blocks, boff, a1, 0, nhead);
  stage((lds_u4)to_lds(s.tail4), A.in.blocks, boff, a1, tail_lo, blen - tail_lo);
  if (t == 0) { s.bad = 0; s.nhead = nhead; s.tail_lo = tail_lo; }
  __syncthreads();
  const Src S{(lds_cu8)to_lds(s.head4), (lds_cu8)to_lds(s.tail4), (glb_cu8)(A.in.blocks + boff), nhead, tail_lo,
              blen};
  if (wave_id() == 0) {
    const uint32_t st = parse_block_wave(S, schema, (A.in.flags & PBL_COL_TIERING) != 0, &s.d);
    if (lane_id() == 0) {
      s.d.status = st;
      s.status = st;
    }
  }
  __syncthreads();
  if (s.status == PBL_OK && s.d.key_end <= nhead) col_rows<true>(s, A, b, schema, S);
  else col_rows<false>(s, A, b, schema, S);
}

template <bool F>
__device__ __forceinline__ void col_rows(Lds& s, const Args& A, uint32_t b, uint32_t schema, const Src& S) {
  const int t = threadIdx.x;
  const pbl_decode_out& O = A.out;
  const uint32_t nb = A.in.n_blocks;
  uint8_t* ws = reinterpret_cast<uint8_t*>(O.workspace);
  uint64_t* lb_state = reinterpret_cast<uint64_t*>(ws + kWsHeader);
  const Desc& d = s.d;
  const bool hdr_ok = s.status == PBL_OK;
  const uint32_t rows = hdr_ok ? d.rows : 0;
  const uint32_t nch = (rows + kChunk - 1) / kChunk;

  // ---- pass 1: key lengths + bounds checks -----------------------------------
  RowParts p0;
  p0.klen = 0;
  p0.ok = true;
  uint64_t my_kb = 0;
  bool my_bad = false;
  for (uint32_t c = 0; c < nch; c++) {
    const uint32_t r = c * kChunk + t;
    if (r < rows) {
      RowParts p = row_parts<F>(S, d, schema, r);
      my_bad |= !p.ok || !value_ok(S, d, r);
      my_kb += p.klen;
      if (c == 0) p0 = p;
    }
  }
  if (my_bad) s.bad = 1;
  uint32_t excl0, tot0, dummy_e, dummy_t;
  block_excl_scan2(p0.klen, 0u, &excl0, &dummy_e, s.scratch, &tot0, &dummy_t);
  const uint64_t kb_tot = block_sum_u64(my_kb, s.red);  // (syncs; also orders s.bad)
  if (t == 0 && s.status == PBL_OK) {
    if (s.bad) s.status = PBL_CORRUPT_BOUNDS;
    else if (kb_tot > 0xffffffffull || uint64_t(d.v_hi - d.v_lo) > 0xffffffffull) s.status = PBL_UNSUPPORTED;
  }
  __syncthreads();
  const bool ok = s.status == PBL_OK;
  uint64_t agg[kNumComp] = {ok ? rows : 0u, ok ? kb_tot : 0ull, ok ? uint64_t(d.v_hi - d.v_lo) : 0ull, 0ull};
  if (wave_id() == 0) lb_publish(lb_state, nb, b, agg);

  // ---- build the (single-chunk) keys in LDS while the look-back resolves -------
  lds_u8 kb8 = (lds_u8)to_lds(s.key4);
  const bool prebuilt = ok && nch == 1 && tot0 <= kKeyBuf;
  if (prebuilt && uint32_t(t) < rows) build_key<F>(S, d, schema, p0, kb8, kKeyPad + excl0);
  if (wave_id() == 0) {
    uint64_t excl[kNumComp];
    lb_resolve(lb_state, nb, b, agg, excl, &O.totals->status_mask);
    if (lane_id() == 0) {
      uint32_t status = s.status;
      if (ok && overflows(O, excl, agg)) status = PBL_OVERFLOW;
      s.status = status;
#pragma unroll
      for (int c = 0; c < kNumComp; c++) s.bases[c] = excl[c];
      if (status != PBL_OK && O.key_off && excl[0] + b < O.kv_cap + nb) {
        O.key_off[excl[0] + b] = 0;
        O.val_off[excl[0] + b] = 0;
      }
      write_block_meta(O, b, nb, status, excl, agg, !F);
    }
  }
  __syncthreads();
  if (s.status != PBL_OK) return;
  const uint64_t kvb = s.bases[0], kbb = s.bases[1], vbb = s.bases[2];

  // ---- per-row arrays ------------------------------------------------------------
  const UCol& vo = d.v_off;
  for (uint32_t r = t; r <= rows; r += kTPB) {
    const uint32_t v = vo.w ? uint32_t(S.le(vo.at + r * vo.w, vo.w)) : 0;
    O.val_off[kvb + b + r] = v - d.v_lo;
    if (r < rows) {
      O.trailer[kvb + r] = with_seq(u_at<F>(S, d.trailers, r), A.in.synthetic_seq_num, 0u);
      if (O.kv_flags) {
        uint8_t fl = 0;
        if (d.pc_at && ((S.le(d.pc_at + 8 * (r >> 6), 8) >> (r & 63)) & 1)) fl |= PBL_KV_PREFIX_CHANGED;
        if (d.obs_at && ((S.le(d.obs_at + 8 * (r >> 6), 8) >> (r & 63)) & 1)) fl |= PBL_KV_OBSOLETE;
        if (d.ext_at && ((S.le(d.ext_at + 8 * (r >> 6), 8) >> (r & 63)) & 1)) {
          const uint32_t v1 = vo.w ? uint32_t(S.le(vo.at + (r + 1) * vo.w, vo.w)) : 0;
          const bool vb = v1 > v && (S.byte(d.v_data + v) & 0xC0) == 0x80;
          fl |= vb ? PBL_KV_VALBLK_HANDLE : PBL_KV_BLOB_HANDLE;
        }
        O.kv_flags[kvb + r] = fl;
      }
      if (O.entry_off) O.entry_off[kvb + r] = r;
      if (O.tiering_span_id) {  // decodeMeta (data_block.go:1633-1641)
        O.tiering_span_id[kvb + r] = u_at_any(S, d.span, r);
        O.tiering_attr[kvb + r] = u_at_any(S, d.attr, r);
      }
    }
  }

  // ---- key bytes --------------------------------------------------------------------
  if (prebuilt) {
    if (uint32_t(t) < rows) O.key_off[kvb + b + t] = excl0;
    if (t == 0) O.key_off[kvb + b + rows] = tot0;
    const uint64_t lo = kbb, hi = kbb + tot0;
    const lds_cu32 W = (lds_cu32)to_lds(s.key4);
    for (uint64_t ga = (lo & ~uint64_t(15)) + 16ull * t; ga < hi; ga += 16ull * kTPB)
      store16(O.key_bytes, ga, lo, hi, lds_bytes16(W, uint32_t(kKeyPad + ga - lo)));
  } else {
    uint32_t cbase = 0;
    for (uint32_t c = 0; c < nch; c++) {
      const uint32_t r = c * kChunk + t;
      RowParts p;
      p.klen = 0;
      if (r < rows) p = row_parts<F>(S, d, schema, r);
      uint32_t ex, tot, de, dt;
      block_excl_scan2(p.klen, 0u, &ex, &de, s.scratch, &tot, &dt);
      if (r < rows) O.key_off[kvb + b + r] = cbase + ex;
      if (tot <= kKeyBuf) {
        if (r < rows) build_key<F>(S, d, schema, p, kb8, kKeyPad + ex);
        __syncthreads();
        const uint64_t lo = kbb + cbase, hi = lo + tot;
        const lds_cu32 W = (lds_cu32)to_lds(s.key4);
        for (uint64_t ga = (lo & ~uint64_t(15)) + 16ull * t; ga < hi; ga += 16ull * kTPB)
          store16(O.key_bytes, ga, lo, hi, lds_bytes16(W, uint32_t(kKeyPad + ga - lo)));
      } else if (r < rows) {
        build_key_global<F>(S, d, schema, p, O.key_bytes + kbb + cbase + ex);
      }
      cbase += tot;
      __syncthreads();
    }
    if (t == 0) O.key_off[kvb + b + rows] = cbase;
  }

  // ---- value bytes: one contiguous range, global -> global --------------------
  {
    const uint64_t src_lo = A.in.block_off[b] + d.v_data + d.v_lo;  // in `blocks`
    const uint64_t n = d.v_hi - d.v_lo;
    const uint64_t lo = vbb, hi = vbb + n;
    const gptr<const uint8_t> G = to_glb(A.in.blocks);
    for (uint64_t ga = (lo & ~uint64_t(15)) + 16ull * t; ga < hi; ga += 16ull * kTPB) {
      // source bytes for destination [ga, ga+16): [sx, sx+16), sx may precede src_lo
      const int64_t sx = int64_t(src_lo) + int64_t(ga) - int64_t(lo);
      const int64_t sa = sx & ~int64_t(15);
      const uint32_t sh = uint32_t(sx - sa);
      const int64_t s_end = int64_t(src_lo + n);
      uint4 x = make_uint4(0, 0, 0, 0), y = make_uint4(0, 0, 0, 0);
      if (sa + 16 > int64_t(src_lo) && sa < s_end) {
        const u32x4 v = *(gptr<const u32x4>)(G + sa);
        x = make_uint4(v.x, v.y, v.z, v.w);
      }
      if (sh && sa + 32 > int64_t(src_lo) && sa + 16 < s_end) {
        const u32x4 v = *(gptr<const u32x4>)(G + sa + 16);
        y = make_uint4(v.x, v.y, v.z, v.w);
      }
      store16(O.val_bytes, ga, lo, hi, sh ? funnel16(x, y, sh) : x);
    }
  }
}

// Row r's isObsolete bit (data_block.go:519; HideObsoletePoints skips such
// rows, :1680-1697) and the values column's offset r.
__device__ __forceinline__ bool row_obsolete(const Src& S, const Desc& d, uint32_t r) {
  return d.obs_at && ((S.le(d.obs_at + 8 * (r >> 6), 8) >> (r & 63)) & 1);
}
__device__ __forceinline__ uint32_t row_voff(const Src& S, const Desc& d, uint32_t r) {
  return d.v_off.w ? uint32_t(S.le(d.v_off.at + r * d.v_off.w, d.v_off.w)) : 0u;
}

}  // namespace col
}  // namespace pbl
