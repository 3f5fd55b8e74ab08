// rowblk_pool.hip.h — the row-format decode with one wave per block, eight
// waves per CU and a shared pool of LDS staging buffers.
//
// Only the parse needs a block's bytes in LDS; the keys and the value bytes
// (80 % of the output) are gathered global->global from the block that was
// just read (L2 / MALL-hot) through compact per-KV metadata in the wave's own
// slot.  So a 32 KiB stage is held only for the DMA, the walk and the
// metadata pass, and the other waves stage their blocks while this one emits.
//
//   acquire   a wave takes a free stage from the workgroup's pool (LDS mask),
//             THEN a ticket (the only order that keeps the look-back
//             deadlock-free: every ticket holder either holds a stage or has
//             published its aggregate)
//   stage     the block HBM -> LDS by LDS-DMA, one round trip
//   walk      lane per restart run (rowblk_writer.go:147-155 cuts the prefix
//             chain there): headers parked in registers, a DPP scan places the
//             runs, the block's aggregate is published
//   meta      per-entry metadata words (key source, shared and key length,
//             prefix parent, header length, flags) and per-KV value offsets
//             written from the registers into the slot; the stage is released
//   resolve   the exclusive prefix by decoupled look-back, issued together
//             with the first step's and the restart words' loads
//   steps     64 KVs per step, keys and values together (a line of the block
//             is fetched once for both), each step's loads issued before the
//             previous step's stores:
//               keys    lane per KV: offsets (a wave scan of the key lengths),
//                       trailer, flags, entry offset, the user key merged from
//                       its prefix chain
//               values  8 lanes per KV, 16-B chunks
//
// LDS per CU: 3 stages x 32.8 KB + 8 slots x ~8 KB (one per wave).
//
// Blocks outside the fast-path limits (more entries than a slot holds, keys
// past kMaxKl, 3-byte header varints, ...) take the wave-serial general walk
// (rowblk_general.hip.h) on the staged bytes; blocks past kMaxFastLen are sized
// by big_block_sizes_kernel before this launch and written by the wave that
// draws their ticket (block_big; rowblk_big.hip.h).  Results are identical on
// every path.
//
// Semantics: cockroachdb/pebble sstable/rowblk/rowblk_iter.go — Init :241-276,
// readFirstKey :418-485, readEntry :333-416, decodeInternalKey :487-504, value
// prefix :1192-1199 (sstable/block/kv.go:14-41), decodeRestart :1092-1096,
// HideObsoletePoints :1168-1179.
#pragma once

namespace pool {

#ifndef PBL_POOL_WAVES
#define PBL_POOL_WAVES 8
#endif
#ifndef PBL_POOL_STAGES
#define PBL_POOL_STAGES 3
#endif
#ifndef PBL_POOL_SLEEP
#define PBL_POOL_SLEEP 8  // s_sleep units (64 cycles) between polls of the stage mask
#endif
#ifndef PBL_POOL_PRIO
#define PBL_POOL_PRIO 2  // the stage holder's issue priority (the emits run at 0)
#endif
constexpr int kNW = PBL_POOL_WAVES;      // waves per workgroup (one workgroup per CU)
constexpr int kNS = PBL_POOL_STAGES;     // staging buffers per workgroup
constexpr int kTPBP = kNW * kWave;
constexpr uint32_t kMaxKl = 4095;        // internal-key bytes per entry on the fast path

// A stage: the block, byte i at kPad + (boff & 15) + i.
struct Stage {
  uint4 x[kLdsBlkBytes / 16];
};

// Per-entry metadata word (m0): key source offset (15 bits: blocks <= 32 KiB),
// shared length (12), internal key length (12), prefix parent (9), entry
// header length (4), PBL_KV_* flags (8; OBSOLETE is added at emit time).
__device__ __forceinline__ uint32_t m_ksrc(uint64_t m) { return uint32_t(m) & 0x7fffu; }
__device__ __forceinline__ uint32_t m_sh(uint64_t m) { return uint32_t(m >> 15) & 0xfffu; }
__device__ __forceinline__ uint32_t m_klen(uint64_t m) { return uint32_t(m >> 27) & 0xfffu; }
__device__ __forceinline__ uint32_t m_par(uint64_t m) { return uint32_t(m >> 39) & 0x1ffu; }
__device__ __forceinline__ uint32_t m_hl(uint64_t m) { return uint32_t(m >> 48) & 0xfu; }
__device__ __forceinline__ uint32_t m_fl(uint64_t m) { return uint32_t(m >> 52) & 0xffu; }
__device__ __forceinline__ uint64_t m_pack(uint32_t ksrc, uint32_t sh, uint32_t kl, uint32_t par, uint32_t hl,
                                           uint32_t fl) {
  return uint64_t(ksrc) | uint64_t(sh) << 15 | uint64_t(kl) << 27 | uint64_t(par) << 39 | uint64_t(hl) << 48 |
         uint64_t(fl) << 52;
}

// A slot (one block's metadata, what the emits need after the stage is gone):
// m0 by entry (the prefix-parent chain runs over every entry), vp and ent by
// visible KV (HideObsoletePoints drops obsolete entries from the outputs, never
// from the chain; without hiding the two indices agree).  Entries per slot:
// what the LDS left after the stages holds, at most 511 (the parent field).
constexpr int kPerSlot = (163840 - kNS * int(sizeof(Stage)) - 256) / kNW;
template <bool kHide>
constexpr int slot_kv() {
  const int n = ((kPerSlot - 32) / (kHide ? 14 : 12)) & ~7;
  return n > 511 ? 511 : n;
}
template <bool kHide>
struct Slot {
  static constexpr int kKv = slot_kv<kHide>();
  uint64_t m0[kKv];
  uint32_t vp[kKv + 5];  // value output offset | value source offset << 16;
                         // entries nkv..nkv+4 hold the value total
  uint16_t ent[kHide ? kKv : 1];  // the entry of visible KV v
};

template <bool kHide>
struct PoolLds {
  Stage st[kNS];
  Slot<kHide> sl[kNW];
  uint32_t free_mask;  // bit s: stage s is free
};
static_assert(sizeof(PoolLds<true>) <= 163840 && sizeof(PoolLds<false>) <= 163840, "one pool workgroup per CU");

typedef u32x4 u32x4_ug __attribute__((aligned(1)));
typedef uint32_t u32_ug __attribute__((aligned(1)));
typedef uint64_t u64_ug __attribute__((aligned(1)));
typedef uint16_t u16_ug __attribute__((aligned(1)));

// Inclusive wave scan by DPP row shifts and row broadcasts (no ds_bpermute).
__device__ __forceinline__ uint32_t dpp_incl_scan(uint32_t v) {
  v += __builtin_amdgcn_update_dpp(0u, v, 0x111, 0xf, 0xf, false);  // row_shr:1
  v += __builtin_amdgcn_update_dpp(0u, v, 0x112, 0xf, 0xf, false);  // row_shr:2
  v += __builtin_amdgcn_update_dpp(0u, v, 0x114, 0xf, 0xf, false);  // row_shr:4
  v += __builtin_amdgcn_update_dpp(0u, v, 0x118, 0xf, 0xf, false);  // row_shr:8
  v += __builtin_amdgcn_update_dpp(0u, v, 0x142, 0xa, 0xf, false);  // row_bcast:15
  v += __builtin_amdgcn_update_dpp(0u, v, 0x143, 0xc, 0xf, false);  // row_bcast:31
  return v;
}
__device__ __forceinline__ uint32_t last_lane(uint32_t v) { return __builtin_amdgcn_readlane(v, kWave - 1); }

// Output stores.  PBL_POOL_NT: non-temporal (streaming) stores, so the
// outputs do not displace the staged blocks' lines that the emit re-reads
// from L2 (A/B).
#ifndef PBL_POOL_NT
#define PBL_POOL_NT 1  // measured: config 2 1200 vs 1183, config 4 1073 vs 1062 GiB/s
#endif
template <class T>
__device__ __forceinline__ void st_out(gptr<T> p, T v) {
#if PBL_POOL_NT
  __builtin_nontemporal_store(v, p);
#else
  *p = v;
#endif
}

// Bytes [0, n) of w (n <= 16) to p, any alignment: one 16-B store when whole,
// else the fewest 8/4/2/1-B stores (nothing past n: the next key belongs to
// another lane).
__device__ __forceinline__ void store_n(gptr<uint8_t> p, const uint4& w, uint32_t n) {
  if (n == 16) {
    st_out((gptr<u32x4_ug>)p, u32x4_ug{w.x, w.y, w.z, w.w});
    return;
  }
  uint64_t lo = uint64_t(w.x) | uint64_t(w.y) << 32, hi = uint64_t(w.z) | uint64_t(w.w) << 32;
  uint32_t o = 0;
  if (n & 8) {
    st_out((gptr<u64_ug>)p, u64_ug(lo));
    lo = hi;
    o = 8;
  }
  if (n & 4) {
    st_out((gptr<u32_ug>)(p + o), u32_ug(lo));
    lo >>= 32;
    o += 4;
  }
  if (n & 2) {
    st_out((gptr<u16_ug>)(p + o), u16_ug(lo));
    lo >>= 16;
    o += 2;
  }
  if (n & 1) st_out(p + o, uint8_t(lo));
}

// 16 bytes of the block in global memory at block offset i (any alignment,
// i may be up to 15 below 0 or end past the block: those bytes are
// don't-cares).  One unaligned load inside the block's 16-B granules; at the
// two edges the general path's aligned pair (never a byte outside them).
__device__ __forceinline__ uint4 gld16(gptr<const uint8_t> g, int32_t i, uint32_t blen, uint32_t end16) {
  if (i >= 0 && uint32_t(i) + 16u <= end16) {
    const u32x4 v = *(gptr<const u32x4_ug>)(g + i);
    return make_uint4(v.x, v.y, v.z, v.w);
  }
  return SlowGlb{g, blen}.ld16(i);
}

// ---- the walk: lane per restart run ------------------------------------------
// Entries are indexed in block order (the prefix-parent chain runs over every
// entry); outputs by visible index (HideObsoletePoints drops obsolete entries
// from the outputs, never from the chain).  Without hiding the two agree.
struct PAcc {
  uint32_t ne, cnt, kb, vb;  // entries, visible KVs, their user-key / value bytes
};
#ifndef PBL_POOL_RUNBUF
#define PBL_POOL_RUNBUF 16  // entries of a run parked in registers by its walk
#endif
constexpr int kRunBuf = PBL_POOL_RUNBUF;
// One run's head, parked in registers by the walk for the metadata pass.
struct PRun {
  uint32_t ea[kRunBuf];  // entry offset | hidden << 15 | shared << 16 | SET-with-value-prefix << 31
  uint32_t eb[kRunBuf];  // unshared | header length << 14 | value length << 17
  uint32_t n, rw, pos, e0, prev_kl, prev_kind;  // parked entries; where a longer run continues
};

// Whether an entry is hidden (HideObsoletePoints: the trailer's kind byte has
// the obsolete bit, rowblk_iter.go:1168-1179) and whether its value carries a
// value prefix (kind SET, :1192-1199).  The kind byte sits at key byte kl - 8:
// in the entry's unshared bytes, or inside the shared prefix, where it is the
// previous key's kind byte if that key has the same length.  Returns false
// when the byte is elsewhere (the general walk takes the block).
template <bool kHide>
__device__ __forceinline__ bool entry_class(const View& V, uint32_t pos, uint32_t h, uint32_t sh, uint32_t kl,
                                            uint32_t k, uint32_t prev_kl, uint32_t& prev_kind, uint32_t flags,
                                            bool vprefix, bool& hidden, bool& setv) {
  hidden = false;
  setv = false;
  if ((kHide || vprefix) && kl >= 8 && !(flags & PBL_ROW_RAW_KEYS)) {
    uint32_t kind;
    if (kl - 8 >= sh) kind = V.byte(pos + h + (kl - 8 - sh));
    else if (k > 0 && prev_kl == kl) kind = prev_kind;
    else return false;
    hidden = kHide && (kind & 64u);
    setv = vprefix && !hidden && (kind & 0xBFu) == 1;
    prev_kind = kind;
  }
  return true;
}

__device__ __forceinline__ uint32_t ukey_len(uint32_t kl, uint32_t flags) {
  return (flags & PBL_ROW_RAW_KEYS) ? kl : (kl >= 8 ? kl - 8 : 0);
}

// Count entries [pos, e0) of a run whose first k entries were already counted
// (prev_kl / prev_kind: the last one's).  `ok` clears where the run is not
// walkable per run, `bad` sets on shared > len(previous key) (rowblk_iter.go:
// 403), `vbad` on a visible SET value without its prefix byte.
template <bool kHide>
__device__ __forceinline__ void count_span(const View& V, uint32_t pos, uint32_t e0, uint32_t k, uint32_t prev_kl,
                                           uint32_t prev_kind, uint32_t flags, bool vprefix, PAcc& acc, bool& ok,
                                           bool& bad, bool& vbad) {
  while (pos < e0) {
    uint32_t sh, un, vl, h;
    const bool hok = rowc::hdr2(V.ld8(pos), &sh, &un, &vl, &h);
    const uint32_t np = pos + h + un + vl;  // < 2^23: no overflow
    if (!hok || (k == 0 && sh != 0) || np > e0) { ok = false; return; }
    bad = bad || (k > 0 && sh > prev_kl);
    const uint32_t kl = sh + un;
    bool hidden, setv;
    if (kl > kMaxKl || !entry_class<kHide>(V, pos, h, sh, kl, k, prev_kl, prev_kind, flags, vprefix, hidden, setv)) {
      ok = false;
      return;
    }
    uint32_t vlen = vl;
    if (setv) {
      if (vl == 0) vbad = true;
      else if ((V.byte(pos + h + un) & 0xC0) == 0 || (flags & PBL_ROW_NO_VALUER)) vlen--;
    }
    acc.ne++;
    if (!hidden) {
      acc.cnt++;
      acc.kb += ukey_len(kl, flags);
      acc.vb += vlen;
    }
    k++;
    prev_kl = kl;
    pos = np;
  }
}

__device__ __forceinline__ bool run_bounds(const View& V, uint32_t r, uint32_t nres, uint32_t roff, uint32_t* rw,
                                           uint32_t* e0) {
  const uint32_t st = roff + 4 * r;
  *rw = V.le32(st);
  const uint32_t s0 = *rw & kRestartMask;
  *e0 = (r + 1 < nres) ? (V.le32(st + 4) & kRestartMask) : roff;
  return (r != 0 || s0 == 0) && s0 < *e0 && *e0 <= roff;
}

// Walk run r once, its first kRunBuf entries parked in registers (static
// indices: no scratch); `over` sets if the run is longer.
template <bool kHide>
__device__ __forceinline__ void run_walk(const View& V, uint32_t r, uint32_t nres, uint32_t roff, uint32_t flags,
                                         bool vprefix, PRun& B, PAcc& acc, bool& ok, bool& bad, bool& vbad,
                                         bool& over) {
  B.n = 0;
  uint32_t e0;
  if (!run_bounds(V, r, nres, roff, &B.rw, &e0)) { ok = false; return; }
  uint32_t pos = B.rw & kRestartMask, n = 0, prev_kl = 0, prev_kind = 0;
  bool go = true;
#pragma unroll
  for (int k = 0; k < kRunBuf; k++) {
    if (go && pos < e0) {
      uint32_t sh, un, vl, h;
      const bool hok = rowc::hdr2(V.ld8(pos), &sh, &un, &vl, &h);
      const uint32_t np = pos + h + un + vl;
      bool hidden = false, setv = false;
      if (!hok || (k == 0 && sh != 0) || np > e0) {
        ok = false;
        go = false;
      } else {
        bad = bad || (k > 0 && sh > prev_kl);
        const uint32_t kl = sh + un;
        if (kl > kMaxKl ||
            !entry_class<kHide>(V, pos, h, sh, kl, uint32_t(k), prev_kl, prev_kind, flags, vprefix, hidden, setv)) {
          ok = false;
          go = false;
        } else {
          uint32_t vlen = vl;
          if (setv) {
            if (vl == 0) vbad = true;
            else if ((V.byte(pos + h + un) & 0xC0) == 0 || (flags & PBL_ROW_NO_VALUER)) vlen--;
          }
          B.ea[k] = pos | uint32_t(hidden) << 15 | sh << 16 | uint32_t(setv) << 31;
          B.eb[k] = un | (h << 14) | (vl << 17);
          acc.ne++;
          if (!hidden) {
            acc.cnt++;
            acc.kb += ukey_len(kl, flags);
            acc.vb += vlen;
          }
          n++;
          prev_kl = kl;
          pos = np;
        }
      }
    }
  }
  if (go && pos < e0) over = true;
  B.n = n;
  B.pos = pos;
  B.e0 = e0;
  B.prev_kl = prev_kl;
  B.prev_kind = prev_kind;
}

// Chain and output state of the metadata pass, carried from one entry of a run
// to the next: entry / visible index, value output offset, the previous
// entry's shared length, its prefix parent and that parent's shared length.
struct MState {
  uint32_t e, v, vb, prev_sh, pp, ppsh;
};

// Metadata of one entry (validated by the walk).  The prefix parent is the
// nearest earlier entry of the run with a smaller shared length (all-nearest-
// smaller-values over the parents, amortised O(1)).
template <bool kHide>
__device__ __forceinline__ void entry_meta(Slot<kHide>& W, const View& V, uint32_t pos, bool hidden, uint32_t sh,
                                           uint32_t un, uint32_t h, uint32_t vl, bool setv, bool first, uint32_t rw,
                                           uint32_t flags, MState& M) {
  const uint32_t kl = sh + un;
  uint32_t par = M.e, parsh = 0;
  if (sh != 0) {
    uint32_t c = M.e - 1, csh = M.prev_sh;
    if (csh >= sh) { c = M.pp; csh = M.ppsh; }
    while (csh >= sh) {
      c = m_par(W.m0[c]);
      csh = m_sh(W.m0[c]);
    }
    par = c;
    parsh = csh;
  }
  uint32_t vs = pos + h + un, vlen = vl, fl = 0;
  if (first) fl = PBL_KV_RESTART | ((rw >> 31) ? PBL_KV_RESTART_SAMEPFX : 0u);
  if (!(flags & PBL_ROW_RAW_KEYS) && kl < 8) fl |= PBL_KV_INVALID_KEY;
  if (setv) {
    const uint32_t pre = V.byte(vs);
    if ((pre & 0xC0) == 0 || (flags & PBL_ROW_NO_VALUER)) { vs++; vlen--; }
    else if ((pre & 0xC0) == 0x80) fl |= PBL_KV_VALBLK_HANDLE;
    else fl |= PBL_KV_BLOB_HANDLE;
  }
  W.m0[M.e] = m_pack(pos + h, sh, kl, par, h, fl);
  if (!(kHide && hidden)) {
    if (kHide) W.ent[M.v] = uint16_t(M.e);
    W.vp[M.v] = M.vb | (vs << 16);
    M.vb += vlen;
    M.v++;
  }
  M.prev_sh = sh;
  M.pp = par;
  M.ppsh = parsh;
  M.e++;
}

// Metadata of the parked entries of a run.
template <bool kHide>
__device__ __forceinline__ void park_meta(Slot<kHide>& W, const View& V, const PRun& B, uint32_t flags, MState& M) {
#pragma unroll
  for (int k = 0; k < kRunBuf; k++) {
    if (uint32_t(k) < B.n)
      entry_meta<kHide>(W, V, B.ea[k] & 0x7fffu, (B.ea[k] >> 15) & 1u, (B.ea[k] >> 16) & 0x7fffu,
                        B.eb[k] & 0x3fffu, (B.eb[k] >> 14) & 7u, B.eb[k] >> 17, B.ea[k] >> 31, k == 0, B.rw, flags, M);
  }
}

// Metadata of entries [pos, e0) of a run, re-read from the stage (k = entries
// of the run before pos; prev_kl / prev_kind: the last one's).
template <bool kHide>
__device__ __forceinline__ void span_meta(Slot<kHide>& W, const View& V, uint32_t pos, uint32_t e0, uint32_t rw,
                                          uint32_t k, uint32_t prev_kl, uint32_t prev_kind, uint32_t flags,
                                          bool vprefix, MState& M) {
  while (pos < e0) {
    uint32_t sh, un, vl, h;
    rowc::hdr2(V.ld8(pos), &sh, &un, &vl, &h);
    const uint32_t kl = sh + un;
    bool hidden, setv;
    entry_class<kHide>(V, pos, h, sh, kl, k, prev_kl, prev_kind, flags, vprefix, hidden, setv);
    entry_meta<kHide>(W, V, pos, hidden, sh, un, h, vl, setv, k == 0, rw, flags, M);
    k++;
    prev_kl = kl;
    pos = pos + h + un + vl;
  }
}

// The block's bytes in global memory for the emits (the stage is gone by
// then).  ld16 windows may start up to 15 bytes before the block.
struct GSrc {
  gptr<const uint8_t> g;
  uint32_t blen, end16;
  __device__ __forceinline__ uint32_t byte(uint32_t i) const { return g[i]; }
  __device__ __forceinline__ uint64_t ld8(uint32_t i) const { return *(gptr<const u64_ug>)(g + i); }
  __device__ __forceinline__ uint32_t le32(uint32_t i) const { return *(gptr<const u32_ug>)(g + i); }
  __device__ __forceinline__ uint4 ld16(int32_t i) const { return gld16(g, i, blen, end16); }
};

// byte p of the internal key of entry j (source = max{i <= j : shared_i <= p})
template <class Src>
__device__ __forceinline__ uint32_t key_byte(const uint64_t* M0, const Src& V, int j, uint32_t p) {
  uint64_t m = M0[j];
  while (p < m_sh(m)) m = M0[--j];
  return V.byte(m_ksrc(m) + p - m_sh(m));
}

template <class Src>
__device__ __forceinline__ uint64_t trailer_of(const uint64_t* M0, const Src& V, int j, uint64_t m, uint32_t* fl,
                                               uint32_t flags) {
  if (flags & PBL_ROW_RAW_KEYS) return 0;
  const uint32_t kl = m_klen(m);
  if (kl < 8) return kKindInvalid;
  const uint32_t sh = m_sh(m);
  uint64_t raw;
  if (kl - 8 >= sh) {
    raw = V.ld8(m_ksrc(m) + (kl - 8 - sh));
  } else {
    raw = 0;
    for (int i = 0; i < 8; i++) raw |= uint64_t(key_byte(M0, V, j, kl - 8 + i)) << (8 * i);
  }
  if (raw & 64u) *fl |= PBL_KV_OBSOLETE;
  return raw & kTrailerObsoleteMask;
}

// Key bytes [c, c + n) of KV m (n <= 16) merged from the segments of its prefix
// chain: each a 16-B read that starts where the chunk's first byte would sit in
// that entry (at most 15 bytes before the block).
template <class Src>
__device__ __forceinline__ uint4 key_chunk(const uint64_t* M0, const Src& V, uint64_t m, uint32_t c, uint32_t n) {
  const uint32_t ce = c + n;
  uint32_t cur = ce;
  uint4 w = make_uint4(0, 0, 0, 0);
  for (;;) {
    const uint32_t shi = m_sh(m);
    const uint32_t lo_i = shi < cur ? shi : cur;
    const uint32_t a = lo_i > c ? lo_i : c;
    if (a < cur) {
      const uint4 v = V.ld16(int32_t(m_ksrc(m)) - int32_t(shi) + int32_t(c));
      if (a == c && cur - a == 16) return v;
      merge16(w, v, a - c, cur - c);
    }
    if (lo_i <= c) break;
    cur = lo_i;
    m = M0[m_par(m)];
  }
  return w;
}

// ---- keys: lane per KV, kKU KVs per lane per batch ---------------------------
// The loads are L2 / MALL round trips, so a batch goes through its metadata
// words (slot), then every global load (the trailer's 8 bytes; the user key's
// segments: its own unshared bytes and, for a key that shares a prefix, its
// prefix parent's bytes), then the merges and stores.  The fast form covers
// keys of at most 16 bytes whose prefix chain ends at the parent (a restart-
// interval row block: the parent is the run's first key) with the trailer in
// the entry's own bytes; the rest take the general form (trailer_of,
// key_chunk).  Only the loaded data and the words they were addressed by are
// held between the loads and the stores.
#ifndef PBL_POOL_KU
#define PBL_POOL_KU 1
#endif
constexpr int kKU = PBL_POOL_KU;
// PBL_POOL_KMETA 0: the metadata words are not held between a batch's loads
// and its stores (re-read from the slot: two LDS reads, fewer VGPRs per
// step in flight).
#ifndef PBL_POOL_KMETA
#define PBL_POOL_KMETA 1
#endif
struct KBatch {
#if PBL_POOL_KMETA
  uint64_t m[kKU], mp[kKU];
#endif
  uint64_t tr[kKU];
  uint4 ka[kKU], kp[kKU];
};
// The metadata word of visible KV j and its prefix parent's (0 past nkv).
template <bool kHide>
__device__ __forceinline__ void kv_meta(const Slot<kHide>& W, uint32_t j, uint32_t nkv, uint64_t* m, uint64_t* mp) {
  const uint32_t e = kHide ? (j < nkv ? uint32_t(W.ent[j]) : 0u) : j;
  *m = j < nkv ? W.m0[e] : 0ull;
  *mp = (j < nkv && m_sh(*m) != 0) ? W.m0[m_par(*m)] : 0ull;
}

__device__ __forceinline__ uint32_t ukl_of(uint64_t m, bool raw) {
  const uint32_t kl = m_klen(m);
  return raw ? kl : (kl >= 8 ? kl - 8 : 0u);
}
__device__ __forceinline__ bool key_fast(uint64_t m, uint64_t mp, bool raw) {
  const uint32_t kl = m_klen(m), sh = m_sh(m);
  return ukl_of(m, raw) <= 16 && (sh == 0 || m_sh(mp) == 0) && (raw || kl < 8 || kl - 8 >= sh);
}

template <bool kHide, class Src>
__device__ __forceinline__ void key_load(const Slot<kHide>& W, const Src& V, bool raw, uint32_t j0, uint32_t nkv,
                                         KBatch& K) {
  const int l = lane_id();
  uint64_t Km[kKU], Kmp[kKU];
#pragma unroll
  for (int u = 0; u < kKU; u++) kv_meta<kHide>(W, j0 + kWave * u + l, nkv, &Km[u], &Kmp[u]);
#if PBL_POOL_KMETA
#pragma unroll
  for (int u = 0; u < kKU; u++) {
    K.m[u] = Km[u];
    K.mp[u] = Kmp[u];
  }
#endif
#pragma unroll
  for (int u = 0; u < kKU; u++) {
    const uint32_t j = j0 + kWave * u + l;
    const uint64_t m = Km[u];
    const uint32_t kl = m_klen(m), sh = m_sh(m), ukl = ukl_of(m, raw);
    const bool fast = j < nkv && key_fast(m, Kmp[u], raw);
    K.tr[u] = 0;
    if (fast && !raw && kl >= 8) K.tr[u] = V.ld8(m_ksrc(m) + (kl - 8 - sh));
    if (fast && ukl) K.ka[u] = V.ld16(int32_t(m_ksrc(m)) - int32_t(sh));
    if (fast && ukl && sh) K.kp[u] = V.ld16(int32_t(m_ksrc(Kmp[u])));
  }
}

// A user key off the fast form (longer than 16 bytes, or a deeper prefix
// chain): the chunks that reach into the shared prefix are merged along the
// chain; the rest lie in the entry's own bytes and go four 16-B loads at a
// time (the loads of a step in flight together).
#ifndef PBL_POOL_KOWN
#define PBL_POOL_KOWN 4
#endif
// Keys whose own bytes run past kWaveKey leave those to the whole wave
// (wave_key_own): only the chunks that reach into the shared prefix are
// stored here.
#ifndef PBL_POOL_WAVEKEY
#define PBL_POOL_WAVEKEY 128
#endif
constexpr uint32_t kWaveKey = PBL_POOL_WAVEKEY;
__device__ __forceinline__ bool wave_key(uint32_t ukl, uint32_t sh) { return ukl > kWaveKey && ukl >= sh + 16; }
template <class Src>
__device__ __forceinline__ void store_key_general(const uint64_t* M0, const Src& V, uint64_t m, uint32_t ukl,
                                                  gptr<uint8_t> dst) {
  const uint32_t sh = m_sh(m);
  const int32_t own = int32_t(m_ksrc(m)) - int32_t(sh);  // block offset of key byte 0 in the entry's bytes
  uint32_t c = 0;
  for (; c < ukl && c < sh; c += 16) {
    const uint32_t n = ukl - c < 16 ? ukl - c : 16u;
    store_n(dst + c, key_chunk(M0, V, m, c, n), n);
  }
  if (wave_key(ukl, sh)) return;
  for (; c < ukl; c += 16 * PBL_POOL_KOWN) {
    uint4 w[PBL_POOL_KOWN];
#pragma unroll
    for (int k = 0; k < PBL_POOL_KOWN; k++) {
      const uint32_t cc = c + 16 * k;
      w[k] = cc < ukl ? V.ld16(own + int32_t(cc)) : make_uint4(0, 0, 0, 0);
    }
#pragma unroll
    for (int k = 0; k < PBL_POOL_KOWN; k++) {
      const uint32_t cc = c + 16 * k;
      if (cc < ukl) store_n(dst + cc, w[k], ukl - cc < 16 ? ukl - cc : 16u);
    }
  }
}

// The batch's stores.  Key output offsets: an exclusive wave scan of the user-
// key lengths per u, `kcar` carrying the running total (KV nkv gets the total).
// kPart (the two-pass row emit splits the stores over two waves): 0 all, 1 all
// but the long keys' own bytes, 2 only those (K unused).
template <bool kHide, class Src, int kPart = 0>
__device__ __forceinline__ void key_store(const Slot<kHide>& W, const Src& V, const Args& A, uint32_t b, uint32_t j0,
                                          uint32_t nkv, uint64_t kvb, uint64_t kbb, const KBatch& K, uint32_t& kcar) {
  const int l = lane_id();
  const uint32_t flags = A.in.flags;
  const pbl_decode_out& O = A.out;
  const gptr<uint8_t> kbytes = to_glb(O.key_bytes) + kbb;
  const bool raw = (flags & PBL_ROW_RAW_KEYS) != 0;
  uint32_t kc0[kKU];
  uint64_t Km[kKU], Kmp[kKU];
#pragma unroll
  for (int u = 0; u < kKU; u++) {
#if PBL_POOL_KMETA
    if (kPart != 2) {
      Km[u] = K.m[u];
      Kmp[u] = K.mp[u];
      continue;
    }
#endif
    kv_meta<kHide>(W, j0 + kWave * u + l, nkv, &Km[u], &Kmp[u]);
  }
#pragma unroll
  for (int u = 0; u < kKU; u++) {
    const uint32_t j = j0 + kWave * u + l;
    const uint64_t m = Km[u];
    const uint32_t ukl = j < nkv ? ukl_of(m, raw) : 0u;
    const uint32_t incl = dpp_incl_scan(ukl);
    kc0[u] = kcar;
    const uint32_t ko = kcar + incl - ukl;
    kcar += last_lane(incl);
    if (kPart == 2 || j > nkv) continue;
    st_out(to_glb(O.key_off) + (kvb + b + j), ko);
    st_out(to_glb(O.val_off) + (kvb + b + j), uint32_t(W.vp[j] & 0xffffu));
    if (j == nkv) continue;
    const uint32_t kl = m_klen(m), sh = m_sh(m);
    uint64_t t;
    uint32_t f = m_fl(m);
    if (!key_fast(m, Kmp[u], raw)) {
      const uint32_t e = kHide ? uint32_t(W.ent[j]) : j;
      t = trailer_of(W.m0, V, int(e), m, &f, flags);
      store_key_general(W.m0, V, m, ukl, kbytes + ko);
    } else {
      if (raw) t = 0;
      else if (kl < 8) t = kKindInvalid;
      else {
        if (K.tr[u] & 64u) f |= PBL_KV_OBSOLETE;
        t = K.tr[u] & kTrailerObsoleteMask;
      }
      if (ukl) {
        const uint32_t lo = sh < ukl ? sh : ukl;
        uint4 w = K.ka[u];
        if (lo) {
          w = make_uint4(0, 0, 0, 0);
          merge16(w, K.ka[u], lo, ukl);
          merge16(w, K.kp[u], 0, lo);
        }
        store_n(kbytes + ko, w, ukl);
      }
    }
    st_out(to_glb(O.trailer) + (kvb + j), uint64_t(with_seq(t, A.in.synthetic_seq_num, flags)));
    if (O.kv_flags) st_out(to_glb(O.kv_flags) + (kvb + j), uint8_t(f));
    if (O.entry_off) st_out(to_glb(O.entry_off) + (kvb + j), uint32_t(m_ksrc(m) - m_hl(m)));
  }
  if (kPart == 1) return;
  // the own bytes [shared, ukl) of long keys: one contiguous range of the
  // entry each, copied by the whole wave (16-B chunks, the last one ending at
  // the key's end, four per lane in flight)
#pragma unroll
  for (int u = 0; u < kKU; u++) {
    const uint32_t j = j0 + kWave * u + l;
    const uint64_t m = Km[u];
    const uint32_t ukl = j < nkv ? ukl_of(m, raw) : 0u, sh = m_sh(m);
    const bool wk = j < nkv && !key_fast(m, Kmp[u], raw) && wave_key(ukl, sh);
    const uint32_t incl = dpp_incl_scan(ukl);  // (the batch's key offsets again)
    const uint32_t ko = kc0[u] + incl - ukl;
    for (uint64_t lm = __ballot(wk); lm; lm &= lm - 1) {
      const int sl = __builtin_ctzll(lm);
      const int32_t src = __shfl(int32_t(m_ksrc(m)), sl, kWave);
      const uint32_t len = __shfl(ukl - sh, sl, kWave), dst = __shfl(ko + sh, sl, kWave);
      for (uint32_t o0 = 16u * l; o0 < len; o0 += 64u * kWave) {
        uint4 y[4];
#pragma unroll
        for (int k = 0; k < 4; k++) {
          const uint32_t o = o0 + 16u * kWave * k, q = o < len - 16 ? o : len - 16;
          y[k] = V.ld16(src + int32_t(o < len ? q : 0u));
        }
#pragma unroll
        for (int k = 0; k < 4; k++) {
          const uint32_t o = o0 + 16u * kWave * k, q = o < len - 16 ? o : len - 16;
          if (o < len) st_out((gptr<u32x4_ug>)(kbytes + dst + q), u32x4_ug{y[k].x, y[k].y, y[k].z, y[k].w});
        }
      }
    }
  }
}

// Value bytes of a block, 8 lanes per KV: lane c of a group copies its
// value's 16-B chunks c, c + 8, ... from the block in global memory to the
// output with plain (unaligned) 16-B loads and stores.  A value's last chunk
// is the one that ENDS at the value's end, overlapping the chunk before it, so
// every store writes bytes of its own value only and no store is partial.
// kVG KVs per group per step, all their first chunks loaded before any store:
// the loads are L2 / MALL round trips, and a step costs about one of them.
// Values shorter than 16 B go byte by byte; values longer than kWaveVal are
// copied by the whole wave, four 16-B chunks per lane in flight.
#ifndef PBL_POOL_VG
#define PBL_POOL_VG 8
#endif
constexpr int kVG = PBL_POOL_VG;
#ifndef PBL_POOL_WAVEVAL
#define PBL_POOL_WAVEVAL 1024
#endif
constexpr uint32_t kWaveVal = PBL_POOL_WAVEVAL;
#ifndef PBL_POOL_MEDU
#define PBL_POOL_MEDU 4
#endif
constexpr int kMedU = PBL_POOL_MEDU;  // chunks per lane in flight for values of 129 B .. kWaveVal
// One step of the value copy: kVG KVs per 8-lane group, j = j0 + 8 u + lane / 8.
// Only the loaded chunks are held between a step's loads and its stores (the
// offsets are re-read from the slot).
struct VBatch {
  u32x4 x[kVG];
};
struct VSeg {
  uint32_t vo, vl, vs, q;
  bool has;
};
__device__ __forceinline__ VSeg val_seg(const uint32_t* vp, uint32_t nkv, uint32_t j) {
  const uint32_t c = uint32_t(lane_id()) & 7u;
  const uint32_t a = j < nkv ? vp[j] : 0u, z = j < nkv ? vp[j + 1] : 0u;
  VSeg S;
  S.vo = a & 0xffffu;
  S.vl = (z & 0xffffu) - S.vo;
  S.vs = a >> 16;
  S.has = S.vl >= 16 && S.vl <= kWaveVal && 16 * c < S.vl;
  S.q = S.has ? (16 * c < S.vl - 16 ? 16 * c : S.vl - 16) : 0u;
  return S;
}

// The step's first chunks from the block (every lane loads, from the block's
// first 16-B aligned granule when it has no chunk: no conditionally defined
// registers, and no read past the block's last granule however short it is).
__device__ __forceinline__ void val_load(const uint32_t* vp, gptr<const uint8_t> g, uint32_t nkv, uint32_t j0, VBatch& B) {
  const uint32_t jl = j0 + (uint32_t(lane_id()) >> 3);
  const uint32_t ph = uint32_t(reinterpret_cast<uintptr_t>(g) & 15u);
#pragma unroll
  for (int u = 0; u < kVG; u++) {
    const VSeg S = val_seg(vp, nkv, jl + 8 * u);
    B.x[u] = *(gptr<const u32x4_ug>)(g + (S.has ? int32_t(S.vs + S.q) : -int32_t(ph)));
  }
}

__device__ __forceinline__ void val_store(const uint32_t* vp, uint32_t nkv, uint32_t j0, const VBatch& B,
                                          gptr<const uint8_t> g, gptr<uint8_t> vbytes) {
  const uint32_t c = uint32_t(lane_id()) & 7u, jl = j0 + (uint32_t(lane_id()) >> 3);
#pragma unroll
  for (int u = 0; u < kVG; u++) {
    const VSeg S = val_seg(vp, nkv, jl + 8 * u);
    if (S.has) st_out((gptr<u32x4_ug>)(vbytes + S.vo + S.q), u32x4_ug(B.x[u]));
    if (S.vl > 128 && S.vl <= kWaveVal) {
      // the value's further chunks, kMedU per lane in flight
      for (uint32_t o0 = 16 * c + 128; o0 < S.vl; o0 += 128 * kMedU) {
        u32x4 y[kMedU];
#pragma unroll
        for (int k = 0; k < kMedU; k++) {
          const uint32_t o = o0 + 128 * k, q = o < S.vl - 16 ? o : S.vl - 16;
          if (o < S.vl) y[k] = *(gptr<const u32x4_ug>)(g + S.vs + q);
        }
#pragma unroll
        for (int k = 0; k < kMedU; k++) {
          const uint32_t o = o0 + 128 * k, q = o < S.vl - 16 ? o : S.vl - 16;
          if (o < S.vl) st_out((gptr<u32x4_ug>)(vbytes + S.vo + q), u32x4_ug(y[k]));
        }
      }
    } else if (S.vl < 16) {
      for (uint32_t o = c; o < S.vl; o += 8) vbytes[S.vo + o] = g[S.vs + o];
    }
  }
}

// Steps are software-pipelined: step i + 1's loads are issued before step i's
// stores (vmcnt retires loads and stores in issue order, so a load issued
// after a store would wait for that store's acknowledgement too).  B: step 0,
// loaded by the caller.
__device__ __forceinline__ void copy_long_values(const uint32_t* vp, gptr<const uint8_t> g, uint32_t nkv,
                                                 gptr<uint8_t> vbytes);

// PBL_POOL_VDEPTH 2: two steps in flight (B: step 0, B1: step 1, both loaded
// by the caller), each step's loads issued two steps ahead of its stores.
#ifndef PBL_POOL_VDEPTH
#define PBL_POOL_VDEPTH 1
#endif
constexpr int kVDepth = PBL_POOL_VDEPTH;
// PBL_POOL_UNI: the keys and the values of 64 KVs per step (one key batch, one
// value step of 8 KVs per 8-lane group)
#ifndef PBL_POOL_UNI
#define PBL_POOL_UNI 1
#endif
constexpr bool kUni = PBL_POOL_UNI != 0;
static_assert(!kUni || (kKU == 1 && 8 * kVG == kWave), "unified steps: one 64-KV key batch = one value step");
static_assert(kVDepth == 1 || kVDepth == 2, "value steps in flight: 1 or 2");
__device__ __forceinline__ void copy_values_grp(const uint32_t* vp, gptr<const uint8_t> g, uint32_t nkv,
                                                gptr<uint8_t> vbytes, VBatch& B, VBatch& B1) {
  const int l = lane_id();
  constexpr uint32_t S = 8 * kVG;  // KVs per step
  if (kVDepth == 1) {
    for (uint32_t j0 = 0; j0 < nkv; j0 += S) {
      if (j0 + S < nkv) {
        VBatch N;
        val_load(vp, g, nkv, j0 + S, N);
        val_store(vp, nkv, j0, B, g, vbytes);
        B = N;
      } else {
        val_store(vp, nkv, j0, B, g, vbytes);
      }
    }
  } else {
    for (uint32_t j0 = 0; j0 < nkv; j0 += 2 * S) {
      VBatch N;
      if (j0 + 2 * S < nkv) val_load(vp, g, nkv, j0 + 2 * S, N);
      val_store(vp, nkv, j0, B, g, vbytes);
      if (j0 + S >= nkv) break;
      VBatch N1;
      if (j0 + 3 * S < nkv) val_load(vp, g, nkv, j0 + 3 * S, N1);
      val_store(vp, nkv, j0 + S, B1, g, vbytes);
      B = N;
      B1 = N1;
    }
  }
  copy_long_values(vp, g, nkv, vbytes);
}

// Values longer than kWaveVal: the whole wave, kLongU 16-B chunks per lane in
// flight.
#ifndef PBL_POOL_LONGU
#define PBL_POOL_LONGU 8  // config 5 RI 16: 889 / 905 / 874 GiB/s at 4 / 8 / 16
#endif
constexpr int kLongU = PBL_POOL_LONGU;
__device__ __forceinline__ void copy_long_values(const uint32_t* vp, gptr<const uint8_t> g, uint32_t nkv,
                                                 gptr<uint8_t> vbytes) {
  const int l = lane_id();
  for (uint32_t j0 = 0; j0 < nkv; j0 += kWave) {
    const uint32_t j = j0 + uint32_t(l);
    const uint32_t a = j < nkv ? vp[j] : 0u, z = j < nkv ? vp[j + 1] : 0u;
    const uint32_t len = (z & 0xffffu) - (a & 0xffffu);
    for (uint64_t lm = __ballot(j < nkv && len > kWaveVal); lm; lm &= lm - 1) {
      const int sl = __builtin_ctzll(lm);
      const uint32_t ls = __shfl(a >> 16, sl, kWave), ll = __shfl(len, sl, kWave), lo = __shfl(a & 0xffffu, sl, kWave);
      for (uint32_t o0 = 16u * l; o0 < ll; o0 += 16u * kLongU * kWave) {
        u32x4 y[kLongU];
#pragma unroll
        for (int k = 0; k < kLongU; k++) {
          const uint32_t o = o0 + 16u * kWave * k, q = o < ll - 16 ? o : ll - 16;
          y[k] = *(gptr<const u32x4_ug>)(g + ls + (o < ll ? q : 0u));
        }
#pragma unroll
        for (int k = 0; k < kLongU; k++) {
          const uint32_t o = o0 + 16u * kWave * k, q = o < ll - 16 ? o : ll - 16;
          if (o < ll) st_out((gptr<u32x4_ug>)(vbytes + lo + q), u32x4_ug(y[k]));
        }
      }
    }
  }
}

// Take a free stage (lane 0 spins on the workgroup's mask); returns its index.
template <bool kHide>
__device__ __forceinline__ uint32_t acquire(PoolLds<kHide>& L) {
  uint32_t s = 0;
  if (lane_id() == 0) {
    for (;;) {
      const uint32_t m = __hip_atomic_load(&L.free_mask, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      if (m) {
        const uint32_t c = uint32_t(__builtin_ctz(m));
        const uint32_t old =
            __hip_atomic_fetch_and(&L.free_mask, ~(1u << c), __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
        if (old & (1u << c)) {
          s = c;
          break;
        }
      } else {
        __builtin_amdgcn_s_sleep(PBL_POOL_SLEEP);
      }
    }
  }
  // the stage holder's work (staging, walk, metadata) gates every wave
  // waiting for a stage: it wins issue arbitration against the emitting waves
  if (PBL_POOL_PRIO) __builtin_amdgcn_s_setprio(PBL_POOL_PRIO);
  return __builtin_amdgcn_readfirstlane(__shfl(s, 0, kWave));
}

// Return stage s to the pool once every LDS read of it has completed.
template <bool kHide>
__device__ __forceinline__ void release(PoolLds<kHide>& L, uint32_t s) {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  wave_sync();
  if (lane_id() == 0) __hip_atomic_fetch_or(&L.free_mask, 1u << s, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
  if (PBL_POOL_PRIO) __builtin_amdgcn_s_setprio(0);
}

// The block [boff, boff + blen) into stage S by LDS-DMA (granule g of the 16-B
// aligned range at x[1 + g]); the caller waits vmcnt(0) before reading it.
__device__ __forceinline__ void stage_dma(Stage& S, const uint8_t* blocks, uint64_t boff, uint32_t blen) {
  const int l = lane_id();
  const uint64_t a0 = boff & ~uint64_t(15), a1 = (boff + blen + 15) & ~uint64_t(15);
  const uint32_t n16 = uint32_t((a1 - a0) >> 4);
  const gptr<const uint8_t> base = to_glb(blocks + a0);
  for (uint32_t g0 = 0; g0 < n16; g0 += kWave) {
    if (g0 + l < n16)
      __builtin_amdgcn_global_load_lds((gptr<const void>)(base + 16ull * (g0 + l)),
                                       (lptr<void>)to_lds_ptr(reinterpret_cast<void*>(&S.x[1 + g0])), 16, 0, 0);
  }
}

// General path for one block (wave-serial Iter.Next) on the staged block, the
// slot as its key buffer; a key that outgrows it re-runs from global memory
// with the whole stage as the key buffer.  Publishes and resolves its own
// look-back and writes every output.  Out of line: rare and large.
__device__ __noinline__ void block_slow(Stage& S, uint8_t* keybuf, uint32_t keycap, const Args A, uint32_t b,
                                        uint64_t boff, uint32_t blen) {
  const int l = lane_id();
  const uint32_t nb = A.in.n_blocks, flags = A.in.flags;
  const pbl_decode_out& O = A.out;
  uint64_t* lb_state = reinterpret_cast<uint64_t*>(reinterpret_cast<uint8_t*>(O.workspace) + kWsHeader);
  SlowState ss;
  uint64_t dummy[kNumComp] = {0, 0, 0, 0}, excl[kNumComp];
  const uint8_t* src = reinterpret_cast<const uint8_t*>(S.x) + kPad + (boff & 15);
  bool from_lds = true;
  slow_walk(src, true, blen, flags, A.in.synthetic_seq_num, keybuf, keycap, kPassCount, O, b, dummy, &ss);
  if (ss.status == PBL_UNSUPPORTED) {
    from_lds = false;
    src = A.in.blocks + boff;
    keybuf = reinterpret_cast<uint8_t*>(S.x);
    keycap = uint32_t(kLdsBlkBytes);
    slow_walk(src, false, blen, flags, A.in.synthetic_seq_num, keybuf, keycap, kPassCount, O, b, dummy, &ss);
  }
  const bool okk = ss.status == PBL_OK;
  const uint64_t agg[kNumComp] = {okk ? ss.nkv : 0, okk ? ss.kb : 0, okk ? ss.vb : 0, okk ? ss.nr : 0};
  lookback(lb_state, nb, b, agg, excl, &O.totals->status_mask);
  uint32_t st2 = ss.status;
  if (okk && overflows(O, excl, agg)) st2 = PBL_OVERFLOW;
  if (st2 == PBL_OK) slow_walk(src, from_lds, blen, flags, A.in.synthetic_seq_num, keybuf, keycap, kPassAll, O, b, excl, &ss);
  else if (l == 0 && O.key_off && excl[0] + b < O.kv_cap + nb) {
    to_glb(O.key_off)[excl[0] + b] = 0;
    to_glb(O.val_off)[excl[0] + b] = 0;
  }
  if (l == 0) write_block_meta(O, b, nb, st2, excl, agg, true);
}

// A block past the stage: big_block_sizes_kernel walked it, published its
// aggregate and left {status, counts} in its block-metadata slots.  Once its
// bases resolve, the wave walks it from global memory and writes its outputs,
// its slot as the key buffer; a key past the slot lists the block for
// big_block_values_kernel (after this launch).  (Config 5: 2195 big blocks,
// one 48 KB value each; the separate values pass took 87 us.)  Out of line.
__device__ __noinline__ void block_big(const Args A, uint32_t b, uint64_t boff, uint32_t blen, uint8_t* keybuf,
                                       uint32_t keycap) {
  const int l = lane_id();
  const uint32_t nb = A.in.n_blocks;
  const pbl_decode_out& O = A.out;
  uint64_t* lb_state = reinterpret_cast<uint64_t*>(reinterpret_cast<uint8_t*>(O.workspace) + kWsHeader);
  const uint32_t st0 = to_glb(O.blk_status)[b];
  const bool okk = st0 == PBL_OK;
  const uint64_t agg[kNumComp] = {okk ? to_glb(O.blk_kv_base)[b] : 0, okk ? to_glb(O.blk_key_base)[b] : 0,
                                  okk ? to_glb(O.blk_val_base)[b] : 0,
                                  okk ? uint64_t(SlowGlb{to_glb(A.in.blocks + boff), blen}.le32(blen - 4)) : 0};
  uint64_t excl[kNumComp];
  lb_resolve(lb_state, nb, b, agg, excl, &O.totals->status_mask);
  uint32_t st2 = st0;
  if (okk && overflows(O, excl, agg)) st2 = PBL_OVERFLOW;
  if (l == 0) {
    if (st2 != PBL_OK && O.key_off && excl[0] + b < O.kv_cap + nb) {
      to_glb(O.key_off)[excl[0] + b] = 0;
      to_glb(O.val_off)[excl[0] + b] = 0;
    }
    write_block_meta(O, b, nb, st2, excl, agg, true);
  }
  if (st2 == PBL_OK) {
    SlowState ss;
    slow_walk_t<SlowGlb, PBL_BIG_U>(SlowGlb{to_glb(A.in.blocks + boff), blen}, blen, A.in.flags,
                                    A.in.synthetic_seq_num, to_lds_ptr(keybuf), keycap, kPassAll, O, b, excl, &ss);
    if (ss.status == PBL_UNSUPPORTED && l == 0) {  // a key past the slot: the values pass rewrites the block
      uint32_t* hdr = reinterpret_cast<uint32_t*>(O.workspace);
      uint32_t* pend = reinterpret_cast<uint32_t*>(reinterpret_cast<uint8_t*>(O.workspace) + ws_pend_offset(nb));
      to_glb(pend)[g_atomic_add(hdr + rowc::kWsBigPend, 1u)] = b;
    } else if (ss.status != PBL_OK && l == 0) {
      // the same walk as the sizes pass over the same bytes cannot disagree
      // with it; if it ever did, the block reports the walk's status
      to_glb(O.blk_status)[b] = ss.status;
      g_atomic_or(&O.totals->status_mask, 1u << ss.status);
      g_atomic_add(&O.totals->n_bad_blocks, 1u);
    }
  }
}

// A block between its walk and its emit: what the emit needs besides the slot.
struct Pend {
  uint64_t boff;
  uint32_t b, status, nkv, tkb, tvb, nres, roff, blen;
  bool live;  // the emit (look-back, outputs) is still to do
};

// Stage, walk and describe block b (stage s held on entry, released before
// return).  The block's aggregate is always published before return, so every
// later ticket can resolve past it while this wave goes on.  Blocks off the
// fast path are finished here (live = false).
template <bool kHide>
__device__ __forceinline__ Pend block_front(PoolLds<kHide>& L, uint32_t s, uint32_t b, uint64_t boff, uint32_t blen,
                                            Slot<kHide>& W, const Args& A) {
  Stage& S = L.st[s];
  const int l = lane_id();
  const uint32_t nb = A.in.n_blocks, flags = A.in.flags;
  const bool vprefix = (flags & PBL_ROW_VALUE_PREFIX) && !(flags & PBL_ROW_RAW_KEYS);
  uint64_t* lb_state = reinterpret_cast<uint64_t*>(reinterpret_cast<uint8_t*>(A.out.workspace) + kWsHeader);
  constexpr uint32_t kKv = uint32_t(Slot<kHide>::kKv);
  Pend P;
  P.b = b;
  P.boff = boff;
  P.blen = blen;
  P.live = false;
  P.nkv = P.tkb = P.tvb = P.nres = P.roff = 0;
  P.status = PBL_OK;

  if (blen > kMaxFastLen) {
    release(L, s);
    block_big(A, b, boff, blen, reinterpret_cast<uint8_t*>(&W), uint32_t(sizeof(W)));
    return P;
  }
  PSTAMP(A, b, 1, l == 0);
  stage_dma(S, A.in.blocks, boff, blen);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  wave_sync();
  PSTAMP(A, b, 2, l == 0);
  const View V = lds_view(S.x, uint32_t(kPad + (boff & 15)));
  uint32_t roff, nres;
  uint32_t status = rowc::init_checks(LdsRd{V}, blen, flags, &roff, &nres);
  bool slow = status == PBL_OK && nres > kKv;
  uint32_t nkv = 0, tkb = 0, tvb = 0;
  bool published = false;
  if (status == PBL_OK && !slow && roff > 0) {
    // lane l owns runs [r0, r1): contiguous, so a lane scan orders them
    const uint32_t R = (nres + kWave - 1) / kWave;
    const uint32_t r0 = min(uint32_t(l) * R, nres), r1 = min(r0 + R, nres);
    PAcc acc{0, 0, 0, 0};
    bool ok = true, bad = false, vbad = false, over = false;
    PRun RB;
    RB.n = 0;
    RB.pos = RB.e0 = RB.prev_kl = RB.prev_kind = RB.rw = 0;
    const bool single = R == 1;
    if (single) {
      if (r0 < nres) run_walk<kHide>(V, r0, nres, roff, flags, vprefix, RB, acc, ok, bad, vbad, over);
      // a run longer than kRunBuf keeps its parked head and counts only its tail
      if (over && ok)
        count_span<kHide>(V, RB.pos, RB.e0, RB.n, RB.prev_kl, RB.prev_kind, flags, vprefix, acc, ok, bad, vbad);
    } else {
      for (uint32_t r = r0; r < r1 && ok; r++) {
        uint32_t rw, e0;
        if (!run_bounds(V, r, nres, roff, &rw, &e0)) ok = false;
        else count_span<kHide>(V, rw & kRestartMask, e0, 0, 0, 0, flags, vprefix, acc, ok, bad, vbad);
      }
    }
    const uint32_t ic = dpp_incl_scan(acc.cnt), ik = dpp_incl_scan(acc.kb), iv = dpp_incl_scan(acc.vb);
    const uint32_t ie = kHide ? dpp_incl_scan(acc.ne) : ic;
    nkv = last_lane(ic);
    tkb = last_lane(ik);
    tvb = last_lane(iv);
    const uint32_t nent = kHide ? last_lane(ie) : nkv;
    if (__ballot(bad)) status = PBL_CORRUPT_BOUNDS;
    else if (__ballot(!ok) || nent > kKv) slow = true;
    else if (__ballot(vbad)) status = PBL_CORRUPT_BOUNDS;  // Go: i.val[0] on an empty SET value
    if (status == PBL_OK && !slow) {
      // the sizes are final: publish, then write the metadata
      const uint64_t agg[kNumComp] = {nkv, tkb, tvb, nres};
      lb_publish(lb_state, nb, b, agg);
      published = true;
      PSTAMP(A, b, 3, l == 0);
      MState M{ie - (kHide ? acc.ne : acc.cnt), ic - acc.cnt, iv - acc.vb, 0, 0, 0};
      if (single) {
        if (r0 < nres) {
          park_meta<kHide>(W, V, RB, flags, M);
          if (over) span_meta<kHide>(W, V, RB.pos, RB.e0, RB.rw, RB.n, RB.prev_kl, RB.prev_kind, flags, vprefix, M);
        }
      } else {
        for (uint32_t r = r0; r < r1; r++) {
          uint32_t rw, e0;
          run_bounds(V, r, nres, roff, &rw, &e0);
          M.prev_sh = M.pp = M.ppsh = 0;
          span_meta<kHide>(W, V, rw & kRestartMask, e0, rw, 0, 0, 0, flags, vprefix, M);
        }
      }
      if (l < 5) W.vp[nkv + l] = tvb;
      PSTAMP(A, b, 4, l == 0);
    }
  }
  if (status == PBL_OK && slow) {
    block_slow(S, reinterpret_cast<uint8_t*>(W.m0), uint32_t(sizeof(W.m0)), A, b, boff, blen);
    release(L, s);
    return P;
  }
  release(L, s);
  if (!published) {  // a failed or empty block: its (zero) aggregate
    const bool okb = status == PBL_OK;
    const uint64_t agg[kNumComp] = {okb ? nkv : 0, okb ? tkb : 0, okb ? tvb : 0, okb ? nres : 0};
    lb_publish(lb_state, nb, b, agg);
    if (l < 5) W.vp[l] = 0;  // (an empty block's lone N+1 offsets)
  }
  P.status = status;
  P.nkv = status == PBL_OK ? nkv : 0;
  P.tkb = status == PBL_OK ? tkb : 0;
  P.tvb = status == PBL_OK ? tvb : 0;
  P.nres = status == PBL_OK ? nres : 0;
  P.roff = roff;
  P.live = true;
  return P;
}

// Resolve block P's look-back and write its outputs from slot W.
template <bool kHide>
__device__ __forceinline__ void block_emit(const Pend& P, const Slot<kHide>& W, const Args& A) {
  const int l = lane_id();
  const uint32_t nb = A.in.n_blocks, flags = A.in.flags, b = P.b;
  const pbl_decode_out& O = A.out;
  uint64_t* lb_state = reinterpret_cast<uint64_t*>(reinterpret_cast<uint8_t*>(O.workspace) + kWsHeader);
  const uint8_t* gblk = A.in.blocks + P.boff;
  const gptr<const uint8_t> gb = to_glb(gblk);
  const GSrc KS{gb, P.blen, uint32_t(((uint64_t(gblk) + P.blen + 15) & ~uint64_t(15)) - uint64_t(gblk))};
  const bool raw = (flags & PBL_ROW_RAW_KEYS) != 0;
  const uint32_t nkv = P.nkv, nres = P.nres;
  // the look-back windows, the first key batch, the first value step and the
  // first restart words: all in one round trip
  LbWindows<kLbWin> G;
  if (b > 0) G.issue(LbPtrs(lb_state, nb), int64_t(b) - 1);
  KBatch K;
  VBatch VB, VB1;
  uint32_t rs0 = 0;
  const bool ok0 = P.status == PBL_OK;
  if (ok0) {
    key_load<kHide, GSrc>(W, KS, raw, 0, nkv, K);
    val_load(W.vp, gb, nkv, 0, VB);
    if (kVDepth == 2) val_load(W.vp, gb, nkv, 8 * kVG, VB1);
    if (O.restarts && uint32_t(l) < nres) rs0 = KS.le32(P.roff + 4 * l);
  }
  const uint64_t agg[kNumComp] = {nkv, P.tkb, P.tvb, nres};
  uint64_t excl[kNumComp];
  lb_finish(lb_state, nb, b, agg, excl, &O.totals->status_mask, G);
  PSTAMP(A, b, 5, l == 0);
  uint32_t status = P.status;
  if (ok0 && overflows(O, excl, agg)) status = PBL_OVERFLOW;
  if (l == 0) {
    if (status != PBL_OK && O.key_off && excl[0] + b < O.kv_cap + nb) {
      to_glb(O.key_off)[excl[0] + b] = 0;
      to_glb(O.val_off)[excl[0] + b] = 0;
    }
    write_block_meta(O, b, nb, status, excl, agg, false);
  }
  if (status != PBL_OK) return;

  // ---- keys and per-KV arrays: lane per KV ------------------------------------
  const uint64_t kvb = excl[0], kbb = excl[1], vbb = excl[2], rbb = excl[3];
  if (O.restarts && uint32_t(l) < nres) to_glb(O.restarts)[rbb + l] = rs0;
  uint32_t kcar = 0;
  const gptr<uint8_t> vbytes = to_glb(O.val_bytes) + vbb;
  if (kUni) {
    // keys and values of the same 64 KVs in one step: a line of the block is
    // fetched once for both
    if (kVDepth == 1) {
      for (uint32_t j0 = 0; j0 <= nkv; j0 += kWave) {
        KBatch KN;
        VBatch VN;
        const bool more = j0 + kWave <= nkv;
        if (more) {
          key_load<kHide, GSrc>(W, KS, raw, j0 + kWave, nkv, KN);
          val_load(W.vp, gb, nkv, j0 + kWave, VN);
        }
        key_store<kHide, GSrc>(W, KS, A, b, j0, nkv, kvb, kbb, K, kcar);
        val_store(W.vp, nkv, j0, VB, gb, vbytes);
        K = KN;
        VB = VN;
      }
    } else {
      // the values two steps ahead, the keys one
      for (uint32_t j0 = 0; j0 <= nkv; j0 += kWave) {
        KBatch KN;
        VBatch VN;
        if (j0 + kWave <= nkv) key_load<kHide, GSrc>(W, KS, raw, j0 + kWave, nkv, KN);
        if (j0 + 2 * kWave < nkv) val_load(W.vp, gb, nkv, j0 + 2 * kWave, VN);
        key_store<kHide, GSrc>(W, KS, A, b, j0, nkv, kvb, kbb, K, kcar);
        val_store(W.vp, nkv, j0, VB, gb, vbytes);
        K = KN;
        VB = VB1;
        VB1 = VN;
      }
    }
    if (O.restarts)
      for (uint32_t r = kWave + l; r < nres; r += kWave) to_glb(O.restarts)[rbb + r] = KS.le32(P.roff + 4 * r);
    copy_long_values(W.vp, gb, nkv, vbytes);
    PSTAMP(A, b, 6, l == 0);
    PSTAMP(A, b, 7, l == 0);
    return;
  }
  key_store<kHide, GSrc>(W, KS, A, b, 0, nkv, kvb, kbb, K, kcar);
  for (uint32_t j0 = kWave * kKU; j0 <= nkv; j0 += kWave * kKU) {
    KBatch N;
    key_load<kHide, GSrc>(W, KS, raw, j0, nkv, N);
    key_store<kHide, GSrc>(W, KS, A, b, j0, nkv, kvb, kbb, N, kcar);
  }
  if (O.restarts)
    for (uint32_t r = kWave + l; r < nres; r += kWave) to_glb(O.restarts)[rbb + r] = KS.le32(P.roff + 4 * r);
  PSTAMP(A, b, 6, l == 0);

  // ---- values, global -> global --------------------------------------------
  if (P.tvb) copy_values_grp(W.vp, gb, nkv, vbytes, VB, VB1);
  PSTAMP(A, b, 7, l == 0);
}

// The persistent kernel: one workgroup of kNW waves per CU, each wave a loop
// of (acquire a stage, take a ticket, stage / walk / describe the block into
// one slot, then emit the block before it from the other slot).
// Deadlock-free for any residency: a wave takes a ticket only while holding a
// stage, publishes the block's aggregate before it lets the stage go, and
// waits (in the look-back) only on smaller tickets, each held by a wave that
// holds a stage or has published.
// `ids` (mixed batches): the ascending ids of the batch's row blocks, their
// count at workspace header word kWsRowCount; the colblk blocks' aggregates are
// published before this launch (mixed_col_size_kernel), so the look-back walks
// through them and still waits only on smaller tickets.  Null: every block.
template <bool kHide>
__global__ void __launch_bounds__(kTPBP, 1) rowblk_pool_kernel(Args A, const uint32_t* ids) {
  __shared__ PoolLds<kHide> L;
  if (threadIdx.x == 0) L.free_mask = (1u << kNS) - 1u;
  __syncthreads();
  Slot<kHide>& W = L.sl[wave_id()];
  const uint32_t nb = A.in.n_blocks;
  uint32_t* tick = reinterpret_cast<uint32_t*>(A.out.workspace);
  const uint32_t nt = ids ? __hip_atomic_load(to_glb(tick) + kWsRowCount, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                          : nb;
  for (;;) {
#ifdef PBL_STAMPS
    const uint64_t t_acq = __builtin_amdgcn_s_memtime();
#endif
    const uint32_t s = acquire(L);
    uint32_t t0 = 0;
    if (lane_id() == 0) t0 = g_atomic_add(tick, 1u);
    t0 = __builtin_amdgcn_readfirstlane(__shfl(t0, 0, kWave));
    if (t0 >= nt) {
      release(L, s);
      break;
    }
    if (ids) t0 = __builtin_amdgcn_readfirstlane(to_glb(ids)[t0]);
    PSTAMP(A, t0, 0, lane_id() == 0);
#ifdef PBL_STAMPS
    if (lane_id() == 0)
      reinterpret_cast<uint64_t*>(reinterpret_cast<uint8_t*>(A.out.workspace) + ws_bytes(nb))[uint64_t(t0) * 16 + 8] = t_acq;
#endif
    const uint64_t boff = to_glb(A.in.block_off)[t0];
    const uint32_t blen = to_glb(A.in.block_len)[t0];
    const Pend Q = block_front<kHide>(L, s, t0, boff, blen, W, A);
    if (Q.live) block_emit<kHide>(Q, W, A);
    wave_sync();  // (the slot is the next block's)
  }
}

}  // namespace pool
