// rowblk_pool.hip.h — the row-format decode with one wave per block, sixteen
// waves per CU, and a shared pool of LDS staging buffers.
//
// Every earlier single-pass form tied one 32 KiB LDS stage to every block in
// flight, so at most 4-5 blocks per CU were ever in flight, each a long chain
// of dependent LDS and HBM round trips.  Only the parse needs
// the staged bytes; the value bytes (80 % of the output) can be copied
// global->global from the block that was just read (L2 / MALL-hot).  So here:
//
//   acquire   a wave takes a free stage from the workgroup's pool (LDS mask),
//             THEN a ticket (the only order that keeps the look-back
//             deadlock-free: every ticket holder either holds a stage or is
//             past needing one)
//   stage     the block HBM -> LDS by LDS-DMA, one round trip
//   walk      lane per restart run (rowblk_writer.go:147-155 cuts the prefix
//             chain there): headers parked in registers, a DPP scan places the
//             runs, the block's aggregate is published and its look-back
//             windows requested at once
//   meta      per-KV metadata written from the registers (key source, shared
//             and key length, prefix parent, key output offset, entry offset,
//             flags: in the stage; value output / source offsets and the
//             value bucket table: in the wave's own small slot)
//   resolve   the exclusive prefix (normally one round trip, already in flight)
//   keys      lane per KV from the stage: offsets, trailer, flags, entry offset,
//             the user key merged from its prefix chain; restart words
//   release   the stage goes back to the pool
//   values    16-B output granules per lane, each gathered from the block in
//             GLOBAL memory (unaligned 16-B loads) through the slot's tables
//
// LDS per CU: 3 stages x 38 KB + 16 slots x 2.1 KB.  16 waves hold 16 blocks
// in flight; a stage is held only from the DMA to the end of the key emit.
//
// Blocks outside the fast-path limits take the wave-serial general walk
// (rowblk_general.hip.h) on the staged bytes; blocks past kMaxFastLen are sized
// and written by big_block_{sizes,values}_kernel around this launch.  Results
// are identical on every path.
//
// Semantics: cockroachdb/pebble sstable/rowblk/rowblk_iter.go — Init :241-276,
// readFirstKey :418-485, readEntry :333-416, decodeInternalKey :487-504, value
// prefix :1192-1199 (sstable/block/kv.go:14-41), decodeRestart :1092-1096.
#pragma once

namespace pool {

#ifndef PBL_POOL_WAVES
#define PBL_POOL_WAVES 8
#endif
#ifndef PBL_POOL_STAGES
#define PBL_POOL_STAGES 3
#endif
#ifndef PBL_POOL_EARLY
#define PBL_POOL_EARLY 1  // 1: the per-KV metadata in the wave's slot; the stage is released after the walk
#endif
#ifndef PBL_POOL_AHEAD
#define PBL_POOL_AHEAD 0  // 1 (with PBL_POOL_EARLY): a released stage is refilled at once with the next ticket's block
#endif
#ifndef PBL_POOL_SLEEP
#define PBL_POOL_SLEEP 8  // s_sleep units (64 cycles) between polls of the stage mask
#endif
#ifndef PBL_POOL_PARKPRIO
#define PBL_POOL_PARKPRIO 0
#endif
#ifndef PBL_POOL_PRIO
#define PBL_POOL_PRIO 2  // the stage holder's issue priority (values run at 0)
#endif
constexpr int kNW = PBL_POOL_WAVES;      // waves per workgroup (one workgroup per CU)
constexpr int kNS = PBL_POOL_STAGES;     // staging buffers per workgroup
constexpr int kTPBP = kNW * kWave;
constexpr int kPKv = PBL_POOL_EARLY ? 300 : 400;  // entries per block on the fast path
constexpr uint32_t kPKeyCap = 65535;     // user-key bytes per block on the fast path (u16 offsets)

// Per-KV metadata of one block.  m0[e] = key source offset | shared << 16 |
// internal key length << 32 | prefix parent << 48, for every entry e; the rest
// by visible index (entries minus hidden obsolete points).
struct Meta {
  uint64_t m0[kPKv];
  uint16_t kout[kPKv + 1];     // user-key output offsets (block relative)
  uint16_t eoff[kPKv];         // entry offsets (KVEncoding.Offset)
  uint16_t ent[kPKv];          // the entry of visible KV v (PBL_ROW_HIDE_OBSOLETE batches)
  uint8_t kvf[kPKv];           // PBL_KV_* (OBSOLETE is added at emit time)
};
// A stage: the block bytes (and, unless PBL_POOL_EARLY, the metadata the key
// emit reads from the stage).
struct Stage {
  uint4 x[kLdsBlkBytes / 16];  // the block, byte i at kPad + (boff & 15) + i
#if !PBL_POOL_EARLY
  Meta m;
#endif
};
// A wave's slot: what the emit needs after the stage is released.
struct Slot {
  uint32_t vp[kPKv + 5];       // value output offset | value source offset << 16;
                               // entries nkv..nkv+4 hold the value total
#if PBL_POOL_EARLY
  Meta m;
#endif
};
// Stage ring state (PBL_POOL_AHEAD): tk[s] = kTkFree, kTkHeld, or the ticket
// whose block has been (or is being) staged into s by the wave that released
// it ("parked"); rdy[s] = 1 once that wave saw its LDS-DMA land.
constexpr uint32_t kTkFree = 0xffffffffu, kTkHeld = 0xfffffffeu;
struct PoolLds {
  Stage st[kNS];
  Slot sl[kNW];
  uint32_t free_mask;          // bit s: stage s is free
  uint32_t tk[kNS], rdy[kNS], pblen[kNS];
  uint64_t pboff[kNS];
  uint32_t inflight;           // parks between their ticket and their tk[] store
};
static_assert(sizeof(PoolLds) <= 163840, "one pool workgroup per CU");

__device__ __forceinline__ uint32_t m_ksrc(uint64_t m) { return uint32_t(m) & 0xffffu; }
__device__ __forceinline__ uint32_t m_sh(uint64_t m) { return uint32_t(m >> 16) & 0xffffu; }
__device__ __forceinline__ uint32_t m_klen(uint64_t m) { return uint32_t(m >> 32) & 0xffffu; }
__device__ __forceinline__ uint32_t m_par(uint64_t m) { return uint32_t(m >> 48); }

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

// Bytes [0, n) of w (n <= 16) to p, any alignment: one 16-B store when whole,
// else the fewest 8/4/2/1-B stores (nothing past n: the next key belongs to
// another lane).
__device__ __forceinline__ void store_n(gptr<uint8_t> p, const uint4& w, uint32_t n) {
  if (n == 16) {
    *(gptr<u32x4_ug>)p = u32x4{w.x, w.y, w.z, w.w};
    return;
  }
  uint64_t lo = uint64_t(w.x) | uint64_t(w.y) << 32, hi = uint64_t(w.z) | uint64_t(w.w) << 32;
  uint32_t o = 0;
  if (n & 8) {
    *(gptr<u64_ug>)p = lo;
    lo = hi;
    o = 8;
  }
  if (n & 4) {
    *(gptr<u32_ug>)(p + o) = uint32_t(lo);
    lo >>= 32;
    o += 4;
  }
  if (n & 2) {
    *(gptr<u16_ug>)(p + o) = uint16_t(lo);
    lo >>= 16;
    o += 2;
  }
  if (n & 1) *(p + o) = uint8_t(lo);
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
constexpr int kRunBuf = 16;
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
    const bool hok = pipe::hdr2(V.ld8(pos), &sh, &un, &vl, &h);
    const uint32_t np = pos + h + un + vl;  // < 2^23: no overflow
    if (!hok || (k == 0 && sh != 0) || np > e0) { ok = false; return; }
    bad = bad || (k > 0 && sh > prev_kl);
    const uint32_t kl = sh + un;
    bool hidden, setv;
    if (!entry_class<kHide>(V, pos, h, sh, kl, k, prev_kl, prev_kind, flags, vprefix, hidden, setv)) {
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
      const bool hok = pipe::hdr2(V.ld8(pos), &sh, &un, &vl, &h);
      const uint32_t np = pos + h + un + vl;
      bool hidden = false, setv = false;
      if (!hok || (k == 0 && sh != 0) || np > e0) {
        ok = false;
        go = false;
      } else {
        bad = bad || (k > 0 && sh > prev_kl);
        const uint32_t kl = sh + un;
        if (!entry_class<kHide>(V, pos, h, sh, kl, uint32_t(k), prev_kl, prev_kind, flags, vprefix, hidden, setv)) {
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
// to the next: entry / visible index, key / value output offsets, the previous
// entry's shared length, its prefix parent and that parent's shared length.
struct MState {
  uint32_t e, v, kb, vb, prev_sh, pp, ppsh;
};

// Per-KV metadata of one entry (validated by the walk).  The prefix parent is
// the nearest earlier entry of the run with a smaller shared length (all-
// nearest-smaller-values over the parents, amortised O(1)).
template <bool kHide>
__device__ __forceinline__ void entry_meta(Meta& Mt, Slot& W, const View& V, uint32_t pos, bool hidden, uint32_t sh,
                                           uint32_t un, uint32_t h, uint32_t vl, bool setv, bool first, uint32_t rw,
                                           uint32_t flags, MState& M) {
  const uint32_t kl = sh + un;
  uint32_t par = M.e, parsh = 0;
  if (sh != 0) {
    uint32_t c = M.e - 1, csh = M.prev_sh;
    if (csh >= sh) { c = M.pp; csh = M.ppsh; }
    while (csh >= sh) {
      c = m_par(Mt.m0[c]);
      csh = m_sh(Mt.m0[c]);
    }
    par = c;
    parsh = csh;
  }
  Mt.m0[M.e] = uint64_t(pos + h) | uint64_t(sh) << 16 | uint64_t(kl) << 32 | uint64_t(par) << 48;
  if (!(kHide && hidden)) {
    uint32_t vs = pos + h + un, vlen = vl;
    uint8_t fl = 0;
    if (first) fl = uint8_t(PBL_KV_RESTART | ((rw >> 31) ? PBL_KV_RESTART_SAMEPFX : 0));
    if (!(flags & PBL_ROW_RAW_KEYS) && kl < 8) fl |= PBL_KV_INVALID_KEY;
    if (setv) {
      const uint32_t pre = V.byte(vs);
      if ((pre & 0xC0) == 0 || (flags & PBL_ROW_NO_VALUER)) { vs++; vlen--; }
      else if ((pre & 0xC0) == 0x80) fl |= PBL_KV_VALBLK_HANDLE;
      else fl |= PBL_KV_BLOB_HANDLE;
    }
    Mt.kout[M.v] = uint16_t(M.kb);
    Mt.eoff[M.v] = uint16_t(pos);
    Mt.kvf[M.v] = fl;
    if (kHide) Mt.ent[M.v] = uint16_t(M.e);
    W.vp[M.v] = M.vb | (vs << 16);
    M.kb += ukey_len(kl, flags);
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
__device__ __forceinline__ void park_meta(Meta& Mt, Slot& W, const View& V, const PRun& B, uint32_t flags, MState& M) {
#pragma unroll
  for (int k = 0; k < kRunBuf; k++) {
    if (uint32_t(k) < B.n)
      entry_meta<kHide>(Mt, W, V, B.ea[k] & 0x7fffu, (B.ea[k] >> 15) & 1u, (B.ea[k] >> 16) & 0x7fffu,
                        B.eb[k] & 0x3fffu, (B.eb[k] >> 14) & 7u, B.eb[k] >> 17, B.ea[k] >> 31, k == 0, B.rw, flags,
                        M);
  }
}

// Metadata of entries [pos, e0) of a run, re-read from the stage (k = entries
// of the run before pos; prev_kl / prev_kind: the last one's).
template <bool kHide>
__device__ __forceinline__ void span_meta(Meta& Mt, Slot& W, const View& V, uint32_t pos, uint32_t e0, uint32_t rw,
                                          uint32_t k, uint32_t prev_kl, uint32_t prev_kind, uint32_t flags,
                                          bool vprefix, MState& M) {
  while (pos < e0) {
    uint32_t sh, un, vl, h;
    pipe::hdr2(V.ld8(pos), &sh, &un, &vl, &h);
    const uint32_t kl = sh + un;
    bool hidden, setv;
    entry_class<kHide>(V, pos, h, sh, kl, k, prev_kl, prev_kind, flags, vprefix, hidden, setv);
    entry_meta<kHide>(Mt, W, V, pos, hidden, sh, un, h, vl, setv, k == 0, rw, flags, M);
    k++;
    prev_kl = kl;
    pos = pos + h + un + vl;
  }
}

// The block's bytes for the key emit: the stage (LDS) or the block in global
// memory (PBL_POOL_EARLY: the stage is gone by then).  ld16 windows may start
// up to 15 bytes before the block.
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
__device__ __forceinline__ uint32_t key_byte(const Meta& Mt, const Src& V, int j, uint32_t p) {
  uint64_t m = Mt.m0[j];
  while (p < m_sh(m)) m = Mt.m0[--j];
  return V.byte(m_ksrc(m) + p - m_sh(m));
}

template <class Src>
__device__ __forceinline__ uint64_t trailer_of(const Meta& Mt, const Src& V, int j, uint64_t m, uint8_t* fl,
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
    for (int i = 0; i < 8; i++) raw |= uint64_t(key_byte(Mt, V, j, kl - 8 + i)) << (8 * i);
  }
  if (raw & 64u) *fl |= PBL_KV_OBSOLETE;
  return raw & kTrailerObsoleteMask;
}

// Key bytes [c, c + n) of KV m (n <= 16) merged from the segments of its prefix
// chain: each a 16-B read that starts where the chunk's first byte would sit in
// that entry (at most 15 bytes before the block).
template <class Src>
__device__ __forceinline__ uint4 key_chunk(const Meta& Mt, const Src& V, uint64_t m, uint32_t c, uint32_t n) {
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
    m = Mt.m0[m_par(m)];
  }
  return w;
}

// Keys, offsets, trailers, flags and entry offsets of a block's visible KVs:
// lane per KV, the key merged from its prefix chain's segments.
template <bool kHide, class Src>
__device__ __forceinline__ void emit_keys(const Meta& Mt, const Slot& W, const Src& V, const Args& A, uint32_t b,
                                          uint32_t nkv, uint64_t kvb, uint64_t kbb) {
  const int l = lane_id();
  const uint32_t flags = A.in.flags;
  const pbl_decode_out& O = A.out;
  const gptr<uint8_t> kbytes = to_glb(O.key_bytes) + kbb;
  const bool raw = (flags & PBL_ROW_RAW_KEYS) != 0;
  for (uint32_t j = l; j <= nkv; j += kWave) {
    to_glb(O.key_off)[kvb + b + j] = Mt.kout[j];
    to_glb(O.val_off)[kvb + b + j] = W.vp[j] & 0xffffu;
    if (j < nkv) {
      const uint32_t e = kHide ? uint32_t(Mt.ent[j]) : j;
      const uint64_t m = Mt.m0[e];
      uint8_t fl = Mt.kvf[j];
      to_glb(O.trailer)[kvb + j] = with_seq(trailer_of(Mt, V, int(e), m, &fl, flags), A.in.synthetic_seq_num, flags);
      if (O.kv_flags) to_glb(O.kv_flags)[kvb + j] = fl;
      if (O.entry_off) to_glb(O.entry_off)[kvb + j] = Mt.eoff[j];
      const uint32_t ukl = raw ? m_klen(m) : (m_klen(m) >= 8 ? m_klen(m) - 8 : 0u);
      const uint32_t ko = Mt.kout[j];
      for (uint32_t c = 0; c < ukl; c += 16) {
        const uint32_t n = ukl - c < 16 ? ukl - c : 16u;
        store_n(kbytes + ko + c, key_chunk(Mt, V, m, c, n), n);
      }
    }
  }
}

// emit_keys for the block in GLOBAL memory (PBL_POOL_EARLY): the loads are
// L2 / MALL round trips, so kKU KVs per lane go through three phases together:
// their metadata from the slot, then every global load (the trailer's 8 bytes;
// the user key's segments: its own unshared bytes and, for a key that shares
// a prefix, its prefix parent's bytes), then the merges and stores.  The fast
// form covers keys of at most 16 bytes whose prefix chain ends at the parent
// (a restart-interval row block: the parent is the run's first key) with the
// trailer in the entry's own bytes; the rest take emit_keys' general form.
#ifndef PBL_POOL_KU
#define PBL_POOL_KU 3
#endif
constexpr int kKU = PBL_POOL_KU;
// One batch of the key emit: kKU KVs per lane, j = j0 + kWave * u + lane.
// Only what the loads produced (and the metadata words they were addressed
// by) is held between the loads and the stores; the rest is re-read from the
// slot at store time (cheaper than the registers across a look-back wait).
struct KBatch {
  uint64_t m[kKU], mp[kKU], tr[kKU];
  uint4 ka[kKU], kp[kKU];
};

__device__ __forceinline__ bool key_fast(uint64_t m, uint64_t mp, bool raw) {
  const uint32_t kl = m_klen(m), sh = m_sh(m), ukl = raw ? kl : (kl >= 8 ? kl - 8 : 0u);
  return ukl <= 16 && (sh == 0 || m_sh(mp) == 0) && (raw || kl < 8 || kl - 8 >= sh);
}

// The batch's metadata words from the slot, then every global load it needs.
template <bool kHide>
__device__ __forceinline__ void key_load(const Meta& Mt, const GSrc& V, bool raw, uint32_t j0, uint32_t nkv,
                                         KBatch& K) {
  const int l = lane_id();
#pragma unroll
  for (int u = 0; u < kKU; u++) {
    const uint32_t j = j0 + kWave * u + l;
    const uint32_t e = kHide ? (j < nkv ? uint32_t(Mt.ent[j]) : 0u) : j;
    K.m[u] = j < nkv ? Mt.m0[e] : 0ull;
    K.mp[u] = (j < nkv && m_sh(K.m[u]) != 0) ? Mt.m0[m_par(K.m[u])] : 0ull;
  }
#pragma unroll
  for (int u = 0; u < kKU; u++) {
    const uint32_t j = j0 + kWave * u + l;
    const uint64_t m = K.m[u];
    const uint32_t kl = m_klen(m), sh = m_sh(m), ukl = raw ? kl : (kl >= 8 ? kl - 8 : 0u);
    const bool fast = j < nkv && key_fast(m, K.mp[u], raw);
    K.tr[u] = 0;
    if (fast && !raw && kl >= 8) K.tr[u] = V.ld8(m_ksrc(m) + (kl - 8 - sh));
    if (fast && ukl) K.ka[u] = V.ld16(int32_t(m_ksrc(m)) - int32_t(sh));
    if (fast && ukl && sh) K.kp[u] = V.ld16(int32_t(m_ksrc(K.mp[u])));
  }
}

// The batch's merges and stores (the general form for KVs off the fast form).
template <bool kHide>
__device__ __forceinline__ void key_store(const Meta& Mt, const Slot& W, const GSrc& V, const Args& A, uint32_t b,
                                          uint32_t j0, uint32_t nkv, uint64_t kvb, uint64_t kbb, const KBatch& K) {
  const int l = lane_id();
  const uint32_t flags = A.in.flags;
  const pbl_decode_out& O = A.out;
  const gptr<uint8_t> kbytes = to_glb(O.key_bytes) + kbb;
  const bool raw = (flags & PBL_ROW_RAW_KEYS) != 0;
#pragma unroll
  for (int u = 0; u < kKU; u++) {
    const uint32_t j = j0 + kWave * u + l;
    if (j > nkv) continue;
    const uint32_t ko = Mt.kout[j];
    to_glb(O.key_off)[kvb + b + j] = ko;
    to_glb(O.val_off)[kvb + b + j] = W.vp[j] & 0xffffu;
    if (j == nkv) continue;
    const uint64_t m = K.m[u];
    const uint32_t kl = m_klen(m), sh = m_sh(m), ukl = raw ? kl : (kl >= 8 ? kl - 8 : 0u);
    uint64_t t;
    uint8_t f = Mt.kvf[j];
    if (!key_fast(m, K.mp[u], raw)) {
      const uint32_t e = kHide ? uint32_t(Mt.ent[j]) : j;
      t = trailer_of(Mt, V, int(e), m, &f, flags);
      for (uint32_t c = 0; c < ukl; c += 16) {
        const uint32_t n = ukl - c < 16 ? ukl - c : 16u;
        store_n(kbytes + ko + c, key_chunk(Mt, V, m, c, n), n);
      }
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
    to_glb(O.trailer)[kvb + j] = with_seq(t, A.in.synthetic_seq_num, flags);
    if (O.kv_flags) to_glb(O.kv_flags)[kvb + j] = f;
    if (O.entry_off) to_glb(O.entry_off)[kvb + j] = Mt.eoff[j];
  }
}

// emit_keys for the block in GLOBAL memory (PBL_POOL_EARLY): the loads are
// L2 / MALL round trips, so kKU KVs per lane go through three phases together:
// their metadata from the slot, then every global load (the trailer's 8 bytes;
// the user key's segments: its own unshared bytes and, for a key that shares
// a prefix, its prefix parent's bytes), then the merges and stores.  The fast
// form covers keys of at most 16 bytes whose prefix chain ends at the parent
// (a restart-interval row block: the parent is the run's first key) with the
// trailer in the entry's own bytes; the rest take emit_keys' general form.
// The first batch (K) was loaded by the caller, before its look-back wait.
template <bool kHide>
__device__ __forceinline__ void emit_keys_glb(const Meta& Mt, const Slot& W, const GSrc& V, const Args& A, uint32_t b,
                                              uint32_t nkv, uint64_t kvb, uint64_t kbb, const KBatch& K) {
  const bool raw = (A.in.flags & PBL_ROW_RAW_KEYS) != 0;
  key_store<kHide>(Mt, W, V, A, b, 0, nkv, kvb, kbb, K);
  for (uint32_t j0 = kWave * kKU; j0 <= nkv; j0 += kWave * kKU) {
    KBatch N;
    key_load<kHide>(Mt, V, raw, j0, nkv, N);
    key_store<kHide>(Mt, W, V, A, b, j0, nkv, kvb, kbb, N);
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
#define PBL_POOL_VG 4
#endif
constexpr int kVG = PBL_POOL_VG;
constexpr uint32_t kWaveVal = 1024;
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
__device__ __forceinline__ VSeg val_seg(const Slot& W, uint32_t nkv, uint32_t j) {
  const uint32_t c = uint32_t(lane_id()) & 7u;
  const uint32_t a = j < nkv ? W.vp[j] : 0u, z = j < nkv ? W.vp[j + 1] : 0u;
  VSeg S;
  S.vo = a & 0xffffu;
  S.vl = (z & 0xffffu) - S.vo;
  S.vs = a >> 16;
  S.has = S.vl >= 16 && S.vl <= kWaveVal && 16 * c < S.vl;
  S.q = S.has ? (16 * c < S.vl - 16 ? 16 * c : S.vl - 16) : 0u;
  return S;
}

// The step's first chunks from the block (every lane loads, from the block's
// first bytes when it has no chunk: no conditionally defined registers).
__device__ __forceinline__ void val_load(const Slot& W, gptr<const uint8_t> g, uint32_t nkv, uint32_t j0, VBatch& B) {
  const uint32_t jl = j0 + (uint32_t(lane_id()) >> 3);
#pragma unroll
  for (int u = 0; u < kVG; u++) {
    const VSeg S = val_seg(W, nkv, jl + 8 * u);
    B.x[u] = *(gptr<const u32x4_ug>)(g + (S.has ? S.vs + S.q : 0u));
  }
}

__device__ __forceinline__ void val_store(const Slot& W, uint32_t nkv, uint32_t j0, const VBatch& B,
                                          gptr<const uint8_t> g, gptr<uint8_t> vbytes) {
  const uint32_t c = uint32_t(lane_id()) & 7u, jl = j0 + (uint32_t(lane_id()) >> 3);
#pragma unroll
  for (int u = 0; u < kVG; u++) {
    const VSeg S = val_seg(W, nkv, jl + 8 * u);
    if (S.has) *(gptr<u32x4_ug>)(vbytes + S.vo + S.q) = B.x[u];
    if (S.vl > 128 && S.vl <= kWaveVal) {
      for (uint32_t o = 16 * c + 128; o < S.vl; o += 128) {
        const uint32_t q = o < S.vl - 16 ? o : S.vl - 16;
        *(gptr<u32x4_ug>)(vbytes + S.vo + q) = *(gptr<const u32x4_ug>)(g + S.vs + q);
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
__device__ __forceinline__ void copy_values_grp(const Slot& W, gptr<const uint8_t> g, uint32_t nkv,
                                                gptr<uint8_t> vbytes, VBatch& B) {
  const int l = lane_id();
  for (uint32_t j0 = 0; j0 < nkv; j0 += 8 * kVG) {
    if (j0 + 8 * kVG < nkv) {
      VBatch N;
      val_load(W, g, nkv, j0 + 8 * kVG, N);
      val_store(W, nkv, j0, B, g, vbytes);
      B = N;
    } else {
      val_store(W, nkv, j0, B, g, vbytes);
    }
  }
  // long values: the whole wave, four 16-B chunks per lane in flight
  for (uint32_t j0 = 0; j0 < nkv; j0 += kWave) {
    const uint32_t j = j0 + uint32_t(l);
    const uint32_t a = j < nkv ? W.vp[j] : 0u, z = j < nkv ? W.vp[j + 1] : 0u;
    const uint32_t len = (z & 0xffffu) - (a & 0xffffu);
    for (uint64_t lm = __ballot(j < nkv && len > kWaveVal); lm; lm &= lm - 1) {
      const int sl = __builtin_ctzll(lm);
      const uint32_t ls = __shfl(a >> 16, sl, kWave), ll = __shfl(len, sl, kWave), lo = __shfl(a & 0xffffu, sl, kWave);
      for (uint32_t o0 = 16u * l; o0 < ll; o0 += 64u * kWave) {
        u32x4 y[4];
#pragma unroll
        for (int k = 0; k < 4; k++) {
          const uint32_t o = o0 + 16u * kWave * k, q = o < ll - 16 ? o : ll - 16;
          y[k] = *(gptr<const u32x4_ug>)(g + ls + (o < ll ? q : 0u));
        }
#pragma unroll
        for (int k = 0; k < 4; k++) {
          const uint32_t o = o0 + 16u * kWave * k, q = o < ll - 16 ? o : ll - 16;
          if (o < ll) *(gptr<u32x4_ug>)(vbytes + lo + q) = y[k];
        }
      }
    }
  }
}

// Take a free stage (lane 0 spins on the workgroup's mask); returns its index.
__device__ __forceinline__ uint32_t acquire(PoolLds& L) {
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
  // the stage holder's work (staging, walk, metadata, look-back, keys) gates
  // every wave waiting for a stage: it wins issue arbitration against the
  // waves copying values
  if (PBL_POOL_PRIO) __builtin_amdgcn_s_setprio(PBL_POOL_PRIO);
  return __builtin_amdgcn_readfirstlane(__shfl(s, 0, kWave));
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

// ---- the stage ring (PBL_POOL_AHEAD) -------------------------------------------
// A wave done with a stage takes the next ticket and starts that block's
// LDS-DMA into the stage before it goes on with its own block ("parks" it);
// the next free wave picks the parked stage with the SMALLEST ticket and finds
// the block staged.  The DMA round trip thus overlaps the parker's look-back
// instead of sitting inside a stage hold.  Deadlock freedom: a wave picks
// only the smallest parked ticket, and only while no park is between its
// ticket and its tk[] store (inflight), so every ticket smaller than a picked
// one has been picked too; a wave's look-back waits only on smaller tickets,
// so the smallest unfinished ticket is always held by a wave that can go on,
// or parked while some wave is free to pick it.
struct Work {
  uint32_t s, t, blen;
  uint64_t boff;
  bool staged;
};

// Park stage s: the next ticket's block is staged into it (or the stage is
// freed when the tickets are exhausted).  Returns whether the caller must
// later mark it ready (after its own vmcnt(0)).
__device__ __forceinline__ bool park(PoolLds& L, uint32_t s, const Args& A) {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // every read of the stage has completed
  wave_sync();
  const uint32_t nb = A.in.n_blocks;
  uint32_t t = 0;
  if (lane_id() == 0) {
    __hip_atomic_fetch_add(&L.inflight, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    t = g_atomic_add(reinterpret_cast<uint32_t*>(A.out.workspace), 1u);
  }
  t = __builtin_amdgcn_readfirstlane(__shfl(t, 0, kWave));
  bool dma = false;
  if (t < nb) {
    const uint64_t boff = to_glb(A.in.block_off)[t];
    const uint32_t blen = to_glb(A.in.block_len)[t];
    dma = blen <= kMaxFastLen;
    if (dma) stage_dma(L.st[s], A.in.blocks, boff, blen);
    if (lane_id() == 0) {
      L.pboff[s] = boff;
      L.pblen[s] = blen;
      __hip_atomic_store(&L.rdy[s], dma ? 0u : 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      __hip_atomic_store(&L.tk[s], t, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
  } else if (lane_id() == 0) {
    __hip_atomic_store(&L.tk[s], kTkFree, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
  }
  if (lane_id() == 0) __hip_atomic_fetch_sub(&L.inflight, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
  // (PBL_POOL_PARKPRIO: a wave whose parked DMA gates the next picker keeps its
  // priority until it has marked the stage ready)
  if (PBL_POOL_PRIO && !(PBL_POOL_PARKPRIO && dma)) __builtin_amdgcn_s_setprio(0);
  return dma;
}

// Mark the stage this wave parked as staged (its DMA has landed: vmcnt(0)).
__device__ __forceinline__ void mark_ready(PoolLds& L, uint32_t s) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  wave_sync();
  if (lane_id() == 0) __hip_atomic_store(&L.rdy[s], 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
  if (PBL_POOL_PRIO && PBL_POOL_PARKPRIO) __builtin_amdgcn_s_setprio(0);
}

// The next block for this wave: the smallest parked ticket (waiting for its
// DMA to land), or a free stage and a fresh ticket.  w.t >= n_blocks: done.
__device__ __forceinline__ Work get_work(PoolLds& L, const Args& A) {
  const uint32_t nb = A.in.n_blocks;
  uint32_t r[5] = {0, 0, 0, 0, 0};  // s, t, blen, boff lo, boff hi | staged << 31
  if (lane_id() == 0) {
    for (;;) {
      if (__hip_atomic_load(&L.inflight, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) != 0) {
        __builtin_amdgcn_s_sleep(1);
        continue;
      }
      uint32_t best = kTkHeld, bs = kNS, fs = kNS;
      for (uint32_t q = 0; q < uint32_t(kNS); q++) {
        const uint32_t x = __hip_atomic_load(&L.tk[q], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
        if (x < best) { best = x; bs = q; }
        if (x == kTkFree) fs = q;
      }
      if (bs < uint32_t(kNS)) {
        uint32_t want = best;
        if (__hip_atomic_compare_exchange_strong(&L.tk[bs], &want, kTkHeld, __ATOMIC_ACQUIRE, __ATOMIC_RELAXED,
                                                 __HIP_MEMORY_SCOPE_WORKGROUP)) {
          while (__hip_atomic_load(&L.rdy[bs], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) == 0)
            __builtin_amdgcn_s_sleep(1);
          const uint64_t boff = L.pboff[bs];
          r[0] = bs; r[1] = best; r[2] = L.pblen[bs];
          r[3] = uint32_t(boff); r[4] = uint32_t(boff >> 32) | 0x80000000u;
          break;
        }
        continue;
      }
      if (fs < uint32_t(kNS)) {
        uint32_t want = kTkFree;
        if (__hip_atomic_compare_exchange_strong(&L.tk[fs], &want, kTkHeld, __ATOMIC_ACQUIRE, __ATOMIC_RELAXED,
                                                 __HIP_MEMORY_SCOPE_WORKGROUP)) {
          // a fresh ticket (counted in flight so no picker passes a smaller one)
          __hip_atomic_fetch_add(&L.inflight, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
          const uint32_t t = g_atomic_add(reinterpret_cast<uint32_t*>(A.out.workspace), 1u);
          __hip_atomic_fetch_sub(&L.inflight, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
          if (t >= nb) {
            __hip_atomic_store(&L.tk[fs], kTkFree, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
          } else {
            const uint64_t boff = to_glb(A.in.block_off)[t];
            r[2] = to_glb(A.in.block_len)[t];
            r[3] = uint32_t(boff);
            r[4] = uint32_t(boff >> 32);  // (not staged: the caller stages it)
          }
          r[0] = fs; r[1] = t < nb ? t : nb;
          break;
        }
        continue;
      }
      __builtin_amdgcn_s_sleep(PBL_POOL_SLEEP);
    }
  }
  Work w;
  w.s = __builtin_amdgcn_readfirstlane(__shfl(r[0], 0, kWave));
  w.t = __builtin_amdgcn_readfirstlane(__shfl(r[1], 0, kWave));
  w.blen = __builtin_amdgcn_readfirstlane(__shfl(r[2], 0, kWave));
  const uint32_t hi = __builtin_amdgcn_readfirstlane(__shfl(r[4], 0, kWave));
  w.boff = uint64_t(__builtin_amdgcn_readfirstlane(__shfl(r[3], 0, kWave))) | uint64_t(hi & 0x7fffffffu) << 32;
  w.staged = (hi >> 31) != 0;
  if (PBL_POOL_PRIO && w.t < nb) __builtin_amdgcn_s_setprio(PBL_POOL_PRIO);
  return w;
}

// Return stage s to the pool once every LDS read of it has completed.
__device__ __forceinline__ void release(PoolLds& L, uint32_t s) {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  wave_sync();
  if (lane_id() == 0) __hip_atomic_fetch_or(&L.free_mask, 1u << s, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
  if (PBL_POOL_PRIO) __builtin_amdgcn_s_setprio(0);
}

// General path for one block (wave-serial Iter.Next) on the staged block, the
// stage's metadata area as its key buffer; a key that outgrows it re-runs from
// global memory with the whole stage as the key buffer.  Resolves its own
// look-back and writes every output.  Out of line: rare and large.
__device__ __noinline__ void block_slow(Stage& S, Meta& Mt, const Args A, uint32_t b, uint64_t boff, uint32_t blen) {
  const int l = lane_id();
  const uint32_t nb = A.in.n_blocks, flags = A.in.flags;
  const pbl_decode_out& O = A.out;
  uint64_t* lb_state = reinterpret_cast<uint64_t*>(reinterpret_cast<uint8_t*>(O.workspace) + kWsHeader);
  SlowState ss;
  uint64_t dummy[kNumComp] = {0, 0, 0, 0}, excl[kNumComp];
  const uint8_t* src = reinterpret_cast<const uint8_t*>(S.x) + kPad + (boff & 15);
  bool from_lds = true;
  uint8_t* keybuf = reinterpret_cast<uint8_t*>(Mt.m0);
  uint32_t keycap = uint32_t(sizeof(Meta)) & ~15u;
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
// aggregate and left {status, counts} in its block-metadata slots;
// big_block_values_kernel writes its outputs after this launch.  Out of line.
__device__ __noinline__ void block_big(const Args A, uint32_t b, uint64_t boff, uint32_t blen) {
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
}

// One block on one wave, stage s held on entry and released before return.
template <bool kHide>
__device__ __forceinline__ void pool_block(PoolLds& L, const Work& wk, Slot& W, const Args& A) {
  const uint32_t s = wk.s, b = wk.t;
  Stage& S = L.st[s];
  // (PBL_POOL_AHEAD) the stage this wave parked, to be marked ready once its
  // DMA has landed; every exit below marks it
  uint32_t pend = kNS;
#if PBL_POOL_AHEAD
#define PBL_STAGE_DONE()                   \
  do {                                     \
    if (park(L, s, A)) pend = s;           \
  } while (0)
#define PBL_MARK_PENDING()                 \
  do {                                     \
    if (pend < uint32_t(kNS)) {            \
      mark_ready(L, pend);                 \
      pend = kNS;                          \
    }                                      \
  } while (0)
#else
#define PBL_STAGE_DONE() release(L, s)
#define PBL_MARK_PENDING() do {} while (0)
#endif
#if PBL_POOL_EARLY
  Meta& Mt = W.m;
#else
  Meta& Mt = S.m;
#endif
  const int l = lane_id();
  const uint32_t nb = A.in.n_blocks, flags = A.in.flags;
  const uint64_t boff = wk.boff;
  const uint32_t blen = wk.blen;
  const bool vprefix = (flags & PBL_ROW_VALUE_PREFIX) && !(flags & PBL_ROW_RAW_KEYS);
  uint8_t* ws = reinterpret_cast<uint8_t*>(A.out.workspace);
  uint64_t* lb_state = reinterpret_cast<uint64_t*>(ws + kWsHeader);
  const uint8_t* gblk = A.in.blocks + boff;
  const pbl_decode_out& O = A.out;

  if (blen > kMaxFastLen) {
    PBL_STAGE_DONE();
    block_big(A, b, boff, blen);
    PBL_MARK_PENDING();
    return;
  }

  PSTAMP(A, b, 1, l == 0);
  if (!wk.staged) {  // the block by LDS-DMA
    stage_dma(S, A.in.blocks, boff, blen);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    wave_sync();
  }
  PSTAMP(A, b, 2, l == 0);
  const View V = lds_view(S.x, uint32_t(kPad + (boff & 15)));
  uint32_t roff, nres;
  uint32_t status = pipe::init_checks(LdsRd{V}, blen, flags, &roff, &nres);
  bool slow = status == PBL_OK && nres > uint32_t(kPKv);
  uint32_t nkv = 0, tkb = 0, tvb = 0;
  bool published = false;
  LbWindows<kLbWin> G;
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
    else if (__ballot(!ok) || nent > uint32_t(kPKv) || tkb > kPKeyCap) slow = true;
    else if (__ballot(vbad)) status = PBL_CORRUPT_BOUNDS;  // Go: i.val[0] on an empty SET value
    if (status == PBL_OK && !slow) {
      // the sizes are final: publish, request the look-back windows, and write
      // the metadata while they are in flight
      const uint64_t agg[kNumComp] = {nkv, tkb, tvb, nres};
      lb_publish(lb_state, nb, b, agg);
      published = true;
      if (b > 0) G.issue(LbPtrs(lb_state, nb), int64_t(b) - 1);
      PSTAMP(A, b, 3, l == 0);
      MState M{ie - (kHide ? acc.ne : acc.cnt), ic - acc.cnt, ik - acc.kb, iv - acc.vb, 0, 0, 0};
      if (single) {
        if (r0 < nres) {
          park_meta<kHide>(Mt, W, V, RB, flags, M);
          if (over) span_meta<kHide>(Mt, W, V, RB.pos, RB.e0, RB.rw, RB.n, RB.prev_kl, RB.prev_kind, flags, vprefix, M);
        }
      } else {
        for (uint32_t r = r0; r < r1; r++) {
          uint32_t rw, e0;
          run_bounds(V, r, nres, roff, &rw, &e0);
          M.prev_sh = M.pp = M.ppsh = 0;
          span_meta<kHide>(Mt, W, V, rw & kRestartMask, e0, rw, 0, 0, 0, flags, vprefix, M);
        }
      }
      if (l < 5) W.vp[nkv + l] = tvb;
      if (l == 0) Mt.kout[nkv] = uint16_t(tkb);
      wave_sync();
      PSTAMP(A, b, 4, l == 0);
    }
  }

  if (status == PBL_OK && slow) {
    block_slow(S, Mt, A, b, boff, blen);
    PBL_STAGE_DONE();
    PBL_MARK_PENDING();
    return;
  }
  const gptr<const uint8_t> gb = to_glb(gblk);
#if PBL_POOL_EARLY
  PBL_STAGE_DONE();  // everything after this reads the slot and the block in global memory
  const GSrc KS{gb, blen, uint32_t(((uint64_t(gblk) + blen + 15) & ~uint64_t(15)) - uint64_t(gblk))};
  // the first key batch, the first value step and the first restarts need no
  // output offsets: their loads go out before the look-back wait
  const bool raw = (flags & PBL_ROW_RAW_KEYS) != 0;
  KBatch K;
  VBatch VB;
  uint32_t rs0 = 0;
  if (published) {
    key_load<kHide>(Mt, KS, raw, 0, nkv, K);
    val_load(W, gb, nkv, 0, VB);
    if (O.restarts && uint32_t(l) < nres) rs0 = KS.le32(roff + 4 * l);
  }
#else
  const View& KS = V;
#endif
  PBL_MARK_PENDING();

  const bool okb = status == PBL_OK;
  const uint64_t agg[kNumComp] = {okb ? nkv : 0, okb ? tkb : 0, okb ? tvb : 0, okb ? nres : 0};
  uint64_t excl[kNumComp];
  if (!published) {
    lb_publish(lb_state, nb, b, agg);
    if (b > 0) G.issue(LbPtrs(lb_state, nb), int64_t(b) - 1);
  }
  lb_finish(lb_state, nb, b, agg, excl, &O.totals->status_mask, G);
  PSTAMP(A, b, 5, l == 0);
  if (okb && overflows(O, excl, agg)) status = PBL_OVERFLOW;
  if (l == 0) {
    if (status != PBL_OK && O.key_off && excl[0] + b < O.kv_cap + nb) {
      to_glb(O.key_off)[excl[0] + b] = 0;
      to_glb(O.val_off)[excl[0] + b] = 0;
    }
    write_block_meta(O, b, nb, status, excl, agg, false);
  }
  if (status != PBL_OK) {
    if (!PBL_POOL_EARLY) release(L, s);
    return;
  }
  if (nkv == 0) {  // a block with no entries: its lone N+1 offsets
    if (l == 0) {
      Mt.kout[0] = 0;
      W.vp[0] = 0;
    }
    wave_sync();
  }

  // ---- keys and per-KV arrays: lane per KV ------------------------------------
  const uint64_t kvb = excl[0], kbb = excl[1], vbb = excl[2], rbb = excl[3];
#if PBL_POOL_EARLY
  if (!published) {
    key_load<kHide>(Mt, KS, raw, 0, nkv, K);
    val_load(W, gb, nkv, 0, VB);
    if (O.restarts && uint32_t(l) < nres) rs0 = KS.le32(roff + 4 * l);
  }
  if (O.restarts && uint32_t(l) < nres) to_glb(O.restarts)[rbb + l] = rs0;
  emit_keys_glb<kHide>(Mt, W, KS, A, b, nkv, kvb, kbb, K);
  if (O.restarts)
    for (uint32_t r = kWave + l; r < nres; r += kWave) to_glb(O.restarts)[rbb + r] = KS.le32(roff + 4 * r);
#else
  emit_keys<kHide>(Mt, W, KS, A, b, nkv, kvb, kbb);
  if (O.restarts)
    for (uint32_t r = l; r < nres; r += kWave) to_glb(O.restarts)[rbb + r] = KS.le32(roff + 4 * r);
  release(L, s);
  VBatch VB;
  val_load(W, gb, nkv, 0, VB);
#endif
  PSTAMP(A, b, 6, l == 0);

  // ---- values, global -> global --------------------------------------------
  if (tvb) copy_values_grp(W, gb, nkv, to_glb(O.val_bytes) + vbb, VB);
  PSTAMP(A, b, 7, l == 0);
  wave_sync();  // (the slot is the next block's)
}

#undef PBL_STAGE_DONE
#undef PBL_MARK_PENDING

// The persistent kernel: one workgroup of kNW waves per CU, each wave an
// independent loop of (acquire a stage, take a ticket, decode the block).
// Deadlock-free for any residency: a wave takes a ticket only while holding a
// stage, and waits (in the look-back) only on smaller tickets, all of them
// taken by waves that hold a stage or no longer need one.
template <bool kHide>
__global__ void __launch_bounds__(kTPBP, 1) rowblk_pool_kernel(Args A) {
  __shared__ PoolLds L;
  if (threadIdx.x == 0) {
    L.free_mask = (1u << kNS) - 1u;
    L.inflight = 0;
  }
  if (threadIdx.x < uint32_t(kNS)) {
    L.tk[threadIdx.x] = kTkFree;
    L.rdy[threadIdx.x] = 0;
  }
  __syncthreads();
  Slot& W = L.sl[wave_id()];
  const uint32_t nb = A.in.n_blocks;
#if PBL_POOL_AHEAD
  static_assert(PBL_POOL_EARLY, "the stage ring parks a stage right after the walk");
  for (;;) {
#ifdef PBL_STAMPS
    const uint64_t t_acq = __builtin_amdgcn_s_memtime();
#endif
    const Work wk = get_work(L, A);
    if (wk.t >= nb) break;
    PSTAMP(A, wk.t, 0, lane_id() == 0);
#ifdef PBL_STAMPS
    if (lane_id() == 0)
      reinterpret_cast<uint64_t*>(reinterpret_cast<uint8_t*>(A.out.workspace) + ws_bytes(nb))[uint64_t(wk.t) * 16 + 8] = t_acq;
#endif
    pool_block<kHide>(L, wk, W, A);
  }
#else
  uint32_t* tick = reinterpret_cast<uint32_t*>(A.out.workspace);
  for (;;) {
#ifdef PBL_STAMPS
    const uint64_t t_acq = __builtin_amdgcn_s_memtime();
#endif
    Work wk;
    wk.s = acquire(L);
    uint32_t t0 = 0;
    if (lane_id() == 0) t0 = g_atomic_add(tick, 1u);
    t0 = __builtin_amdgcn_readfirstlane(__shfl(t0, 0, kWave));
    if (t0 >= nb) {
      release(L, wk.s);
      break;
    }
    PSTAMP(A, t0, 0, lane_id() == 0);
#ifdef PBL_STAMPS
    if (lane_id() == 0)
      reinterpret_cast<uint64_t*>(reinterpret_cast<uint8_t*>(A.out.workspace) + ws_bytes(nb))[uint64_t(t0) * 16 + 8] = t_acq;
#endif
    wk.t = t0;
    wk.boff = to_glb(A.in.block_off)[t0];
    wk.blen = to_glb(A.in.block_len)[t0];
    wk.staged = false;
    pool_block<kHide>(L, wk, W, A);
  }
#endif
}

}  // namespace pool
