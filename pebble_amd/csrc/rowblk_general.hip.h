// rowblk_general.hip.h — the general (non-LDS-fast-path) row-block decoder and
// the per-block metadata helpers shared by both paths.  Included by
// rowblk_decode.hip inside namespace pbl::row (needs Args, kTrailerObsoleteMask,
// kKindInvalid, kRestartMask).
#pragma once


// ---------------------------------------------------------------------------
// General path: a wave-serial restatement of Iter.First/Next (block bytes read
// through a generic pointer: LDS when staged, else global), current key in LDS.
// Executed by wave 0 only.
// ---------------------------------------------------------------------------
struct SlowState {
  uint64_t nkv, kb, vb, nr;
  uint32_t status;
};

__device__ inline uint32_t g_varint(const uint8_t* p, const uint8_t* end, uint32_t* v) {
  uint32_t r = 0;
  for (int i = 0; i < 5; i++) {
    if (p + i >= end) return 0;
    uint32_t b = p[i];
    if (i == 4) { *v = r | (b << 28); return 5; }
    if (b < 128) { *v = r | (b << (7 * i)); return i + 1; }
    r |= (b & 0x7f) << (7 * i);
  }
  return 0;
}

__device__ inline uint32_t g_le32(const uint8_t* p) {
  return uint32_t(p[0]) | uint32_t(p[1]) << 8 | uint32_t(p[2]) << 16 | uint32_t(p[3]) << 24;
}

// Block sources of the general path.  Both read bytes, LE32 words and 16-byte
// windows at block offsets; an ld16 window may start up to 15 bytes before the
// block or end past it (those bytes are don't-cares; nothing outside the
// block's 16-B granules is touched).  Typed address spaces throughout: a
// generic (FLAT) LDS read would wait for every outstanding global store.
struct SlowLds {  // block staged in LDS (byte 0 at B[base])
  View V;
  __device__ __forceinline__ uint32_t byte(uint64_t i) const { return V.byte(uint32_t(i)); }
  __device__ __forceinline__ uint32_t le32(uint64_t i) const { return V.le32(uint32_t(i)); }
  __device__ __forceinline__ uint4 ld16(int64_t i) const { return V.ld16(int32_t(i)); }
};
struct SlowGlb {  // block in global memory
  gptr<const uint8_t> g;
  uint64_t len;
  __device__ __forceinline__ uint32_t byte(uint64_t i) const { return g[i]; }
  __device__ __forceinline__ uint32_t le32(uint64_t i) const {
    return uint32_t(g[i]) | uint32_t(g[i + 1]) << 8 | uint32_t(g[i + 2]) << 16 | uint32_t(g[i + 3]) << 24;
  }
  __device__ __forceinline__ uint4 ld16(int64_t i) const {
    const uint64_t s0 = uint64_t(g), s1 = s0 + len, sx = s0 + uint64_t(i), sa = sx & ~uint64_t(15);
    const uint32_t sh = uint32_t(sx - sa);
    uint4 x = make_uint4(0, 0, 0, 0), y = make_uint4(0, 0, 0, 0);
    if (sa + 16 > s0 && sa < s1) {
      const u32x4 v = *(gptr<const u32x4>)(sa);
      x = make_uint4(v.x, v.y, v.z, v.w);
    }
    if (sh && sa + 32 > s0 && sa + 16 < s1) {
      const u32x4 v = *(gptr<const u32x4>)(sa + 16);
      y = make_uint4(v.x, v.y, v.z, v.w);
    }
    return sh ? col::funnel16(x, y, sh) : x;
  }
  // Block bytes from offset v -> out[lo, hi), 16-B destination granules, U per
  // lane in flight.  Every granule's two source loads are issued before any is
  // used, at addresses clamped to the block's own granules (those bytes feed
  // only masked destination bytes); the shift is one per value.  Through ld16
  // each granule's guarded loads and funnel waited in turn: config 5's
  // big-block values pass, one 48 KB value per block, took 125 us.
  template <int U>
  __device__ __forceinline__ void copy(uint64_t v, uint8_t* out, uint64_t lo, uint64_t hi) const {
    const uint64_t s0 = uint64_t(g), g_lo = s0 & ~uint64_t(15), g_hi = (s0 + len - 1) & ~uint64_t(15);
    const uint64_t d = s0 + v - lo;  // source address of destination offset ga: d + ga
    const uint32_t sh = __builtin_amdgcn_readfirstlane(uint32_t(d) & 15u);
    for (uint64_t g0 = (lo & ~uint64_t(15)) + 16ull * lane_id(); g0 < hi; g0 += 16ull * kWave * U) {
      u32x4 x[U], y[U];
#pragma unroll
      for (int u = 0; u < U; u++) {
        const uint64_t sa = (d + g0 + 16ull * kWave * u) & ~uint64_t(15);
        x[u] = *(gptr<const u32x4>)(min(max(sa, g_lo), g_hi));
        if (sh) y[u] = *(gptr<const u32x4>)(min(max(sa + 16, g_lo), g_hi));
      }
#pragma unroll
      for (int u = 0; u < U; u++) {
        const uint64_t ga = g0 + 16ull * kWave * u;
        const uint4 a = make_uint4(x[u].x, x[u].y, x[u].z, x[u].w);
        if (ga < hi)
          store16(out, ga, lo, hi, sh ? col::funnel16(a, make_uint4(y[u].x, y[u].y, y[u].z, y[u].w), sh) : a);
      }
    }
  }
};

// byte k (< 16) of a 16-byte window, by shifts (a runtime-indexed register
// array would live in scratch)
__device__ __forceinline__ uint32_t win_byte(const uint4& w, uint32_t k) {
  const uint64_t q = k < 8 ? (uint64_t(w.x) | uint64_t(w.y) << 32) : (uint64_t(w.z) | uint64_t(w.w) << 32);
  return uint32_t(q >> (8 * (k & 7))) & 0xffu;
}

// varint at window bytes [i0, n) (g_varint's rules: 5th byte << 28, none past n)
__device__ __forceinline__ uint32_t w_varint(const uint4& w, uint32_t i0, uint32_t n, uint32_t* v) {
  uint32_t r = 0;
#pragma unroll
  for (uint32_t i = 0; i < 5; i++) {
    if (i0 + i >= n) return 0;
    const uint32_t b = win_byte(w, i0 + i);
    if (i == 4) { *v = r | (b << 28); return 5; }
    if (b < 128) { *v = r | (b << (7 * i)); return i + 1; }
    r |= (b & 0x7f) << (7 * i);
  }
  return 0;
}

// Key buffer: LDS bytes with a 16-B front pad and a 32-B tail so that 16-B
// gathers around the key stay inside it.
constexpr uint32_t kKeyBufPad = 16, kKeyBufSlack = 48;

// Walk passes: kPassCount counts; kPassAll writes every output at the given bases.
enum { kPassCount = 0, kPassAll = 1 };

#ifndef PBL_SLOW_U
#define PBL_SLOW_U 1
#endif

// U: value granules per lane in flight.
template <class Src, int U>
__device__ __forceinline__ void slow_walk_t(const Src S, uint64_t len, uint32_t flags, uint64_t seq, lptr<uint8_t> kbuf,
                                            uint32_t keycap, int pass, const pbl_decode_out& O, uint32_t b,
                                            const uint64_t bases[kNumComp], SlowState* st) {
  const int l = lane_id();
  lptr<uint8_t> keybuf = kbuf + kKeyBufPad;
  const lptr<const uint32_t> KW = (lptr<const uint32_t>)kbuf;
  keycap = keycap > kKeyBufSlack ? keycap - kKeyBufSlack : 0;
  const gptr<uint64_t> o_trailer = to_glb(O.trailer);
  const gptr<uint8_t> o_flags = to_glb(O.kv_flags);
  const gptr<uint32_t> o_entry = to_glb(O.entry_off), o_koff = to_glb(O.key_off), o_voff = to_glb(O.val_off);
  const int32_t nr = int32_t(S.le32(len - 4));
  const int64_t restarts = int64_t(len) - 4 * (1 + int64_t(nr));
  uint64_t nkv = 0, kb = 0, vb = 0, full_len = 0;
  int64_t offset = 0;
  uint32_t ri = 0;
  // restart word ri, held in a register: re-read only when the walk passes it
  uint32_t rw_ri = (pass == kPassAll && nr > 0 && restarts >= 0) ? S.le32(uint64_t(restarts)) : 0u;
  uint32_t status = PBL_OK;
  // the next entry's header window is loaded before this entry's stores: a
  // load's data waits for every older vector-memory op, so a header read
  // behind the value stores would wait for all of them (config 5's values walk:
  // see rowblk_global.hip.h)
  uint4 hw_next = restarts > 0 ? S.ld16(0) : make_uint4(0, 0, 0, 0);
  while (offset >= 0 && offset < restarts) {
    // the header's bytes in one window, the three varints from registers
    const uint4 hw = hw_next;
    const uint32_t hn = uint32_t(min<int64_t>(15, int64_t(len) - offset));
    uint32_t shared, unshared, vlen;
    const uint32_t a = w_varint(hw, 0, hn, &shared);
    const uint32_t bb = a ? w_varint(hw, a, hn, &unshared) : 0;
    const uint32_t c = bb ? w_varint(hw, a + bb, hn, &vlen) : 0;
    if (!c) { status = PBL_CORRUPT_BOUNDS; break; }
    const uint64_t kp = uint64_t(offset) + a + bb + c;
    if (len - kp < unshared) { status = PBL_CORRUPT_BOUNDS; break; }
    const uint64_t vp = kp + unshared;
    if (len - vp < vlen) { status = PBL_CORRUPT_BOUNDS; break; }
    if (shared > full_len) { status = PBL_CORRUPT_BOUNDS; break; }
    const uint64_t klen = uint64_t(shared) + unshared;
    if (klen > keycap) { status = PBL_UNSUPPORTED; break; }
    if (int64_t(vp + vlen) < restarts) hw_next = S.ld16(int64_t(vp + vlen));
    wave_sync();
    // unshared key bytes -> keybuf[shared, klen): one 16-B window per lane step
    for (uint32_t i0 = 16u * l; i0 < unshared; i0 += 16u * kWave) {
      const uint4 w = S.ld16(int64_t(kp + i0));
      const uint32_t n = min(16u, unshared - i0);
#pragma unroll
      for (uint32_t k = 0; k < 16; k++)
        if (k < n) keybuf[shared + i0 + k] = uint8_t(win_byte(w, k));
    }
    wave_sync();
    full_len = klen;
    uint64_t trailer, ukl;
    uint8_t fl = 0;
    if (flags & PBL_ROW_RAW_KEYS) {
      trailer = 0;
      ukl = klen;
    } else if (klen >= 8) {
      uint64_t raw = 0;
#pragma unroll
      for (int i = 0; i < 8; i++) raw |= uint64_t(keybuf[klen - 8 + i]) << (8 * i);
      if (raw & 64u) fl |= PBL_KV_OBSOLETE;
      trailer = raw & kTrailerObsoleteMask;
      ukl = klen - 8;
    } else {
      trailer = kKindInvalid;
      ukl = 0;
      fl |= PBL_KV_INVALID_KEY;
    }
    // blockiter.Transforms.HideObsoletePoints: the entry is skipped before its
    // value is looked at (rowblk_iter.go:1168-1179); its key still feeds the
    // prefix compression of the entries after it
    if ((flags & PBL_ROW_HIDE_OBSOLETE) && (fl & PBL_KV_OBSOLETE)) {
      offset = int64_t(vp) + vlen;
      continue;
    }
    uint64_t v = vp, vl = vlen;
    if ((flags & PBL_ROW_VALUE_PREFIX) && !(flags & PBL_ROW_RAW_KEYS) && (trailer & 0xff) == 1) {
      if (vl == 0) { status = PBL_CORRUPT_BOUNDS; break; }
      const uint32_t pre = S.byte(v);
      if ((pre & 0xC0) == 0 || (flags & PBL_ROW_NO_VALUER)) { v++; vl--; }
      else if ((pre & 0xC0) == 0x80) fl |= PBL_KV_VALBLK_HANDLE;
      else fl |= PBL_KV_BLOB_HANDLE;
    }
    if (pass == kPassAll) {
      while (ri < uint32_t(nr) && int64_t(rw_ri & kRestartMask) < offset) {
        ri++;
        if (ri < uint32_t(nr)) rw_ri = S.le32(uint64_t(restarts) + 4 * ri);
      }
      if (ri < uint32_t(nr)) {
        const uint32_t rw = rw_ri;
        if (int64_t(rw & kRestartMask) == offset) {
          fl |= PBL_KV_RESTART;
          if (rw & 0x80000000u) fl |= PBL_KV_RESTART_SAMEPFX;
        }
      }
      const uint64_t kv = bases[0] + nkv, o = bases[0] + b + nkv;
      if (l == 0) {
        o_trailer[kv] = with_seq(trailer, seq, flags);
        if (O.kv_flags) o_flags[kv] = fl;
        if (O.entry_off) o_entry[kv] = uint32_t(offset);
        o_koff[o] = uint32_t(kb);
        o_voff[o] = uint32_t(vb);
      }
      // user key: 16-B destination granules gathered from the key buffer
      {
        const uint64_t lo = bases[1] + kb, hi = lo + ukl;
        for (uint64_t ga = (lo & ~uint64_t(15)) + 16ull * l; ga < hi; ga += 16ull * kWave)
          store16(O.key_bytes, ga, lo, hi, lds_gather16(KW, uint32_t(int64_t(kKeyBufPad) + int64_t(ga - lo))));
      }
    }
    if (pass == kPassAll) {
      // value: 16-B destination granules from source windows, U per lane in flight
      const uint64_t lo = bases[2] + vb, hi = lo + vl;
      if constexpr (std::is_same<Src, SlowGlb>::value) {
        S.template copy<U>(v, O.val_bytes, lo, hi);
      } else {
        for (uint64_t g0 = (lo & ~uint64_t(15)) + 16ull * l; g0 < hi; g0 += 16ull * kWave * U) {
          uint4 w[U];
#pragma unroll
          for (int u = 0; u < U; u++) {
            const uint64_t ga = g0 + 16ull * kWave * u;
            w[u] = ga < hi ? S.ld16(int64_t(v) + int64_t(ga - lo)) : make_uint4(0, 0, 0, 0);
          }
#pragma unroll
          for (int u = 0; u < U; u++) {
            const uint64_t ga = g0 + 16ull * kWave * u;
            if (ga < hi) store16(O.val_bytes, ga, lo, hi, w[u]);
          }
        }
      }
    }
    nkv++;
    kb += ukl;
    vb += vl;
    offset = int64_t(vp) + vlen;
  }
  if (status == PBL_OK && (kb >> 32 || vb >> 32)) status = PBL_UNSUPPORTED;
  if (pass == kPassAll && status == PBL_OK) {
    const uint64_t o = bases[0] + b + nkv;
    if (l == 0) { o_koff[o] = uint32_t(kb); o_voff[o] = uint32_t(vb); }
    if (O.restarts) {
      const gptr<uint32_t> o_rst = to_glb(O.restarts);
      for (int32_t r = l; r < nr; r += kWave) o_rst[bases[3] + r] = S.le32(uint64_t(restarts) + 4ull * r);
    }
  }
  st->status = status;
  st->nkv = nkv;
  st->kb = kb;
  st->vb = vb;
  st->nr = uint64_t(nr);
}

// blk: the block's first byte, in LDS (staged, blk_lds) or global memory;
// keybuf: LDS (dword aligned) of keycap bytes.
__device__ __noinline__ void slow_walk(const uint8_t* blk, bool blk_lds, uint64_t len, uint32_t flags, uint64_t seq,
                                       uint8_t* keybuf, uint32_t keycap, int pass, const pbl_decode_out O,
                                       uint32_t b, const uint64_t* bases_p, SlowState* st) {
  const uint64_t bases[kNumComp] = {bases_p[0], bases_p[1], bases_p[2], bases_p[3]};
  const lptr<uint8_t> kbuf = to_lds_ptr(keybuf);
  if (blk_lds) {
    // View base: the 16-B granule below the block's own granule (ld16 windows
    // start up to 15 bytes early; the staging buffers carry a 16-B front pad)
    const uint32_t a = uint32_t(uint64_t(to_lds_ptr(blk)));
    const uint32_t base = 16u + (a & 15u);
    slow_walk_t<SlowLds, PBL_SLOW_U>(SlowLds{lds_view(reinterpret_cast<const void*>(blk - base), base)}, len, flags,
                                     seq, kbuf, keycap, pass, O, b, bases, st);
  } else {
    slow_walk_t<SlowGlb, PBL_SLOW_U>(SlowGlb{to_glb(blk), len}, len, flags, seq, kbuf, keycap, pass, O, b, bases, st);
  }
}


