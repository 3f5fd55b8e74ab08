// rowblk_run.hip.h — the row-format decode with one wave per block, five
// blocks in flight per CU, and outputs written run-major straight from the
// restart-run walk (no per-KV metadata round trip).
//
// The two LDS kernels before this one hold 4 blocks per CU (pipeline: 2 x 2
// staging buffers + metadata; flat: 4 x (32 KiB + 5.4 KB of metadata)), and a
// block's life there is a latency chain: flat's phase stamps were stage 7 K,
// count walk 12 K, metadata walk 11 K, look-back 9 K, lane-per-KV emit 27 K
// cycles.  Two of those phases exist only to turn the run walk into per-KV
// metadata and back.  Here:
//
//   stage   the block HBM -> LDS by LDS-DMA into the wave's 32 KiB slot (five
//           slots = the CU's 160 KiB: nothing else lives in LDS)
//   count   lane l walks a contiguous span of g = ceil(nres / 64) restart runs
//           (rowblk_writer.go:147-155 cuts the prefix chain at each): entries,
//           user-key and value bytes, the checks of readEntry; a DPP scan gives
//           each lane its span's bases; the block's aggregate is published and
//           the look-back windows are requested
//   resolve the block's exclusive prefix (lb_finish)
//   emit    the same lane walks its span again and writes every output of each
//           entry as it goes: the internal key is kept in four 64-bit registers
//           (fullKey[:shared] + unshared, rowblk_iter.go:400), the trailer is
//           its last 8 bytes, the user key and the value leave as 16-B stores
//           (value bytes read from LDS), per-KV arrays at j = span base + k.
//           The next entry's header is read before this entry's stores.
//
// Blocks this path does not take (an internal key longer than kRKey, a restart
// table inconsistent with per-run walks, a value-prefix kind byte inside the
// shared prefix, 3-byte length varints) take the wave-serial general walk
// (rowblk_general.hip.h), from the staged block; blocks that do not fit the slot
// with their 16-B phase run it from global memory; blocks past kMaxFastLen are
// sized and written by big_block_{sizes,values}_kernel around this launch.
// Results are identical on every path.
//
// Semantics: cockroachdb/pebble sstable/rowblk/rowblk_iter.go — Init :241-276,
// readFirstKey :418-485, readEntry :333-416, decodeInternalKey :487-504, value
// prefix :1192-1199 (sstable/block/kv.go:14-41), decodeRestart :1092-1096,
// RawIter.readEntry :1784-1794.
#pragma once

namespace runk {

constexpr int kRW = 5;                              // waves (= blocks in flight) per CU
constexpr int kRTPB = kRW * kWave;
constexpr uint32_t kSlotBytes = 32768;              // one wave's LDS slot
constexpr uint32_t kSlotSlack = 32;                 // bytes a 16-B read may run past a key / value
constexpr uint32_t kRKey = 32;                      // internal-key bytes kept in registers
#ifndef PBL_RUN_LONG
#define PBL_RUN_LONG 256  // values longer than this are copied by the whole wave after the walk
#endif
constexpr uint32_t kRLongVal = PBL_RUN_LONG;
#ifndef PBL_RUN_LBWIN
#define PBL_RUN_LBWIN 8  // look-back windows per round trip: ~500 blocks are between publish and prefix here
#endif
constexpr int kRLbWin = PBL_RUN_LBWIN;

struct RLds {
  uint4 x[kRW][kSlotBytes / 16];
};
static_assert(sizeof(RLds) <= 163840, "five slots per CU");

using flat::Acc;
using flat::dpp_incl_scan;
using flat::last_lane;
using flat::store_n;

// LE64 of register-key bytes [o, o + 8), o <= 24.
__device__ __forceinline__ uint64_t key_u64(const uint64_t k[4], uint32_t o) {
  const uint32_t w = o >> 3, s = (o & 7u) * 8u;
  const uint64_t lo = w == 0 ? k[0] : w == 1 ? k[1] : w == 2 ? k[2] : k[3];
  const uint64_t hi = w == 0 ? k[1] : w == 1 ? k[2] : w == 2 ? k[3] : 0ull;
  return s ? (lo >> s) | (hi << (64u - s)) : lo;
}

// restart run r's end offset (the next run's start, or the restart table)
__device__ __forceinline__ uint32_t run_end(const View& V, uint32_t r, uint32_t nres, uint32_t roff) {
  return r + 1 < nres ? (V.le32(roff + 4 * (r + 1)) & kRestartMask) : roff;
}

// Count walk over runs [r0, r1) (one contiguous byte span): entries, output
// bytes and the largest internal key; `ok` clears where the span is not
// walkable per run (general path), `bad` sets on shared > len(previous key)
// (rowblk_iter.go:403), `vbad` on a SET value without its prefix byte.
__device__ __forceinline__ void count_span(const View& V, uint32_t r0, uint32_t r1, uint32_t nres, uint32_t roff,
                                           uint32_t flags, bool vprefix, Acc& acc, uint32_t& maxkl, bool& ok,
                                           bool& bad, bool& vbad) {
  uint32_t pos = V.le32(roff + 4 * r0) & kRestartMask;
  uint32_t rend = run_end(V, r0, nres, roff);
  if ((r0 == 0 && pos != 0) || pos >= rend || rend > roff) { ok = false; return; }
  uint32_t r = r0, prev_kl = 0, cnt = 0, kb = 0, vb = 0, mk = 0;
  bool first = true;
  for (;;) {
    if (pos == rend) {
      if (++r >= r1) break;
      const uint32_t e = run_end(V, r, nres, roff);
      if (e <= pos || e > roff) { ok = false; return; }
      rend = e;
      first = true;
    }
    uint32_t sh, un, vl, h;
    const bool hok = pipe::hdr2(V.ld8(pos), &sh, &un, &vl, &h);
    const uint32_t np = pos + h + un + vl;
    if (!hok || (first && sh != 0) || np > rend) { ok = false; return; }
    bad = bad || (!first && sh > prev_kl);
    const uint32_t kl = sh + un;
    uint32_t vlen = vl;
    if (vprefix && kl >= 8) {
      if (kl - 8 < sh) { ok = false; return; }  // kind byte inside the shared prefix
      if ((V.byte(pos + h + (kl - 8 - sh)) & 0xBF) == 1) {
        if (vl == 0) vbad = true;
        else if ((V.byte(pos + h + un) & 0xC0) == 0 || (flags & PBL_ROW_NO_VALUER)) vlen--;
      }
    }
    kb += (flags & PBL_ROW_RAW_KEYS) ? kl : (kl >= 8 ? kl - 8 : 0);
    vb += vlen;
    mk = kl > mk ? kl : mk;
    cnt++;
    prev_kl = kl;
    first = false;
    pos = np;
  }
  acc = Acc{cnt, kb, vb};
  maxkl = mk;
}

// A 16-B store at p when [p, p + 16) lies below `end` (the lane's own output
// range: bytes past this key / value belong to its later entries, whose stores
// come later in program order and overwrite them), else exactly the bytes below
// `end`.
__device__ __forceinline__ void store_clip(gptr<uint8_t> base, uint32_t at, uint32_t end, const uint4& w) {
  if (at + 16 <= end) *(gptr<flat::u32x4_ug>)(base + at) = u32x4{w.x, w.y, w.z, w.w};
  else store_n(base + at, w, end - at);
}

// Emit walk over runs [r0, r1), validated by count_span: every output of
// each entry, KV j = S.cnt + k of the block; the lane's key and value bytes
// end at E.kb / E.vb.  Values longer than kRLongVal are left to the wave
// (their lanes return true).
__device__ __forceinline__ bool emit_span(const View& V, uint32_t r0, uint32_t r1, uint32_t nres, uint32_t roff,
                                          uint32_t flags, bool vprefix, uint64_t seq, Acc S, Acc E,
                                          const pbl_decode_out& O, uint64_t kvb, uint32_t b, gptr<uint8_t> kbytes,
                                          gptr<uint8_t> vbytes) {
  const bool rawk = (flags & PBL_ROW_RAW_KEYS) != 0;
  uint32_t pos = V.le32(roff + 4 * r0) & kRestartMask;
  uint32_t rw = V.le32(roff + 4 * r0), rend = run_end(V, r0, nres, roff), r = r0;
  uint64_t k[4] = {0, 0, 0, 0};
  uint64_t hw = V.ld8(pos);
  bool first = true, has_long = false;
  uint32_t kb = S.kb, vb = S.vb;
  const gptr<uint64_t> o_tr = to_glb(O.trailer) + kvb + S.cnt;
  const gptr<uint8_t> o_fl = to_glb(O.kv_flags) + kvb + S.cnt;
  const gptr<uint32_t> o_eo = to_glb(O.entry_off) + kvb + S.cnt;
  const gptr<uint32_t> o_ko = to_glb(O.key_off) + kvb + b + S.cnt, o_vo = to_glb(O.val_off) + kvb + b + S.cnt;
  const bool has_fl = O.kv_flags != nullptr, has_eo = O.entry_off != nullptr;
  for (uint32_t j = 0;; j++) {
    if (pos == rend) {
      if (++r >= r1) break;
      rw = V.le32(roff + 4 * r);
      rend = run_end(V, r, nres, roff);
      first = true;
    }
    uint32_t sh, un, vl, h;
    pipe::hdr2(hw, &sh, &un, &vl, &h);
    const uint32_t np = pos + h + un + vl;
    if (np < rend || r + 1 < r1) hw = V.ld8(np);  // the next header, ahead of this entry's work
    const uint32_t kl = sh + un, ks = pos + h;
    // fullKey = fullKey[:shared] + unshared: key byte p >= shared sits at LDS ks - sh + p
    {
      const int32_t src = int32_t(ks) - int32_t(sh);
      const uint4 n0 = V.ld16(src), n1 = V.ld16(src + 16);
      const uint64_t n[4] = {uint64_t(n0.x) | uint64_t(n0.y) << 32, uint64_t(n0.z) | uint64_t(n0.w) << 32,
                             uint64_t(n1.x) | uint64_t(n1.y) << 32, uint64_t(n1.z) | uint64_t(n1.w) << 32};
#pragma unroll
      for (int w = 0; w < 4; w++) {
        const int32_t d = int32_t(sh) - 8 * w;  // bytes of word w kept from the previous key
        const uint64_t m = d >= 8 ? ~0ull : d <= 0 ? 0ull : ((1ull << (8 * d)) - 1ull);
        k[w] = (k[w] & m) | (n[w] & ~m);
      }
    }
    uint8_t fl = first ? uint8_t(PBL_KV_RESTART | ((rw >> 31) ? PBL_KV_RESTART_SAMEPFX : 0)) : uint8_t(0);
    uint64_t tr = 0;
    uint32_t vs = ks + un, vlen = vl;
    if (!rawk) {
      if (kl < 8) {
        fl |= PBL_KV_INVALID_KEY;
        tr = kKindInvalid;
      } else {
        const uint64_t raw = key_u64(k, kl - 8);
        if (raw & 64u) fl |= PBL_KV_OBSOLETE;
        tr = raw & kTrailerObsoleteMask;
        if (vprefix && (uint32_t(raw) & 0xBFu) == 1u) {
          const uint32_t pre = V.byte(vs);
          if ((pre & 0xC0) == 0 || (flags & PBL_ROW_NO_VALUER)) { vs++; vlen--; }
          else if ((pre & 0xC0) == 0x80) fl |= PBL_KV_VALBLK_HANDLE;
          else fl |= PBL_KV_BLOB_HANDLE;
        }
      }
    }
    const uint32_t ukl = rawk ? kl : (kl >= 8 ? kl - 8 : 0u);
    o_tr[j] = with_seq(tr, seq, flags);
    if (has_fl) o_fl[j] = fl;
    if (has_eo) o_eo[j] = pos;
    o_ko[j] = kb;
    o_vo[j] = vb;
    if (ukl) {
      store_clip(kbytes, kb, E.kb, make_uint4(uint32_t(k[0]), uint32_t(k[0] >> 32), uint32_t(k[1]), uint32_t(k[1] >> 32)));
      if (ukl > 16)
        store_clip(kbytes, kb + 16, E.kb, make_uint4(uint32_t(k[2]), uint32_t(k[2] >> 32), uint32_t(k[3]), uint32_t(k[3] >> 32)));
    }
    if (vlen <= kRLongVal) {
      for (uint32_t c = 0; c < vlen; c += 16) store_clip(vbytes, vb + c, E.vb, V.ld16(int32_t(vs + c)));
    } else {
      has_long = true;
    }
    kb += ukl;
    vb += vlen;
    first = false;
    pos = np;
  }
  return has_long;
}

// The long values of lane s's span, copied by the whole wave (wave-uniform
// re-walk of that span's headers; values in LDS, 16 B per lane per step).
__device__ __forceinline__ void long_values(const View& V, uint32_t r0, uint32_t r1, uint32_t nres, uint32_t roff,
                                            uint32_t flags, bool vprefix, uint32_t vb, gptr<uint8_t> vbytes) {
  const uint32_t l = lane_id();
  const bool rawk = (flags & PBL_ROW_RAW_KEYS) != 0;
  uint32_t pos = V.le32(roff + 4 * r0) & kRestartMask, rend = run_end(V, r0, nres, roff), r = r0;
  for (;;) {
    if (pos == rend) {
      if (++r >= r1) break;
      rend = run_end(V, r, nres, roff);
    }
    uint32_t sh, un, vl, h;
    pipe::hdr2(V.ld8(pos), &sh, &un, &vl, &h);
    const uint32_t kl = sh + un, ks = pos + h;
    uint32_t vs = ks + un, vlen = vl;
    if (vprefix && !rawk && kl >= 8) {
      // the kind byte is in this entry's unshared bytes (count_span sends the
      // other case to the general path)
      if ((V.byte(ks + (kl - 8 - sh)) & 0xBF) == 1) {
        const uint32_t pre = V.byte(vs);
        if ((pre & 0xC0) == 0 || (flags & PBL_ROW_NO_VALUER)) { vs++; vlen--; }
      }
    }
    if (vlen > kRLongVal)
      for (uint32_t c = 16u * l; c < vlen; c += 16u * kWave) {
        const uint32_t n = vlen - c < 16 ? vlen - c : 16u;
        store_n(vbytes + vb + c, V.ld16(int32_t(vs + c)), n);
      }
    vb += vlen;
    pos = pos + h + un + vl;
  }
}

// The block HBM -> LDS by LDS-DMA: granule g of the 16-B aligned source range
// lands at x[g] (block byte i at (boff & 15) + i).
__device__ __forceinline__ void stage(lptr<uint4> slot, const uint8_t* blocks, uint64_t boff, uint32_t blen) {
  const uint64_t a0 = boff & ~uint64_t(15), a1 = (boff + blen + 15) & ~uint64_t(15);
  const uint32_t n16 = uint32_t((a1 - a0) >> 4);
  const uint32_t l = lane_id();
  const gptr<const uint8_t> base = to_glb(blocks + a0);
  for (uint32_t g0 = 0; g0 < n16; g0 += kWave) {
    if (g0 + l < n16)
      __builtin_amdgcn_global_load_lds((gptr<const void>)(base + 16ull * (g0 + l)), (lptr<void>)(slot + g0), 16, 0,
                                       0);
  }
}

// One block on one wave.
__device__ __forceinline__ void run_block(uint4* slot_g, const Args& A, uint32_t b) {
  const uint32_t l = lane_id();
  const uint32_t nb = A.in.n_blocks, flags = A.in.flags;
  const uint64_t boff = to_glb(A.in.block_off)[b];
  const uint32_t blen = to_glb(A.in.block_len)[b];
  const bool vprefix = (flags & PBL_ROW_VALUE_PREFIX) && !(flags & PBL_ROW_RAW_KEYS);
  uint8_t* ws = reinterpret_cast<uint8_t*>(A.out.workspace);
  uint64_t* lb_state = reinterpret_cast<uint64_t*>(ws + kWsHeader);
  const uint8_t* gblk = A.in.blocks + boff;

  if (blen > kMaxFastLen) {
    // past kMaxFastLen: big_block_sizes_kernel walked it, published its
    // aggregate and left {status, counts} in its block-metadata slots;
    // big_block_values_kernel writes its outputs after this launch
    const uint32_t st0 = to_glb(A.out.blk_status)[b];
    const bool okk = st0 == PBL_OK;
    const uint64_t agg[kNumComp] = {okk ? to_glb(A.out.blk_kv_base)[b] : 0, okk ? to_glb(A.out.blk_key_base)[b] : 0,
                                    okk ? to_glb(A.out.blk_val_base)[b] : 0,
                                    okk ? uint64_t(SlowGlb{to_glb(gblk), blen}.le32(blen - 4)) : 0};
    uint64_t excl[kNumComp];
    lb_resolve(lb_state, nb, b, agg, excl, &A.out.totals->status_mask);
    uint32_t st2 = st0;
    if (okk && overflows(A.out, excl, agg)) st2 = PBL_OVERFLOW;
    if (l == 0) {
      if (st2 != PBL_OK && A.out.key_off && excl[0] + b < A.out.kv_cap + nb) {
        to_glb(A.out.key_off)[excl[0] + b] = 0;
        to_glb(A.out.val_off)[excl[0] + b] = 0;
      }
      write_block_meta(A.out, b, nb, st2, excl, agg, true);
    }
    return;
  }

  const uint32_t phase = uint32_t(boff & 15);
  const bool fits = phase + blen + kSlotSlack <= kSlotBytes;
  const lptr<uint4> slot = to_lds_ptr(slot_g);
  PSTAMP(A, b, 0, l == 0);
  if (fits) {
    stage(slot, A.in.blocks, boff, blen);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    wave_sync();
  }
  PSTAMP(A, b, 1, l == 0);
  const View V = lds_view(slot_g, phase);
  uint32_t roff = 0, nres = 0;
  uint32_t status = fits ? pipe::init_checks(LdsRd{V}, blen, flags, &roff, &nres)
                         : pipe::init_checks(GlbRd{gblk}, blen, flags, &roff, &nres);
  bool slow = !fits;
  uint32_t nkv = 0, tkb = 0, tvb = 0, r0 = 0, r1 = 0, cnt_l = 0, kb_l = 0, vb_l = 0;
  Acc base{0, 0, 0};
  bool published = false;
  LbWindows<kRLbWin> G;
  if (status == PBL_OK && !slow && roff > 0) {
    const uint32_t g = (nres + kWave - 1) / kWave;
    r0 = l * g;
    r1 = r0 + g < nres ? r0 + g : nres;
    bool ok = true, bad = false, vbad = false;
    Acc acc{0, 0, 0};
    uint32_t mk = 0;
    if (r0 < nres) count_span(V, r0, r1, nres, roff, flags, vprefix, acc, mk, ok, bad, vbad);
    const uint32_t ic = dpp_incl_scan(acc.cnt), ik = dpp_incl_scan(acc.kb), iv = dpp_incl_scan(acc.vb);
    base = Acc{ic - acc.cnt, ik - acc.kb, iv - acc.vb};
    cnt_l = acc.cnt;
    kb_l = acc.kb;
    vb_l = acc.vb;
    nkv = last_lane(ic);
    tkb = last_lane(ik);
    tvb = last_lane(iv);
    if (__ballot(bad)) status = PBL_CORRUPT_BOUNDS;
    else if (__ballot(!ok || mk > kRKey)) slow = true;
    else if (__ballot(vbad)) status = PBL_CORRUPT_BOUNDS;  // Go: i.val[0] on an empty SET value
    if (status == PBL_OK && !slow) {
      const uint64_t agg[kNumComp] = {nkv, tkb, tvb, nres};
      lb_publish(lb_state, nb, b, agg);
      published = true;
      PSTAMP(A, b, 2, l == 0);
      if (b > 0) G.issue(LbPtrs(lb_state, nb), int64_t(b) - 1);
    }
  }

  if (status == PBL_OK && slow) {
    // general path (wave-serial Iter.Next): on the staged block with the
    // slot's tail as its key buffer when that holds the keys, else from
    // global memory with the whole slot as the key buffer
    SlowState ss;
    uint64_t dummy[kNumComp] = {0, 0, 0, 0}, excl[kNumComp];
    const uint8_t* src = gblk;
    bool from_lds = false;
    uint8_t* keybuf = reinterpret_cast<uint8_t*>(slot_g);
    uint32_t keycap = kSlotBytes;
    const uint32_t used = (phase + blen + kSlotSlack + 15) & ~15u;
    // (the staged form reads 16-B windows from up to 16 bytes before the
    // block's granule: not from the first slot, which starts at LDS address 0)
    const bool lds_ok = uint32_t(uint64_t(to_lds_ptr(slot_g))) >= 16u;
    if (fits && lds_ok && kSlotBytes - used >= 1024) {
      src = reinterpret_cast<const uint8_t*>(slot_g) + phase;
      from_lds = true;
      keybuf = reinterpret_cast<uint8_t*>(slot_g) + used;
      keycap = kSlotBytes - used;
      slow_walk(src, true, blen, flags, A.in.synthetic_seq_num, keybuf, keycap, kPassCount, A.out, b, dummy, &ss);
      if (ss.status == PBL_UNSUPPORTED) {
        wave_sync();
        from_lds = false;
        src = gblk;
        keybuf = reinterpret_cast<uint8_t*>(slot_g);
        keycap = kSlotBytes;
      }
    }
    if (!from_lds)
      slow_walk(src, false, blen, flags, A.in.synthetic_seq_num, keybuf, keycap, kPassCount, A.out, b, dummy, &ss);
    const bool okk = ss.status == PBL_OK;
    const uint64_t agg[kNumComp] = {okk ? ss.nkv : 0, okk ? ss.kb : 0, okk ? ss.vb : 0, okk ? ss.nr : 0};
    lookback(lb_state, nb, b, agg, excl, &A.out.totals->status_mask);
    uint32_t st2 = ss.status;
    if (okk && overflows(A.out, excl, agg)) st2 = PBL_OVERFLOW;
    if (st2 == PBL_OK)
      slow_walk(src, from_lds, blen, flags, A.in.synthetic_seq_num, keybuf, keycap, kPassAll, A.out, b, excl, &ss);
    else if (l == 0 && A.out.key_off && excl[0] + b < A.out.kv_cap + nb) {
      to_glb(A.out.key_off)[excl[0] + b] = 0;
      to_glb(A.out.val_off)[excl[0] + b] = 0;
    }
    if (l == 0) write_block_meta(A.out, b, nb, st2, excl, agg, true);
    wave_sync();
    return;
  }

  const bool okb = status == PBL_OK;
  const uint64_t agg[kNumComp] = {okb ? nkv : 0, okb ? tkb : 0, okb ? tvb : 0, okb ? nres : 0};
  uint64_t excl[kNumComp];
  if (!published) {
    lb_publish(lb_state, nb, b, agg);
    if (b > 0) G.issue(LbPtrs(lb_state, nb), int64_t(b) - 1);
  }
  lb_finish(lb_state, nb, b, agg, excl, &A.out.totals->status_mask, G);
  PSTAMP(A, b, 3, l == 0);
  if (okb && overflows(A.out, excl, agg)) status = PBL_OVERFLOW;
  if (l == 0) {
    if (status != PBL_OK && A.out.key_off && excl[0] + b < A.out.kv_cap + nb) {
      to_glb(A.out.key_off)[excl[0] + b] = 0;
      to_glb(A.out.val_off)[excl[0] + b] = 0;
    }
    write_block_meta(A.out, b, nb, status, excl, agg, false);
  }
  if (status != PBL_OK) {
    wave_sync();
    return;
  }

  // ---- emit: lane per span of restart runs ----------------------------------
  const pbl_decode_out& O = A.out;
  const uint64_t kvb = excl[0], rbb = excl[3];
  const gptr<uint8_t> kbytes = to_glb(O.key_bytes) + excl[1], vbytes = to_glb(O.val_bytes) + excl[2];
  if (l == 0) {  // the block's N+1-th offsets
    to_glb(O.key_off)[kvb + b + nkv] = tkb;
    to_glb(O.val_off)[kvb + b + nkv] = tvb;
  }
  bool has_long = false;
  if (r0 < nres && roff > 0)
    has_long = emit_span(V, r0, r1, nres, roff, flags, vprefix, A.in.synthetic_seq_num, base,
                         Acc{base.cnt + cnt_l, base.kb + kb_l, base.vb + vb_l}, O, kvb, b, kbytes, vbytes);
  for (uint64_t lm = __ballot(has_long); lm; lm &= lm - 1) {
    const int s = __builtin_ctzll(lm);
    const uint32_t s0 = __builtin_amdgcn_readlane(r0, s), s1 = __builtin_amdgcn_readlane(r1, s);
    const uint32_t svb = __builtin_amdgcn_readlane(base.vb, s);
    long_values(V, s0, s1, nres, roff, flags, vprefix, svb, vbytes);
  }
  if (O.restarts)
    for (uint32_t r = l; r < nres; r += kWave) to_glb(O.restarts)[rbb + r] = V.le32(roff + 4 * r);
  PSTAMP(A, b, 4, l == 0);
  wave_sync();  // (the slot is the next block's)
}

// The persistent kernel: one workgroup of five waves per CU, each wave an
// independent stream of tickets (one block each), decoded in order.
// Deadlock-free for any residency: a block's look-back waits only on smaller
// tickets, all taken by resident waves that publish before they wait.
__global__ void __launch_bounds__(kRTPB, 1) rowblk_run_kernel(Args A) {
  __shared__ RLds L;
  uint4* slot = L.x[wave_id()];
  const uint32_t nb = A.in.n_blocks;
  uint32_t* tick = reinterpret_cast<uint32_t*>(A.out.workspace);
  for (;;) {
    uint32_t t0 = 0;
    if (lane_id() == 0) t0 = g_atomic_add(tick, 1u);
    t0 = __builtin_amdgcn_readfirstlane(__shfl(t0, 0, kWave));
    if (t0 >= nb) break;
    run_block(slot, A, t0);
  }
}

}  // namespace runk
