// rowblk_flat.hip.h — the row-format decode with one wave per block and
// lane-per-KV output, four independent waves per CU.
//
// The LDS pipeline (rowblk_pipe.hip.h) splits a block over two stages (a parse
// wave, three emit waves) and writes outputs granule by granule: ~9 K vector
// instructions per block, most of them the per-granule lookups of the value
// copy, and 4 blocks in flight per CU.  Here each wave owns a block end to end:
//
//   stage    the block HBM -> LDS by LDS-DMA (global_load_lds_dwordx4, no
//            registers), one round trip
//   pass 1   lane per restart run (rowblk_writer.go:147-155 cuts the prefix
//            chain there) walks its entries' headers: counts and the checks of
//            readEntry; the block's aggregate is published, and the look-back
//            windows are requested at once
//   pass 2   the same walk writes per-KV metadata at final indices (key source
//            offset, shared and key length, prefix parent, key / value output
//            offsets, value source, entry offset, flags) while the look-back
//            loads are in flight; then the exclusive prefix is resolved
//   emit     lane per KV: trailer, flags, offsets; the user key as 16-B chunks
//            merged from its prefix chain's LDS segments; the value as 16-B
//            chunks read straight from LDS; every store is a plain (unaligned)
//            global store, exact at each key's and value's tail.  Values longer
//            than kLongVal are copied by the whole wave, 1 KiB per instruction.
//
// Per block that is a few hundred wave instructions for the outputs instead of
// thousands.  The wave is alone on its SIMD (4 x 38 KB of LDS per CU), so the
// loops keep independent work in flight rather than relying on other waves.
//
// (A first form read the block from global memory with 20 waves per CU and no
// stage: every dependent global round trip then cost ~3 us under load and a
// block took ~240 us; 655 GiB/s against the pipeline's 1034.)
//
// Blocks this path does not take (more than kFKv KVs or 2 x 64 runs, more than
// 64 KiB of user-key bytes, a restart table inconsistent with per-run walks, a
// value-prefix kind byte inside the shared prefix) take the wave-serial general
// walk (rowblk_general.hip.h); blocks past kMaxFastLen are sized and written by
// big_block_{sizes,values}_kernel around this launch.  Results are identical on
// every path.
//
// Semantics: cockroachdb/pebble sstable/rowblk/rowblk_iter.go — Init :241-276,
// readFirstKey :418-485, readEntry :333-416, decodeInternalKey :487-504, value
// prefix :1192-1199 (sstable/block/kv.go:14-41), decodeRestart :1092-1096.
#pragma once

namespace flat {

#ifndef PBL_FLAT_TICKET
// consecutive blocks per ticket.  Keep 1: a wave publishes its second block
// only after the first is fully written, so with 2 every ticket's first block
// waits on the previous ticket's completion and the whole batch serialises
// (measured 631 ms per launch against 1.9 ms)
#define PBL_FLAT_TICKET 1
#endif
#ifndef PBL_FLAT_VG
#define PBL_FLAT_VG 0  // 1: values by 8-lane groups (contiguous stores; measured 932 vs 978 GiB/s lane per KV)
#endif
#ifndef PBL_FLAT_LONG
#define PBL_FLAT_LONG 256  // values longer than this are copied by the whole wave
#endif

constexpr int kFW = 4;                   // waves per workgroup, one workgroup per CU
constexpr int kFTPB = kFW * kWave;
constexpr int kFKv = 320;                // KVs per block on this path
constexpr int kFRounds = 2;              // restart runs per lane (<= 128 runs)
constexpr uint32_t kFKeyCap = 65535;     // user-key bytes per block (u16 offsets)
constexpr uint32_t kLongVal = PBL_FLAT_LONG;

// One wave's block: the staged bytes and the per-KV metadata.  m0[j] = key
// source offset | shared << 16 | internal key length << 32 | prefix parent << 48.
struct WSlot {
  uint4 x[kLdsBlkBytes / 16];  // the block, byte i at kPad + (boff & 15) + i
  uint64_t m0[kFKv];
  uint32_t vp[kFKv + 1];       // value output offset | value source offset << 16
  uint16_t kout[kFKv + 1];     // user-key output offsets
  uint16_t eoff[kFKv];         // entry offsets (KVEncoding.Offset)
  uint8_t kvf[kFKv];           // PBL_KV_* (OBSOLETE is added at emit time)
};
struct FLds {
  WSlot w[kFW];
};
static_assert(sizeof(FLds) <= 163840, "four waves' slots per CU");

__device__ __forceinline__ uint32_t m_ksrc(uint64_t m) { return uint32_t(m) & 0xffffu; }
__device__ __forceinline__ uint32_t m_sh(uint64_t m) { return uint32_t(m >> 16) & 0xffffu; }
__device__ __forceinline__ uint32_t m_klen(uint64_t m) { return uint32_t(m >> 32) & 0xffffu; }
__device__ __forceinline__ uint32_t m_par(uint64_t m) { return uint32_t(m >> 48); }
__device__ __forceinline__ uint32_t f_vout(const WSlot& M, uint32_t j) { return M.vp[j] & 0xffffu; }
__device__ __forceinline__ uint32_t f_vsrc(const WSlot& M, uint32_t j) { return M.vp[j] >> 16; }

typedef u32x4 u32x4_ug __attribute__((aligned(1)));
typedef uint32_t u32_ug __attribute__((aligned(1)));
typedef uint64_t u64_ug __attribute__((aligned(1)));
typedef uint16_t u16_ug __attribute__((aligned(1)));

// Inclusive wave scan by DPP row shifts and row broadcasts (no ds_bpermute):
// Hillis-Steele inside each row of 16 lanes, then the last lane of rows 0/2
// into rows 1/3 (row_bcast:15), then of rows 0-1 into rows 2-3 (row_bcast:31).
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
// else the fewest 8/4/2/1-B stores (nothing past n: the next key or value
// belongs to another lane).
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

struct Acc {
  uint32_t cnt, kb, vb;
};

// Pass 1 over entries [pos, e0) of a run whose first `cnt` entries were
// already counted (prev_kl = the length of the last one): entry count and
// output bytes; `ok` clears where the run is not walkable per run, `bad` sets
// on shared > len(previous key) (rowblk_iter.go:403), `vbad` on a SET value
// without its prefix byte.
__device__ __forceinline__ void f_count_span(const View& V, uint32_t pos, uint32_t e0, uint32_t cnt, uint32_t prev_kl,
                                             uint32_t flags, bool vprefix, Acc& acc, bool& ok, bool& bad,
                                             bool& vbad) {
  const uint32_t cnt0 = cnt;
  while (pos < e0) {
    uint32_t sh, un, vl, h;
    const bool hok = pipe::hdr2(V.ld8(pos), &sh, &un, &vl, &h);
    const uint32_t np = pos + h + un + vl;
    if (!hok || (cnt == 0 && sh != 0) || np > e0) { ok = false; return; }
    bad = bad || (cnt > 0 && sh > prev_kl);
    const uint32_t kl = sh + un;
    uint32_t vlen = vl;
    if (vprefix && kl >= 8) {
      if (kl - 8 < sh) { ok = false; return; }  // kind byte inside the shared prefix
      if ((V.byte(pos + h + (kl - 8 - sh)) & 0xBF) == 1) {
        if (vl == 0) vbad = true;
        else if ((V.byte(pos + h + un) & 0xC0) == 0 || (flags & PBL_ROW_NO_VALUER)) vlen--;
      }
    }
    acc.kb += (flags & PBL_ROW_RAW_KEYS) ? kl : (kl >= 8 ? kl - 8 : 0);
    acc.vb += vlen;
    cnt++;
    prev_kl = kl;
    pos = np;
  }
  acc.cnt += cnt - cnt0;
}

__device__ __forceinline__ bool run_bounds(const View& V, uint32_t r, uint32_t nres, uint32_t roff, uint32_t* rw,
                                           uint32_t* e0) {
  const uint32_t st = roff + 4 * r;
  *rw = V.le32(st);
  const uint32_t s0 = *rw & kRestartMask;
  *e0 = (r + 1 < nres) ? (V.le32(st + 4) & kRestartMask) : roff;
  return (r != 0 || s0 == 0) && s0 < *e0 && *e0 <= roff;
}

// Pass 1 over run r, its first kPark entries' headers parked in registers
// (static indices, no scratch: a wave is alone on its SIMD, so registers are
// plentiful) for pass 2; a longer run counts its tail unparked.
constexpr int kPark = 32;
struct Park {
  uint32_t ea[kPark];  // entry offset | shared << 16
  uint32_t eb[kPark];  // unshared | header length << 14 | value length << 17
  uint32_t cnt, rw, pos, e0, prev_kl;
};

__device__ __forceinline__ void f_count_park(const View& V, uint32_t r, uint32_t nres, uint32_t roff, uint32_t flags,
                                             bool vprefix, Park& P, Acc& acc, bool& ok, bool& bad, bool& vbad) {
  P.cnt = 0;
  if (!run_bounds(V, r, nres, roff, &P.rw, &P.e0)) { ok = false; return; }
  const uint32_t e0 = P.e0;
  uint32_t pos = P.rw & kRestartMask, cnt = 0, prev_kl = 0;
  bool go = true;
#pragma unroll
  for (int k = 0; k < kPark; k++) {
    if (go && pos < e0) {
      uint32_t sh, un, vl, h;
      const bool hok = pipe::hdr2(V.ld8(pos), &sh, &un, &vl, &h);
      const uint32_t np = pos + h + un + vl;
      if (!hok || (k == 0 && sh != 0) || np > e0) {
        ok = false;
        go = false;
      } else {
        bad = bad || (k > 0 && sh > prev_kl);
        const uint32_t kl = sh + un;
        uint32_t vlen = vl;
        if (vprefix && kl >= 8) {
          if (kl - 8 < sh) { ok = false; go = false; }  // kind byte inside the shared prefix
          else if ((V.byte(pos + h + (kl - 8 - sh)) & 0xBF) == 1) {
            if (vl == 0) vbad = true;
            else if ((V.byte(pos + h + un) & 0xC0) == 0 || (flags & PBL_ROW_NO_VALUER)) vlen--;
          }
        }
        P.ea[k] = pos | (sh << 16);
        P.eb[k] = un | (h << 14) | (vl << 17);
        acc.kb += (flags & PBL_ROW_RAW_KEYS) ? kl : (kl >= 8 ? kl - 8 : 0);
        acc.vb += vlen;
        cnt++;
        prev_kl = kl;
        pos = np;
      }
    }
  }
  P.cnt = cnt;
  P.pos = pos;
  P.prev_kl = prev_kl;
  acc.cnt += cnt;
  if (go && pos < e0) f_count_span(V, pos, e0, cnt, prev_kl, flags, vprefix, acc, ok, bad, vbad);
}

// Pass 1 over run r without parking.
__device__ __forceinline__ void f_count_run(const View& V, uint32_t r, uint32_t nres, uint32_t roff, uint32_t flags,
                                            bool vprefix, Acc& acc, bool& ok, bool& bad, bool& vbad) {
  uint32_t rw, e0;
  if (!run_bounds(V, r, nres, roff, &rw, &e0)) { ok = false; return; }
  f_count_span(V, rw & kRestartMask, e0, 0, 0, flags, vprefix, acc, ok, bad, vbad);
}

// Chain state of pass 2 carried from one entry of a run to the next: output
// index / key / value offsets, the previous entry's shared length, its prefix
// parent and that parent's shared length.
struct WState {
  uint32_t j, kb, vb, prev_sh, pp, ppsh;
};

// Per-KV metadata of one entry (pass 2).
__device__ __forceinline__ void f_meta(WSlot& M, const View& V, uint32_t pos, uint32_t sh, uint32_t un, uint32_t vl,
                                       uint32_t h, bool first, uint32_t rw, uint32_t flags, bool vprefix, WState& S) {
  const uint32_t kl = sh + un;
  uint32_t vs = pos + h + un, vlen = vl;
  uint8_t fl = 0;
  if (first) fl = uint8_t(PBL_KV_RESTART | ((rw >> 31) ? PBL_KV_RESTART_SAMEPFX : 0));
  if (!(flags & PBL_ROW_RAW_KEYS) && kl < 8) fl |= PBL_KV_INVALID_KEY;
  if (vprefix && kl >= 8 && (V.byte(pos + h + (kl - 8 - sh)) & 0xBF) == 1) {
    const uint32_t pre = V.byte(vs);
    if ((pre & 0xC0) == 0 || (flags & PBL_ROW_NO_VALUER)) { vs++; vlen--; }
    else if ((pre & 0xC0) == 0x80) fl |= PBL_KV_VALBLK_HANDLE;
    else fl |= PBL_KV_BLOB_HANDLE;
  }
  // prefix parent: nearest earlier entry of the run with a smaller shared
  // length (all-nearest-smaller-values over the parents, amortised O(1)); the
  // previous entry and its parent are kept in registers
  uint32_t par = S.j, parsh = 0;
  if (sh != 0) {
    uint32_t c = S.j - 1, csh = S.prev_sh;
    if (csh >= sh) { c = S.pp; csh = S.ppsh; }
    while (csh >= sh) {
      c = m_par(M.m0[c]);
      csh = m_sh(M.m0[c]);
    }
    par = c;
    parsh = csh;
  }
  M.m0[S.j] = uint64_t(pos + h) | uint64_t(sh) << 16 | uint64_t(kl) << 32 | uint64_t(par) << 48;
  M.vp[S.j] = S.vb | (vs << 16);
  M.kout[S.j] = uint16_t(S.kb);
  M.eoff[S.j] = uint16_t(pos);
  M.kvf[S.j] = fl;
  S.prev_sh = sh;
  S.pp = par;
  S.ppsh = parsh;
  S.kb += (flags & PBL_ROW_RAW_KEYS) ? kl : (kl >= 8 ? kl - 8 : 0);
  S.vb += vlen;
  S.j++;
}

// Pass 2 over entries [pos, e0) of a run (validated by pass 1), re-read from LDS.
__device__ __forceinline__ void f_write_span(WSlot& M, const View& V, uint32_t pos, uint32_t e0, uint32_t rw,
                                             bool first, uint32_t flags, bool vprefix, WState& S) {
  while (pos < e0) {
    uint32_t sh, un, vl, h;
    pipe::hdr2(V.ld8(pos), &sh, &un, &vl, &h);
    f_meta(M, V, pos, sh, un, vl, h, first, rw, flags, vprefix, S);
    first = false;
    pos = pos + h + un + vl;
  }
}

// Pass 2 over run r (validated by pass 1): per-KV metadata at final indices
// from acc (the run's bases).
__device__ __forceinline__ void f_write_run(WSlot& M, const View& V, uint32_t r, uint32_t nres, uint32_t roff,
                                            uint32_t flags, bool vprefix, Acc acc) {
  uint32_t rw, e0;
  run_bounds(V, r, nres, roff, &rw, &e0);
  WState S{acc.cnt, acc.kb, acc.vb, 0, 0, 0};
  f_write_span(M, V, rw & kRestartMask, e0, rw, true, flags, vprefix, S);
}

// Pass 2 from the parked headers (then the unparked tail, if any).
__device__ __forceinline__ void f_write_park(WSlot& M, const View& V, const Park& P, uint32_t flags, bool vprefix,
                                             Acc acc) {
  WState S{acc.cnt, acc.kb, acc.vb, 0, 0, 0};
#pragma unroll
  for (int k = 0; k < kPark; k++) {
    if (uint32_t(k) < P.cnt)
      f_meta(M, V, P.ea[k] & 0xffffu, P.ea[k] >> 16, P.eb[k] & 0x3fffu, P.eb[k] >> 17, (P.eb[k] >> 14) & 7u, k == 0,
             P.rw, flags, vprefix, S);
  }
  if (P.pos < P.e0) f_write_span(M, V, P.pos, P.e0, P.rw, false, flags, vprefix, S);
}

// byte p of the internal key of KV j (source = max{i <= j : shared_i <= p})
__device__ __forceinline__ uint32_t f_key_byte(const WSlot& M, const View& V, int j, uint32_t p) {
  uint64_t m = M.m0[j];
  while (p < m_sh(m)) m = M.m0[--j];
  return V.byte(m_ksrc(m) + p - m_sh(m));
}

__device__ __forceinline__ uint64_t f_trailer(const WSlot& M, const View& V, int j, uint64_t m, uint8_t* fl,
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
    for (int i = 0; i < 8; i++) raw |= uint64_t(f_key_byte(M, V, j, kl - 8 + i)) << (8 * i);
  }
  if (raw & 64u) *fl |= PBL_KV_OBSOLETE;
  return raw & kTrailerObsoleteMask;
}

// Key bytes [c, c + n) of KV j (a chunk of <= 16 bytes, n > 0) merged from the
// segments of its prefix chain: each an LDS read that starts where the chunk's
// first byte would sit in that entry (at most 15 bytes before the block: the
// stage's front pad), masked to its part of the chunk.
__device__ __forceinline__ uint4 f_key_chunk(const WSlot& M, const View& V, uint64_t m, uint32_t c, uint32_t n) {
  const uint32_t ce = c + n;
  uint32_t cur = ce;  // bytes [c, cur) are still to be found
  uint4 w = make_uint4(0, 0, 0, 0);
  for (;;) {
    const uint32_t shi = m_sh(m);
    const uint32_t lo_i = shi < cur ? shi : cur;  // this entry supplies [max(sh, c), cur)
    const uint32_t a = lo_i > c ? lo_i : c;
    if (a < cur) {
      const uint4 v = V.ld16(int32_t(m_ksrc(m)) - int32_t(shi) + int32_t(c));
      if (a == c && cur - a == 16) return v;
      merge16(w, v, a - c, cur - c);
    }
    if (lo_i <= c) break;
    cur = lo_i;
    m = M.m0[m_par(m)];
  }
  return w;
}

// The block HBM -> LDS by LDS-DMA: granule g of the 16-B aligned source range
// lands at x[1 + g].  The caller waits vmcnt(0) before reading it.
__device__ __forceinline__ void f_stage(WSlot& M, const uint8_t* blocks, uint64_t boff, uint32_t blen) {
  const uint64_t a0 = boff & ~uint64_t(15), a1 = (boff + blen + 15) & ~uint64_t(15);
  const uint32_t n16 = uint32_t((a1 - a0) >> 4);
  const uint32_t l = lane_id();
  const gptr<const uint8_t> base = to_glb(blocks + a0);
  for (uint32_t g0 = 0; g0 < n16; g0 += kWave) {
    if (g0 + l < n16)  // (EXEC masks the lanes past the end: nothing lands past the stage)
      __builtin_amdgcn_global_load_lds((gptr<const void>)(base + 16ull * (g0 + l)),
                                       (lptr<void>)to_lds_ptr(reinterpret_cast<void*>(&M.x[1 + g0])), 16, 0, 0);
  }
}

// One block on one wave.
__device__ __forceinline__ void flat_block(WSlot& M, const Args& A, uint32_t b) {
  const int l = lane_id();
  const uint32_t nb = A.in.n_blocks, flags = A.in.flags;
  const uint64_t boff = to_glb(A.in.block_off)[b];
  const uint32_t blen = to_glb(A.in.block_len)[b];
  const bool fits = blen <= kMaxFastLen;
  const bool vprefix = (flags & PBL_ROW_VALUE_PREFIX) && !(flags & PBL_ROW_RAW_KEYS);
  uint8_t* ws = reinterpret_cast<uint8_t*>(A.out.workspace);
  uint64_t* lb_state = reinterpret_cast<uint64_t*>(ws + kWsHeader);
  const uint8_t* gblk = A.in.blocks + boff;

  if (!fits) {
    // a block past kMaxFastLen: big_block_sizes_kernel walked it, published its
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

  PSTAMP(A, b, 0, l == 0);
  f_stage(M, A.in.blocks, boff, blen);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  wave_sync();
  PSTAMP(A, b, 1, l == 0);
  const View V = lds_view(M.x, uint32_t(kPad + (boff & 15)));
  uint32_t roff, nres;
  uint32_t status = pipe::init_checks(LdsRd{V}, blen, flags, &roff, &nres);
  bool slow = status == PBL_OK && nres > uint32_t(kFRounds * kWave);
  uint32_t nkv = 0, tkb = 0, tvb = 0;
  Acc base[kFRounds];
  bool published = false;
  LbWindows<kLbWin> G;
  if (status == PBL_OK && !slow && roff > 0) {
    bool ok = true, bad = false, vbad = false;
    uint32_t c0 = 0, k0 = 0, v0 = 0;
    Park P;
    P.cnt = 0;
    P.pos = P.e0 = 0;
#pragma unroll
    for (int i = 0; i < kFRounds; i++) {
      Acc acc{0, 0, 0};
      const uint32_t r = uint32_t(l + kWave * i);
      if (i == 0) {
        if (r < nres) f_count_park(V, r, nres, roff, flags, vprefix, P, acc, ok, bad, vbad);
      } else if (uint32_t(kWave * i) < nres && r < nres) {
        f_count_run(V, r, nres, roff, flags, vprefix, acc, ok, bad, vbad);
      }
      const uint32_t ic = dpp_incl_scan(acc.cnt), ik = dpp_incl_scan(acc.kb), iv = dpp_incl_scan(acc.vb);
      base[i] = Acc{c0 + ic - acc.cnt, k0 + ik - acc.kb, v0 + iv - acc.vb};
      c0 += last_lane(ic);
      k0 += last_lane(ik);
      v0 += last_lane(iv);
    }
    nkv = c0;
    tkb = k0;
    tvb = v0;
    if (__ballot(bad)) status = PBL_CORRUPT_BOUNDS;
    else if (__ballot(!ok) || nkv > uint32_t(kFKv) || tkb > kFKeyCap) slow = true;
    else if (__ballot(vbad)) status = PBL_CORRUPT_BOUNDS;  // Go: i.val[0] on an empty SET value
    if (status == PBL_OK && !slow) {
      // the sizes are final: publish, request the look-back windows, and write
      // the metadata while they are in flight
      const uint64_t agg[kNumComp] = {nkv, tkb, tvb, nres};
      lb_publish(lb_state, nb, b, agg);
      published = true;
      PSTAMP(A, b, 2, l == 0);
      if (b > 0) G.issue(LbPtrs(lb_state, nb), int64_t(b) - 1);
      if (uint32_t(l) < nres) f_write_park(M, V, P, flags, vprefix, base[0]);
#pragma unroll
      for (int i = 1; i < kFRounds; i++) {
        const uint32_t r = uint32_t(l + kWave * i);
        if (uint32_t(kWave * i) < nres && r < nres) f_write_run(M, V, r, nres, roff, flags, vprefix, base[i]);
      }
      if (l == 0) {
        M.vp[nkv] = tvb;
        M.kout[nkv] = uint16_t(tkb);
      }
      wave_sync();
      PSTAMP(A, b, 3, l == 0);
    }
  }

  if (status == PBL_OK && slow) {
    // general path (wave-serial Iter.Next) on the staged block, the metadata
    // area as its key buffer; a key that outgrows it re-runs from global
    // memory with the whole staging buffer as the key buffer
    SlowState ss;
    uint64_t dummy[kNumComp] = {0, 0, 0, 0}, excl[kNumComp];
    const uint8_t* src = reinterpret_cast<const uint8_t*>(M.x) + kPad + (boff & 15);
    bool from_lds = true;
    uint8_t* keybuf = reinterpret_cast<uint8_t*>(M.m0);
    uint32_t keycap = uint32_t(sizeof(WSlot) - offsetof(WSlot, m0)) & ~15u;
    slow_walk(src, true, blen, flags, A.in.synthetic_seq_num, keybuf, keycap, kPassCount, A.out, b, dummy, &ss);
    if (ss.status == PBL_UNSUPPORTED) {
      from_lds = false;
      src = gblk;
      keybuf = reinterpret_cast<uint8_t*>(M.x);
      keycap = uint32_t(kLdsBlkBytes);
      slow_walk(src, false, blen, flags, A.in.synthetic_seq_num, keybuf, keycap, kPassCount, A.out, b, dummy, &ss);
    }
    const bool okk = ss.status == PBL_OK;
    const uint64_t agg[kNumComp] = {okk ? ss.nkv : 0, okk ? ss.kb : 0, okk ? ss.vb : 0, okk ? ss.nr : 0};
    lookback(lb_state, nb, b, agg, excl, &A.out.totals->status_mask);
    uint32_t st2 = ss.status;
    if (okk && overflows(A.out, excl, agg)) st2 = PBL_OVERFLOW;
    if (st2 == PBL_OK) slow_walk(src, from_lds, blen, flags, A.in.synthetic_seq_num, keybuf, keycap, kPassAll, A.out, b, excl, &ss);
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
  PSTAMP(A, b, 4, l == 0);
  if (okb && overflows(A.out, excl, agg)) status = PBL_OVERFLOW;
  if (l == 0) {
    if (status != PBL_OK && A.out.key_off && excl[0] + b < A.out.kv_cap + nb) {
      to_glb(A.out.key_off)[excl[0] + b] = 0;
      to_glb(A.out.val_off)[excl[0] + b] = 0;
    }
    write_block_meta(A.out, b, nb, status, excl, agg, false);
  }
  if (status != PBL_OK) return;
  if (nkv == 0) {  // a block with no entries: its lone N+1 offsets
    if (l == 0) {
      M.kout[0] = 0;
      M.vp[0] = 0;
    }
    wave_sync();
  }

  // ---- emit: lane per KV --------------------------------------------------
  const pbl_decode_out& O = A.out;
  const uint64_t kvb = excl[0], kbb = excl[1], vbb = excl[2], rbb = excl[3];
  const gptr<uint8_t> kbytes = to_glb(O.key_bytes) + kbb, vbytes = to_glb(O.val_bytes) + vbb;
  const bool raw = (flags & PBL_ROW_RAW_KEYS) != 0;
  for (uint32_t j0 = 0; j0 <= nkv; j0 += kWave) {
    const uint32_t j = j0 + l;
    uint32_t vlen = 0, vsrc = 0, vo = 0;
    if (j <= nkv) {
      const uint32_t ko = M.kout[j];
      vo = f_vout(M, j);
      to_glb(O.key_off)[kvb + b + j] = ko;
      to_glb(O.val_off)[kvb + b + j] = vo;
      if (j < nkv) {
        const uint64_t m = M.m0[j];
        uint8_t fl = M.kvf[j];
#ifndef PBL_FLAT_EXP_NOARR
        to_glb(O.trailer)[kvb + j] = with_seq(f_trailer(M, V, int(j), m, &fl, flags), A.in.synthetic_seq_num, flags);
        if (O.kv_flags) to_glb(O.kv_flags)[kvb + j] = fl;
        if (O.entry_off) to_glb(O.entry_off)[kvb + j] = M.eoff[j];
#else
        (void)fl;
#endif
        // user key: 16-B chunks of its prefix chain
        const uint32_t ukl = raw ? m_klen(m) : (m_klen(m) >= 8 ? m_klen(m) - 8 : 0u);
#ifndef PBL_FLAT_EXP_NOKEY
        for (uint32_t c = 0; c < ukl; c += 16) {
          const uint32_t n = ukl - c < 16 ? ukl - c : 16u;
          store_n(kbytes + ko + c, f_key_chunk(M, V, m, c, n), n);
        }
#else
        (void)ukl;
#endif
        // value: 16-B chunks straight from the stage (short values; long ones below)
        vsrc = f_vsrc(M, j);
        vlen = f_vout(M, j + 1) - vo;
#if !PBL_FLAT_VG && !defined(PBL_FLAT_EXP_NOVAL)
        if (vlen <= kLongVal) {
          // full 16-B chunks four at a time (their LDS reads together), then the tail
          const uint32_t nf = vlen & ~15u;
          for (uint32_t c = 0; c < nf; c += 64) {
            uint4 x[4];
#pragma unroll
            for (int u = 0; u < 4; u++)
              if (c + 16 * u < nf) x[u] = V.ld16(int32_t(vsrc + c + 16 * u));
#pragma unroll
            for (int u = 0; u < 4; u++)
              if (c + 16 * u < nf)
                *(gptr<u32x4_ug>)(vbytes + vo + c + 16 * u) = u32x4{x[u].x, x[u].y, x[u].z, x[u].w};
          }
          if (vlen & 15u) store_n(vbytes + vo + nf, V.ld16(int32_t(vsrc + nf)), vlen & 15u);
        }
#endif
      }
    }
#if PBL_FLAT_VG
    vlen = 0;  // (values are copied by the grouped loop below)
#endif
    // long values: the whole wave, 16 B per lane per step
    for (uint64_t lm = __ballot(j < nkv && vlen > kLongVal); lm; lm &= lm - 1) {
      const int s = __builtin_ctzll(lm);
      const uint32_t ls = __shfl(vsrc, s, kWave), ll = __shfl(vlen, s, kWave), lo = __shfl(vo, s, kWave);
      for (uint32_t c = 16u * l; c < ll; c += 16u * kWave) {
        const uint32_t n = ll - c < 16 ? ll - c : 16u;
        store_n(vbytes + lo + c, V.ld16(int32_t(ls + c)), n);
      }
    }
  }
#if PBL_FLAT_VG && !defined(PBL_FLAT_EXP_NOVAL)
  // values: 8 lanes per KV, lane k copying the KV's 16-B chunks k, k+8, ...;
  // a store instruction then writes 8 contiguous runs instead of 64 scattered
  // chunks.  Two groups' worth of KVs per lane step, their LDS reads together.
  {
    const uint32_t gk = uint32_t(l) & 7u, gi = uint32_t(l) >> 3;
    for (uint32_t j0 = 0; j0 < nkv; j0 += 16) {
      uint32_t vo2[2], vl2[2], vs2[2];
#pragma unroll
      for (int u = 0; u < 2; u++) {
        const uint32_t j = j0 + 8 * u + gi;
        const uint32_t a = j < nkv ? M.vp[j] : 0u, z = j < nkv ? M.vp[j + 1] : 0u;
        vo2[u] = a & 0xffffu;
        vl2[u] = (z & 0xffffu) - vo2[u];
        vs2[u] = a >> 16;
      }
#pragma unroll
      for (int u = 0; u < 2; u++) {
        for (uint32_t c = 16u * gk; c < vl2[u]; c += 128u) {
          const uint32_t n = vl2[u] - c < 16 ? vl2[u] - c : 16u;
          store_n(vbytes + vo2[u] + c, V.ld16(int32_t(vs2[u] + c)), n);
        }
      }
    }
  }
#endif
  if (O.restarts)
    for (uint32_t r = l; r < nres; r += kWave) to_glb(O.restarts)[rbb + r] = V.le32(roff + 4 * r);
  PSTAMP(A, b, 5, l == 0);
  wave_sync();  // (the slot is the next block's)
}

// The persistent kernel: one workgroup per CU, each wave an independent stream
// of tickets of PBL_FLAT_TICKET consecutive blocks, decoded in order.
// Deadlock-free for any residency: a block's look-back waits only on smaller
// tickets, all taken by resident waves that publish before they wait.
__global__ void __launch_bounds__(kFTPB, 1) rowblk_flat_kernel(Args A) {
  __shared__ FLds L;
  WSlot& M = L.w[wave_id()];
  const uint32_t nb = A.in.n_blocks;
  uint32_t* tick = reinterpret_cast<uint32_t*>(A.out.workspace);
  for (;;) {
    uint32_t t0 = 0;
    if (lane_id() == 0) t0 = g_atomic_add(tick, uint32_t(PBL_FLAT_TICKET));
    t0 = __builtin_amdgcn_readfirstlane(__shfl(t0, 0, kWave));
    if (t0 >= nb) break;
    const uint32_t t1 = nb - t0 < uint32_t(PBL_FLAT_TICKET) ? nb : t0 + uint32_t(PBL_FLAT_TICKET);
    for (uint32_t b = t0; b < t1; b++) flat_block(M, A, b);
  }
}

}  // namespace flat
