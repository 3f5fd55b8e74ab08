// rowblk_flat.hip.h — the row-format decode, one wave per block, with the block
// read from global memory instead of an LDS stage.
//
// Why: the LDS pipeline (rowblk_pipe.hip.h) stages every block in LDS for its
// whole life (parse + emit), so LDS caps it at 4 blocks in flight per CU, and
// each block is a ~30 K-cycle latency chain: 0.29 of HBM peak.  Here a wave
// owns a block end to end and keeps only its per-KV metadata in LDS (6.5 KB),
// so ~20 blocks are in flight per CU and the latency of each is hidden by the
// others:
//
//   prefetch   the whole block is pulled towards the CU with LDS-DMA loads into
//              a dump area that is never read (32 x 1 KB in flight: one HBM
//              round trip for the block instead of one per restart-run step)
//   pass 1     lane per restart run (rowblk_writer.go:147-155 cuts the prefix
//              chain there) walks its entries' headers from global memory (L2
//              hits after the prefetch): counts and the checks of readEntry;
//              the block's aggregate is published to the look-back at once
//   pass 2     the same walk again, writing per-KV metadata at final indices
//              (entry / key source offsets, shared and key lengths, the prefix
//              parent of each key, key and value output offsets, flags), then
//              128-B output bucket tables; then the exclusive prefix is resolved
//   emit       per-KV arrays, restart words, key bytes (each 16-B output
//              granule the merge of its keys' prefix-chain segments) and value
//              bytes (each 16-B output granule one or two unaligned global
//              loads), all 64 lanes, 16-B aligned stores
//
// Blocks this path does not take (more than kFKv KVs or 128 runs, more than
// 64 KiB of user-key bytes, a restart table inconsistent with per-run walks, a
// value-prefix kind byte inside the shared prefix) run the wave-serial general
// walk (rowblk_general.hip.h) with the wave's metadata area as its key buffer;
// blocks past kFMaxLen are sized and written by big_block_{sizes,values}_kernel
// around this launch, as for the pipeline.  Results are identical on every path.
//
// Semantics: cockroachdb/pebble sstable/rowblk/rowblk_iter.go — Init :241-276,
// readFirstKey :418-485, readEntry :333-416, decodeInternalKey :487-504, value
// prefix :1192-1199 (sstable/block/kv.go:14-41), decodeRestart :1092-1096.
#pragma once

namespace flat {

#ifndef PBL_FLAT_WAVES
#define PBL_FLAT_WAVES 4  // waves per workgroup (each an independent block stream)
#endif
#ifndef PBL_FLAT_WPE
#define PBL_FLAT_WPE 5  // waves per SIMD the registers are budgeted for
#endif
#ifndef PBL_FLAT_TICKET
#define PBL_FLAT_TICKET 2  // consecutive blocks per ticket (one atomic per ticket)
#endif
#ifndef PBL_FLAT_PF
#define PBL_FLAT_PF 1  // whole-block LDS-DMA prefetch
#endif
#ifndef PBL_FLAT_VU
#define PBL_FLAT_VU 4  // value granules per lane per emit step
#endif

constexpr int kFW = PBL_FLAT_WAVES;
constexpr int kFTPB = kFW * kWave;
constexpr int kFKv = 320;                // KVs per block on this path
constexpr int kFRounds = 2;              // restart runs per lane (<= 128 runs)
constexpr uint32_t kFMaxLen = 32768;     // block length (u16 offsets)
constexpr uint32_t kFKeyCap = 65535;     // user-key bytes per block (u16 offsets)
constexpr int kFKBs = 8, kFVBs = 7;      // output bucket sizes: keys 256 B, values 128 B
constexpr int kFKBkt = (kFKeyCap + 1) >> kFKBs;
constexpr int kFVBkt = kFMaxLen >> kFVBs;
constexpr int kFVU = PBL_FLAT_VU;

// One wave's parsed block.  m0[j] = key source offset | shared << 16 | internal
// key length << 32 | prefix parent << 48.
struct FMeta {
  uint64_t m0[kFKv];
  uint32_t vp[kFKv + 5];    // value output offset | value source offset << 16; [nkv, nkv+4]: the total
  uint16_t kout[kFKv + 1];  // user-key output offsets
  uint16_t eoff[kFKv];      // entry offsets (KVEncoding.Offset)
  uint16_t kbkt[kFKBkt];    // KV holding key output byte q << kFKBs
  uint16_t vbkt[kFVBkt];    // KV holding value output byte q << kFVBs
  uint8_t kvf[kFKv];        // PBL_KV_* (OBSOLETE is added at emit time)
};
struct FLds {
  FMeta m[kFW];
  u32x4 dump[kWave];  // LDS-DMA target of the block prefetch (never read)
};

__device__ __forceinline__ uint32_t m_ksrc(uint64_t m) { return uint32_t(m) & 0xffffu; }
__device__ __forceinline__ uint32_t m_sh(uint64_t m) { return uint32_t(m >> 16) & 0xffffu; }
__device__ __forceinline__ uint32_t m_klen(uint64_t m) { return uint32_t(m >> 32) & 0xffffu; }
__device__ __forceinline__ uint32_t m_par(uint64_t m) { return uint32_t(m >> 48); }

typedef u32x2 u32x2_ug __attribute__((aligned(1)));
typedef u32x4 u32x4_ug __attribute__((aligned(1)));
typedef uint32_t u32_ug __attribute__((aligned(1)));

// The block in global memory.  Bytes [0, rlim) are readable (the ABI's 16-B
// slack after every block); unaligned loads are used where they stay inside.
struct GView {
  gptr<const uint8_t> g;
  uint32_t rlim;
  __device__ __forceinline__ uint32_t byte(uint32_t i) const { return g[i]; }
  __device__ __forceinline__ uint32_t le32(uint32_t i) const { return *(gptr<const u32_ug>)(g + i); }
  __device__ __forceinline__ uint64_t ld8(uint32_t i) const {
    if (__builtin_expect(i + 8 <= rlim, 1)) {
      const u32x2 v = *(gptr<const u32x2_ug>)(g + i);
      return uint64_t(v.y) << 32 | v.x;
    }
    uint64_t r = 0;
    for (uint32_t k = 0; k < 8; k++)
      if (i + k < rlim) r |= uint64_t(g[i + k]) << (8 * k);
    return r;
  }
  // 16 bytes starting at block offset i (i < rlim)
  __device__ __forceinline__ uint4 ld16(uint32_t i) const {
    if (__builtin_expect(i + 16 <= rlim, 1)) {
      const u32x4 v = *(gptr<const u32x4_ug>)(g + i);
      return make_uint4(v.x, v.y, v.z, v.w);
    }
    const uint64_t a = uint64_t(g) + i, sa = a & ~uint64_t(15), end = uint64_t(g) + rlim;
    const uint32_t sh = uint32_t(a - sa);
    const u32x4 x = *(gptr<const u32x4>)(sa);
    u32x4 y = u32x4{0, 0, 0, 0};
    if (sh && sa + 16 < end) y = *(gptr<const u32x4>)(sa + 16);
    return sh ? col::funnel16(make_uint4(x.x, x.y, x.z, x.w), make_uint4(y.x, y.y, y.z, y.w), sh)
              : make_uint4(x.x, x.y, x.z, x.w);
  }
};
struct GRd {  // init_checks' reader
  GView V;
  __device__ uint32_t byte(uint32_t i) const { return V.byte(i); }
  __device__ uint32_t le32(uint32_t i) const { return V.le32(i); }
  __device__ uint32_t varint(uint32_t p, uint32_t end, uint32_t* v) const {
    return g_varint(reinterpret_cast<const uint8_t*>(V.g) + p, reinterpret_cast<const uint8_t*>(V.g) + end, v);
  }
};

// v placed at byte gq of a granule (bytes below gq zero)
__device__ __forceinline__ uint4 place16(const uint4& v, uint32_t gq) {
  return gq ? col::funnel16(make_uint4(0, 0, 0, 0), v, 16u - gq) : v;
}

struct Acc {
  uint32_t cnt, kb, vb;
};

// Pass 1 over run r: entry count and output bytes; `ok` clears where the run is
// not walkable per run, `bad` sets on shared > len(previous key)
// (rowblk_iter.go:403), `vbad` on a SET value without its prefix byte.
__device__ __forceinline__ void f_count_run(const GView& V, uint32_t r, uint32_t nres, uint32_t roff, uint32_t flags,
                                            bool vprefix, Acc& acc, bool& ok, bool& bad, bool& vbad) {
  const uint32_t st = roff + 4 * r;
  const uint32_t s0 = V.le32(st) & kRestartMask;
  const uint32_t e0 = (r + 1 < nres) ? (V.le32(st + 4) & kRestartMask) : roff;
  if (!((r != 0 || s0 == 0) && s0 < e0 && e0 <= roff)) { ok = false; return; }
  uint32_t pos = s0, cnt = 0, prev_kl = 0;
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
  acc.cnt += cnt;
}

// Pass 2 over run r (validated by pass 1): per-KV metadata at final indices
// acc.cnt.. (acc = the run's bases).
__device__ __forceinline__ void f_write_run(FMeta& M, const GView& V, uint32_t r, uint32_t nres, uint32_t roff,
                                            uint32_t flags, bool vprefix, Acc acc) {
  const uint32_t st = roff + 4 * r;
  const uint32_t rw = V.le32(st);
  const uint32_t e0 = (r + 1 < nres) ? (V.le32(st + 4) & kRestartMask) : roff;
  uint32_t pos = rw & kRestartMask;
  uint32_t j = acc.cnt, kb = acc.kb, vb = acc.vb;
  uint32_t prev_sh = 0, pp = 0, ppsh = 0;
  bool first = true;
  while (pos < e0) {
    uint32_t sh, un, vl, h;
    pipe::hdr2(V.ld8(pos), &sh, &un, &vl, &h);
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
    // length (all-nearest-smaller-values over the parents, amortised O(1));
    // the previous entry and its parent are kept in registers
    uint32_t par = j, parsh = 0;
    if (sh != 0) {
      uint32_t c = j - 1, csh = prev_sh;
      if (csh >= sh) { c = pp; csh = ppsh; }
      while (csh >= sh) {
        const uint64_t m = M.m0[c];
        c = m_par(m);
        csh = m_sh(M.m0[c]);
      }
      par = c;
      parsh = csh;
    }
    M.m0[j] = uint64_t(pos + h) | uint64_t(sh) << 16 | uint64_t(kl) << 32 | uint64_t(par) << 48;
    M.vp[j] = vb | (vs << 16);
    M.kout[j] = uint16_t(kb);
    M.eoff[j] = uint16_t(pos);
    M.kvf[j] = fl;
    prev_sh = sh;
    pp = par;
    ppsh = parsh;
    kb += (flags & PBL_ROW_RAW_KEYS) ? kl : (kl >= 8 ? kl - 8 : 0);
    vb += vlen;
    j++;
    first = false;
    pos = pos + h + un + vl;
  }
}

// byte p of the internal key of KV j (source = max{i <= j : shared_i <= p})
__device__ __forceinline__ uint32_t f_key_byte(const FMeta& M, const GView& V, int j, uint32_t p) {
  uint64_t m = M.m0[j];
  while (p < m_sh(m)) m = M.m0[--j];
  return V.byte(m_ksrc(m) + p - m_sh(m));
}

__device__ __forceinline__ uint64_t f_trailer(const FMeta& M, const GView& V, int j, uint8_t* fl, uint32_t flags) {
  if (flags & PBL_ROW_RAW_KEYS) return 0;
  const uint64_t m = M.m0[j];
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

// Merge user-key bytes [p_lo, p_hi) of KV j (user-key length ukl) into granule
// bytes [q, ...) of w: walk the prefix-parent chain, one global load per segment.
__device__ __forceinline__ void f_key_part(uint4& w, const FMeta& M, const GView& V, int j, uint32_t ukl,
                                           uint32_t p_lo, uint32_t p_hi, uint32_t q) {
  uint32_t cur = ukl;
  int i = j;
  while (cur > p_lo) {
    const uint64_t m = M.m0[i];
    const uint32_t shi = m_sh(m);
    const uint32_t lo_i = shi < cur ? shi : cur;
    const uint32_t a = lo_i > p_lo ? lo_i : p_lo, z = cur < p_hi ? cur : p_hi;
    if (a < z) {
      const uint32_t gq = q + (a - p_lo);
      const uint4 v = V.ld16(m_ksrc(m) - shi + a);
      if (gq == 0 && z - a == 16) w = v;
      else merge16(w, place16(v, gq), gq, gq + (z - a));
    }
    cur = lo_i;
    i = int(m_par(m));
  }
}

__device__ __forceinline__ uint32_t f_vout(const FMeta& M, uint32_t j) { return M.vp[j] & 0xffffu; }
__device__ __forceinline__ uint32_t f_vsrc(const FMeta& M, uint32_t j) { return M.vp[j] >> 16; }

// The whole block towards the CU: LDS-DMA loads of its 16-B granules into a
// dump area nobody reads.  Issued before the first header load, so the walk's
// loads then find their lines in L2.
__device__ __forceinline__ void f_prefetch(u32x4* dump, const uint8_t* blocks, uint64_t boff, uint32_t blen) {
#if PBL_FLAT_PF
  const uint64_t a0 = boff & ~uint64_t(15), a1 = (boff + blen + 15) & ~uint64_t(15);
  const uint32_t n16 = uint32_t((a1 - a0) >> 4);
  const uint32_t l = lane_id();
  const gptr<const uint8_t> base = to_glb(blocks + a0);
  lptr<void> d = (lptr<void>)to_lds_ptr(reinterpret_cast<void*>(dump));
  for (uint32_t g0 = 0; g0 < n16; g0 += kWave) {
    const uint32_t g = g0 + l < n16 ? g0 + l : n16 - 1;
    __builtin_amdgcn_global_load_lds((gptr<const void>)(base + 16ull * g), d, 16, 0, 0);
  }
#else
  (void)dump; (void)blocks; (void)boff; (void)blen;
#endif
}

// One block on one wave.
__device__ __noinline__ void flat_block(FMeta& M, u32x4* dump, const Args A, uint32_t b) {
  const int l = lane_id();
  const uint32_t nb = A.in.n_blocks, flags = A.in.flags;
  const uint64_t boff = to_glb(A.in.block_off)[b];
  const uint32_t blen = to_glb(A.in.block_len)[b];
  const bool fits = blen <= kFMaxLen;
  const bool vprefix = (flags & PBL_ROW_VALUE_PREFIX) && !(flags & PBL_ROW_RAW_KEYS);
  uint8_t* ws = reinterpret_cast<uint8_t*>(A.out.workspace);
  uint64_t* lb_state = reinterpret_cast<uint64_t*>(ws + kWsHeader);
  const uint8_t* gblk = A.in.blocks + boff;
  const GView V{to_glb(gblk), uint32_t(((boff + blen + 15) & ~uint64_t(15)) - boff)};

  if (!fits) {
    // a block past kFMaxLen: big_block_sizes_kernel walked it, published its
    // aggregate and left {status, counts} in its block-metadata slots;
    // big_block_values_kernel writes its outputs after this launch
    const uint32_t st0 = to_glb(A.out.blk_status)[b];
    const bool okk = st0 == PBL_OK;
    const uint64_t agg[kNumComp] = {okk ? to_glb(A.out.blk_kv_base)[b] : 0, okk ? to_glb(A.out.blk_key_base)[b] : 0,
                                    okk ? to_glb(A.out.blk_val_base)[b] : 0,
                                    okk ? uint64_t(V.le32(blen - 4)) : 0};
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

  f_prefetch(dump, A.in.blocks, boff, blen);
  uint32_t roff, nres;
  uint32_t status = pipe::init_checks(GRd{V}, blen, flags, &roff, &nres);
  bool slow = status == PBL_OK && nres > uint32_t(kFRounds * kWave);
  uint32_t nkv = 0, tkb = 0, tvb = 0;
  Acc base[kFRounds];
  bool published = false;
  if (status == PBL_OK && !slow && roff > 0) {
    bool ok = true, bad = false, vbad = false;
    uint32_t c0 = 0, k0 = 0, v0 = 0;
#pragma unroll
    for (int i = 0; i < kFRounds; i++) {
      Acc acc{0, 0, 0};
      const uint32_t r = uint32_t(l + kWave * i);
      if (uint32_t(kWave * i) < nres && r < nres) f_count_run(V, r, nres, roff, flags, vprefix, acc, ok, bad, vbad);
      const uint32_t ic = wave_incl_scan(acc.cnt), ik = wave_incl_scan(acc.kb), iv = wave_incl_scan(acc.vb);
      base[i] = Acc{c0 + ic - acc.cnt, k0 + ik - acc.kb, v0 + iv - acc.vb};
      c0 += pipe::wave_bcast_last(ic);
      k0 += pipe::wave_bcast_last(ik);
      v0 += pipe::wave_bcast_last(iv);
    }
    nkv = c0;
    tkb = k0;
    tvb = v0;
    if (__ballot(bad)) status = PBL_CORRUPT_BOUNDS;
    else if (__ballot(!ok) || nkv > uint32_t(kFKv) || tkb > kFKeyCap) slow = true;
    else if (__ballot(vbad)) status = PBL_CORRUPT_BOUNDS;  // Go: i.val[0] on an empty SET value
    if (status == PBL_OK && !slow) {
      // the sizes are final: publish before the write pass
      const uint64_t agg[kNumComp] = {nkv, tkb, tvb, nres};
      lb_publish(lb_state, nb, b, agg);
      published = true;
#pragma unroll
      for (int i = 0; i < kFRounds; i++) {
        const uint32_t r = uint32_t(l + kWave * i);
        if (uint32_t(kWave * i) < nres && r < nres) f_write_run(M, V, r, nres, roff, flags, vprefix, base[i]);
      }
      if (l < 5) M.vp[nkv + l] = tvb;
      if (l == 0) M.kout[nkv] = uint16_t(tkb);
      wave_sync();
      // output buckets: the KV holding byte q << kFKBs / q << kFVBs
      for (uint32_t j = l; j < nkv; j += kWave) {
        const uint32_t k0b = M.kout[j], k1b = M.kout[j + 1];
        for (uint32_t q = (k0b + (1u << kFKBs) - 1) >> kFKBs; (q << kFKBs) < k1b; q++) M.kbkt[q] = uint16_t(j);
        const uint32_t v0b = f_vout(M, j), v1b = f_vout(M, j + 1);
        for (uint32_t q = (v0b + (1u << kFVBs) - 1) >> kFVBs; (q << kFVBs) < v1b; q++) M.vbkt[q] = uint16_t(j);
      }
      wave_sync();
    }
  }

  if (status == PBL_OK && slow) {
    // general path: the wave-serial walk, the metadata area as its key buffer
    SlowState ss;
    uint64_t dummy[kNumComp] = {0, 0, 0, 0}, excl[kNumComp];
    uint8_t* keybuf = reinterpret_cast<uint8_t*>(&M);
    const uint32_t keycap = uint32_t(sizeof(FMeta)) & ~3u;
    slow_walk(gblk, false, blen, flags, keybuf, keycap, kPassCount, A.out, b, dummy, &ss);
    const bool okk = ss.status == PBL_OK;
    const uint64_t agg[kNumComp] = {okk ? ss.nkv : 0, okk ? ss.kb : 0, okk ? ss.vb : 0, okk ? ss.nr : 0};
    lookback(lb_state, nb, b, agg, excl, &A.out.totals->status_mask);
    uint32_t st2 = ss.status;
    if (okk && overflows(A.out, excl, agg)) st2 = PBL_OVERFLOW;
    if (st2 == PBL_OK) slow_walk(gblk, false, blen, flags, keybuf, keycap, kPassAll, A.out, b, excl, &ss);
    else if (l == 0 && A.out.key_off && excl[0] + b < A.out.kv_cap + nb) {
      to_glb(A.out.key_off)[excl[0] + b] = 0;
      to_glb(A.out.val_off)[excl[0] + b] = 0;
    }
    if (l == 0) write_block_meta(A.out, b, nb, st2, excl, agg, true);
    wave_sync();  // (the key buffer is the next block's metadata area)
    return;
  }

  const bool okb = status == PBL_OK;
  const uint64_t agg[kNumComp] = {okb ? nkv : 0, okb ? tkb : 0, okb ? tvb : 0, okb ? nres : 0};
  if (!published) lb_publish(lb_state, nb, b, agg);
  uint64_t excl[kNumComp];
  lb_resolve(lb_state, nb, b, agg, excl, &A.out.totals->status_mask);
  if (okb && overflows(A.out, excl, agg)) status = PBL_OVERFLOW;
  if (l == 0) {
    if (status != PBL_OK && A.out.key_off && excl[0] + b < A.out.kv_cap + nb) {
      to_glb(A.out.key_off)[excl[0] + b] = 0;
      to_glb(A.out.val_off)[excl[0] + b] = 0;
    }
    write_block_meta(A.out, b, nb, status, excl, agg, false);
  }
  if (status != PBL_OK) return;

  // ---- emit ---------------------------------------------------------------
  const pbl_decode_out& O = A.out;
  const uint64_t kvb = excl[0], kbb = excl[1], vbb = excl[2], rbb = excl[3];

  // value bytes: one 16-B aligned output granule per lane, kFVU per step with
  // their loads in flight together: (1) bucket -> first KV, (2) a 5-word window
  // of packed (vout | vsrc) words -> the KV holding the granule's first byte and
  // the next one, (3) one or two unaligned global loads, merged when the
  // granule straddles two values.  Granules touching 3+ values (values < 16 B)
  // or past the window take the general loop.
  if (tvb) {
    const uint64_t d0 = vbb, d1 = vbb + tvb;
    const gptr<uint8_t> vbytes = to_glb(O.val_bytes);
    for (uint64_t a = (d0 & ~uint64_t(15)) + 16 * uint64_t(l); a < d1; a += 16ull * kFVU * kWave) {
      uint4 w[kFVU], ga[kFVU], gb[kFVU];
      uint32_t lo[kFVU], hi[kFVU], o[kFVU], oe[kFVU], j0[kFVU], sa[kFVU], ea[kFVU], sb[kFVU], eb[kFVU];
      uint32_t srca[kFVU], srcb[kFVU];
      bool live[kFVU], gen[kFVU], two[kFVU];
#pragma unroll
      for (int u = 0; u < kFVU; u++) {
        const uint64_t g = a + uint64_t(u) * 16 * kWave;
        live[u] = g < d1;
        lo[u] = g < d0 ? uint32_t(d0 - g) : 0u;
        hi[u] = !live[u] ? 0u : (g + 16 <= d1 ? 16u : uint32_t(d1 - g));
        o[u] = live[u] ? uint32_t(g + lo[u] - d0) : 0u;
        oe[u] = live[u] ? uint32_t(g + hi[u] - d0) : 0u;
        j0[u] = M.vbkt[o[u] >> kFVBs];
      }
#pragma unroll
      for (int u = 0; u < kFVU; u++) {
        uint32_t vw[5];
#pragma unroll
        for (int k = 0; k < 5; k++) vw[k] = M.vp[j0[u] + k];
        const uint32_t q = o[u];
        const bool s1 = (vw[1] & 0xffff) <= q;
        const bool s2 = s1 && (vw[2] & 0xffff) <= q;
        const bool s3 = s2 && (vw[3] & 0xffff) <= q;
        const uint32_t k = uint32_t(s1) + uint32_t(s2) + uint32_t(s3);
        const uint32_t A0 = k == 0 ? vw[0] : k == 1 ? vw[1] : k == 2 ? vw[2] : vw[3];
        const uint32_t A1 = k == 0 ? vw[1] : k == 1 ? vw[2] : k == 2 ? vw[3] : vw[4];
        const uint32_t A2 = k == 0 ? vw[2] : k == 1 ? vw[3] : k == 2 ? vw[4] : vw[4];
        const uint32_t v0 = A0 & 0xffff, v1 = A1 & 0xffff, v2 = A2 & 0xffff;
        gen[u] = live[u] && ((s3 && (vw[4] & 0xffff) <= q) || (oe[u] > v1 && oe[u] > v2) || k == 3);
        sa[u] = q;
        ea[u] = oe[u] < v1 ? oe[u] : v1;
        sb[u] = v1;
        eb[u] = oe[u] < v2 ? oe[u] : v2;
        two[u] = live[u] && !gen[u] && oe[u] > v1;
        srca[u] = (A0 >> 16) + (sa[u] - v0);
        srcb[u] = A1 >> 16;
      }
#pragma unroll
      for (int u = 0; u < kFVU; u++) {
        if (live[u] && !gen[u]) ga[u] = V.ld16(srca[u]);
        if (two[u]) gb[u] = V.ld16(srcb[u]);
      }
#pragma unroll
      for (int u = 0; u < kFVU; u++) {
        if (!live[u]) continue;
        const uint64_t g = a + uint64_t(u) * 16 * kWave;
        if (!gen[u]) {
          const uint32_t gqa = uint32_t(d0 + sa[u] - g);
          if (gqa == 0 && ea[u] - sa[u] == 16) {
            w[u] = ga[u];
          } else {
            w[u] = make_uint4(0, 0, 0, 0);
            merge16(w[u], place16(ga[u], gqa), gqa, gqa + (ea[u] - sa[u]));
            if (two[u]) {
              const uint32_t gqb = gqa + (sb[u] - sa[u]);
              merge16(w[u], place16(gb[u], gqb), gqb, gqb + (eb[u] - sb[u]));
            }
          }
        } else {
          uint32_t j = j0[u];
          while (f_vout(M, j + 1) <= o[u]) j++;
          w[u] = make_uint4(0, 0, 0, 0);
          for (;;) {
            const uint32_t x0 = f_vout(M, j), x1 = f_vout(M, j + 1);
            const uint32_t s_ = o[u] > x0 ? o[u] : x0, e_ = oe[u] < x1 ? oe[u] : x1;
            if (s_ < e_) {
              const uint32_t gq = uint32_t(d0 + s_ - g);
              merge16(w[u], place16(V.ld16(f_vsrc(M, j) + (s_ - x0)), gq), gq, gq + (e_ - s_));
            }
            if (x1 >= oe[u]) break;
            j++;
          }
        }
        pipe::put16(vbytes, g, w[u], lo[u], hi[u]);
      }
    }
  }

  // per-KV arrays (thread per KV) and restart words
  {
    const gptr<uint32_t> key_off = to_glb(O.key_off), val_off = to_glb(O.val_off);
    const gptr<uint64_t> trailer = to_glb(O.trailer);
    for (uint32_t j = l; j <= nkv; j += kWave) {
      const uint64_t oi = kvb + b + j;
      key_off[oi] = M.kout[j];
      val_off[oi] = f_vout(M, j);
      if (j < nkv) {
        uint8_t fl = M.kvf[j];
        trailer[kvb + j] = f_trailer(M, V, int(j), &fl, flags);
        if (O.kv_flags) to_glb(O.kv_flags)[kvb + j] = fl;
        if (O.entry_off) to_glb(O.entry_off)[kvb + j] = M.eoff[j];
      }
    }
    if (O.restarts)
      for (uint32_t r = l; r < nres; r += kWave) to_glb(O.restarts)[rbb + r] = V.le32(roff + 4 * r);
  }

  // key bytes: one 16-B aligned output granule per lane; each the merge of the
  // segments of the 1-2 keys it overlaps (each key its prefix chain)
  if (tkb) {
    const uint64_t d0 = kbb, d1 = kbb + tkb;
    for (uint64_t a = (d0 & ~uint64_t(15)) + 16 * uint64_t(l); a < d1; a += 16 * kWave) {
      const uint32_t lo = a < d0 ? uint32_t(d0 - a) : 0u, hi = a + 16 <= d1 ? 16u : uint32_t(d1 - a);
      const uint32_t o = uint32_t(a + lo - d0), oe = uint32_t(a + hi - d0);
      uint32_t j = M.kbkt[o >> kFKBs];
      while (M.kout[j + 1] <= o) j++;
      uint4 w = make_uint4(0, 0, 0, 0);
      for (;;) {
        const uint32_t k0 = M.kout[j], k1 = M.kout[j + 1];
        const uint32_t s = o > k0 ? o : k0, e = oe < k1 ? oe : k1;
        if (s < e) f_key_part(w, M, V, int(j), k1 - k0, s - k0, e - k0, uint32_t(d0 + s - a));
        if (k1 >= oe) break;
        j++;
      }
      pipe::put16(to_glb(O.key_bytes), a, w, lo, hi);
    }
  }
  wave_sync();  // (the metadata area is the next block's)
}

// The persistent kernel: each wave takes tickets of PBL_FLAT_TICKET consecutive
// blocks and decodes them in order.  Deadlock-free for any residency: a block's
// look-back waits only on smaller tickets, all taken by resident waves that
// publish before they wait.
__global__ void __launch_bounds__(kFTPB) __attribute__((amdgpu_waves_per_eu(PBL_FLAT_WPE)))
rowblk_flat_kernel(Args A) {
  __shared__ FLds L;
  FMeta& M = L.m[wave_id()];
  const uint32_t nb = A.in.n_blocks;
  uint32_t* tick = reinterpret_cast<uint32_t*>(A.out.workspace);
  for (;;) {
    uint32_t t0 = 0;
    if (lane_id() == 0) t0 = g_atomic_add(tick, uint32_t(PBL_FLAT_TICKET));
    t0 = __builtin_amdgcn_readfirstlane(__shfl(t0, 0, kWave));
    if (t0 >= nb) break;
    const uint32_t t1 = nb - t0 < uint32_t(PBL_FLAT_TICKET) ? nb : t0 + uint32_t(PBL_FLAT_TICKET);
    for (uint32_t b = t0; b < t1; b++) flat_block(M, L.dump, A, b);
  }
}

}  // namespace flat
