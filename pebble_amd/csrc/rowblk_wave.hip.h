// rowblk_wave.hip.h — row batches of variable-length blocks (PBL_BATCH_VARLEN:
// config 5's Zipf-sized KVs) in two passes, no look-back:
//
//   sizes   row_wave_size_kernel: LANE per block.  Each lane walks its block's
//           entry headers in global memory (one 16-B window per entry, the
//           three varints from registers) and leaves {status, KVs, user-key
//           bytes, value bytes} in blk_status / blk_{kv,key,val}_base[b] and
//           the restart count at ws_rcnt_offset.  A Zipf block holds ~8-13
//           entries, so a wave sizes 64 blocks in ~13 dependent round trips
//           and touches only the header lines (about 1/10 of the bytes).
//   scan    bases_scan_kernel<true> (colblk_wave.hip.h): the four components'
//           exclusive scan in place, totals at [n].
//   emit    row_wave_emit_kernel: one wave per block (four per CU), its bases
//           final.  The block by LDS-DMA into the wave's stage, the pool
//           kernel's lane-per-run walk and metadata pass into the wave's slot,
//           then every output from LDS: keys lane per KV, the values (97 % of
//           a Zipf block's bytes) LDS -> HBM in 16-B chunks, so a block is read
//           once.  Blocks off that form take the general walk (below).
//
// Against the staging-pool kernel (rowblk_pool.hip.h) on config 5: no look-back
// (16 K of its 95 K cycles per block), no second read of the values from
// L2 / HBM after the stage is released (1.56x traffic), no per-value round
// trips of the global->global copies.  Fixed-size batches (config 2: 271 KVs
// per block) stay on the pool kernel: there the lane walk would be 271 round
// trips deep and the wave-serial emit 271 entries long.
//
// Results are the general walk's: the size walk applies slow_walk_t's checks
// in slow_walk_t's order (rowblk_general.hip.h; Iter.Init rowblk_iter.go:
// 241-276, readEntry :333-416, the key-buffer limit of the general path); the
// emit's lane-parallel form is taken only where its walk agrees with those
// sizes, else the emit IS slow_walk_t.  (The wave-serial walk alone measured
// 2.87 ms on config 5 RI 16: ~6.9 K cycles per entry of dependent LDS steps.)  Flags that need a key's bytes
// to size it (HideObsoletePoints, value prefixes, on internal keys) take the
// pool kernel.
#pragma once

namespace rwave {

#ifndef PBL_RW_VALU
#define PBL_RW_VALU 4  // value granules per lane in flight, LDS -> HBM
#endif

// the general walk's key limit with the whole stage as its key buffer
constexpr uint64_t kKeyCapMax = uint64_t(kLdsBlkBytes) - kKeyBufSlack;

// Whether a batch's flags let the size pass count without key bytes.
__host__ __device__ inline bool sizes_without_keys(uint32_t flags) {
  return (flags & PBL_ROW_RAW_KEYS) || !(flags & (PBL_ROW_HIDE_OBSOLETE | PBL_ROW_VALUE_PREFIX));
}

// ---- the size pass: lane per block -------------------------------------------
// A lane walks its block's first kDenseProbe entries; a block that, at that
// pace, would hold more than 2 kEntRec entries in at least eight restart runs is
// DENSE (config-2-shaped: 271 entries, a 271-deep chain of round trips for one
// lane): it is listed for
// row_wave_dense_kernel, which sizes it lane per restart run, and its entry
// records are marked absent (entry 0 recorded as 0xffff).  Which kernel sizes
// a block changes only the speed: both give the general walk's sizes.
constexpr uint32_t kDenseProbe = 16;
__device__ __forceinline__ void put_sizes(const pbl_decode_out& O, gptr<uint64_t> rcnt, uint64_t b, uint32_t status,
                                          uint64_t nkv, uint64_t kb, uint64_t vb, uint32_t nres) {
  const bool ok = status == PBL_OK;
  to_glb(O.blk_kv_base)[b] = ok ? nkv : 0;
  to_glb(O.blk_key_base)[b] = ok ? kb : 0;
  to_glb(O.blk_val_base)[b] = ok ? vb : 0;
  rcnt[b] = ok ? nres : 0;
  to_glb(O.blk_status)[b] = status;
}

// slow_walk_t's loop from block offset `off` (entries before it counted into
// nkv / kb / vb, `full` the last key's length), its checks in its order,
// without the key bytes; at most `limit` entries (then *more is set).
__device__ __forceinline__ uint32_t seq_count(const SlowGlb& S, uint32_t blen, uint32_t roff, bool raw, uint64_t& off,
                                              uint64_t& full, uint64_t& nkv, uint64_t& kb, uint64_t& vb,
                                              uint32_t limit, bool* more, gptr<uint16_t> rec) {
  uint32_t n = 0;
  *more = false;
  while (off < roff) {
    if (n == limit) { *more = true; return PBL_OK; }
    const uint4 hw = S.ld16(int64_t(off));
    const uint32_t hn = uint32_t(min<uint64_t>(15, uint64_t(blen) - off));
    uint32_t shared, unshared, vlen;
    const uint32_t a = w_varint(hw, 0, hn, &shared);
    const uint32_t bb = a ? w_varint(hw, a, hn, &unshared) : 0;
    const uint32_t c = bb ? w_varint(hw, a + bb, hn, &vlen) : 0;
    if (!c) return PBL_CORRUPT_BOUNDS;
    const uint64_t kp = off + a + bb + c;
    if (blen - kp < unshared) return PBL_CORRUPT_BOUNDS;
    const uint64_t vp = kp + unshared;
    if (blen - vp < vlen) return PBL_CORRUPT_BOUNDS;
    if (shared > full) return PBL_CORRUPT_BOUNDS;
    const uint64_t klen = uint64_t(shared) + unshared;
    if (klen > kKeyCapMax) return PBL_UNSUPPORTED;
    full = klen;
    if (rec && nkv < kEntRec) rec[nkv] = uint16_t(off);  // (for the emit)
    nkv++;
    n++;
    kb += raw ? klen : (klen >= 8 ? klen - 8 : 0);
    vb += vlen;
    off = vp + vlen;
  }
  return (kb >> 32 || vb >> 32) ? PBL_UNSUPPORTED : PBL_OK;
}

__global__ void __launch_bounds__(kWave) row_wave_size_kernel(Args A) {
  const uint32_t nb = A.in.n_blocks, flags = A.in.flags;
  const pbl_decode_out& O = A.out;
  const bool raw = (flags & PBL_ROW_RAW_KEYS) != 0;
  uint8_t* ws = reinterpret_cast<uint8_t*>(O.workspace);
  const gptr<uint64_t> rcnt = to_glb(reinterpret_cast<uint64_t*>(ws + ws_rcnt_offset(nb)));
  const gptr<uint16_t> rec = to_glb(reinterpret_cast<uint16_t*>(ws + ws_ent_offset(nb)));
  uint32_t* hdr = reinterpret_cast<uint32_t*>(ws);
  const gptr<uint32_t> dense_ids = to_glb(reinterpret_cast<uint32_t*>(ws + ws_redo_offset(nb)));
  for (uint64_t b0 = uint64_t(blockIdx.x) * kWave; b0 < nb; b0 += uint64_t(gridDim.x) * kWave) {
    const uint64_t b = b0 + lane_id();
    bool dense = false;
    if (b < nb) {
      const uint32_t blen = to_glb(A.in.block_len)[b];
      const uint8_t* g = A.in.blocks + to_glb(A.in.block_off)[b];
      uint32_t roff, nres;
      uint32_t status = rowc::init_checks(GlbRd{g}, blen, flags, &roff, &nres);
      uint64_t nkv = 0, kb = 0, vb = 0;
      if (status == PBL_OK) {
        const SlowGlb S{to_glb(g), blen};
        const gptr<uint16_t> r = blen <= kMaxFastLen ? rec + b * kEntRec : gptr<uint16_t>(nullptr);
        uint64_t off = 0, full = 0;
        bool more = false;
        status = seq_count(S, blen, roff, raw, off, full, nkv, kb, vb, kDenseProbe, &more, r);
        if (status == PBL_OK && more) {
          // at this pace more than 2 kEntRec entries, in at least eight
          // restart runs to walk side by side (config 5 RI 16 with the
          // threshold at kEntRec entries and four runs: 1558 -> 1480 GiB/s,
          // its long-run blocks walked lane per run and emitted without
          // their entry records)
          dense = nres >= 8 && uint64_t(roff) * kDenseProbe > off * (2 * kEntRec);
          if (dense) {
            if (r) r[0] = 0xffffu;
          } else {
            status = seq_count(S, blen, roff, raw, off, full, nkv, kb, vb, ~0u, &more, r);
          }
        }
      }
      if (!dense) put_sizes(O, rcnt, b, status, nkv, kb, vb, nres);
    }
    // the dense blocks' ids, one atomic per wave
    const uint64_t m = __ballot(dense);
    if (m) {
      uint32_t base = 0;
      if (lane_id() == 0) base = g_atomic_add(hdr + rowc::kWsBigRedo, uint32_t(__popcll(m)));
      base = __shfl(base, 0, kWave);
      if (dense) dense_ids[base + __popcll(m & ((1ull << lane_id()) - 1))] = uint32_t(b);
    }
  }
}

// Dense blocks: a wave per block, lane per restart run, each run walked from
// global memory (the pool kernel's per-run rules: runs_bounds, a restart entry
// with shared 0, each run ending at the next run's start).  Where the runs tile
// the entries exactly and every entry is clean, the per-run sums ARE the
// sequential walk's; any other block is counted by seq_count (lane 0).
__global__ void __launch_bounds__(kWave) row_wave_dense_kernel(Args A) {
  const uint32_t nb = A.in.n_blocks, flags = A.in.flags;
  const pbl_decode_out& O = A.out;
  const bool raw = (flags & PBL_ROW_RAW_KEYS) != 0;
  const int l = lane_id();
  uint8_t* ws = reinterpret_cast<uint8_t*>(O.workspace);
  const gptr<uint64_t> rcnt = to_glb(reinterpret_cast<uint64_t*>(ws + ws_rcnt_offset(nb)));
  const uint32_t* hdr = reinterpret_cast<const uint32_t*>(ws);
  const uint32_t n = __hip_atomic_load(to_glb(hdr) + rowc::kWsBigRedo, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const gptr<const uint32_t> dense_ids = to_glb(reinterpret_cast<const uint32_t*>(ws + ws_redo_offset(nb)));
  for (uint32_t i = blockIdx.x; i < n; i += gridDim.x) {
    const uint32_t b = dense_ids[i];
    const uint32_t blen = to_glb(A.in.block_len)[b];
    const uint8_t* g = A.in.blocks + to_glb(A.in.block_off)[b];
    const SlowGlb S{to_glb(g), blen};
    const uint32_t nres = S.le32(blen - 4), roff = blen - 4u * (1u + nres);  // (the size pass checked them)
    uint64_t nkv = 0, kb = 0, vb = 0;
    bool ok = true;
    for (uint32_t r = l; r < nres && ok; r += kWave) {
      const uint32_t s0 = S.le32(roff + 4ull * r) & kRestartMask;
      const uint32_t e0 = r + 1 < nres ? (S.le32(roff + 4ull * r + 4) & kRestartMask) : roff;
      if (!((r != 0 || s0 == 0) && s0 < e0 && e0 <= roff)) { ok = false; break; }
      uint64_t off = s0, prev = 0;
      bool first = true;
      while (off < e0) {
        const uint4 hw = S.ld16(int64_t(off));
        const uint32_t hn = uint32_t(min<uint64_t>(15, uint64_t(blen) - off));
        uint32_t shared, unshared, vlen;
        const uint32_t a = w_varint(hw, 0, hn, &shared);
        const uint32_t bb = a ? w_varint(hw, a, hn, &unshared) : 0;
        const uint32_t c = bb ? w_varint(hw, a + bb, hn, &vlen) : 0;
        const uint64_t np = off + a + bb + c + unshared + vlen;
        const uint64_t klen = uint64_t(shared) + unshared;
        if (!c || np > e0 || (first ? shared != 0 : shared > prev) || klen > kKeyCapMax) { ok = false; break; }
        nkv++;
        kb += raw ? klen : (klen >= 8 ? klen - 8 : 0);
        vb += vlen;
        prev = klen;
        first = false;
        off = np;
      }
    }
    ok = !__ballot(!ok);
    nkv = wave_sum(nkv);
    kb = wave_sum(kb);
    vb = wave_sum(vb);
    uint32_t status = PBL_OK;
    if (!ok || kb >> 32 || vb >> 32) {
      uint64_t off = 0, full = 0;
      bool more;
      nkv = kb = vb = 0;
      status = seq_count(S, blen, roff, raw, off, full, nkv, kb, vb, ~0u, &more, gptr<uint16_t>(nullptr));
    }
    if (l == 0) put_sizes(O, rcnt, b, status, nkv, kb, vb, nres);
  }
}

// ---- the emit pass: wave per block -------------------------------------------
// The block staged, then the staging-pool kernel's lane-per-run walk and its
// metadata pass (rowblk_pool.hip.h: run_walk / count_span, park_meta /
// span_meta into the wave's slot), then the outputs: keys and per-KV arrays
// lane per KV (key_load / key_store with the stage as the key source), values
// from the stage.  A block off that form (not walkable per run, more entries
// than a slot holds, an empty or failing block, sizes that disagree with the
// size pass) takes the wave-serial general walk on the stage with the slot as
// its key buffer; a key past the slot, or a block past the stage, walks global
// memory with the stage as the key buffer (as block_slow does).
#ifndef PBL_RW_FAST
#define PBL_RW_FAST 1  // 0: every block on the general walk (A/B)
#endif
#ifndef PBL_RW_PAR
#define PBL_RW_PAR 1  // 0: every block through the serial per-run walk (A/B)
#endif
struct ELds {
  pool::Stage st;
  pool::Slot<false> sl;
};
static_assert(4 * sizeof(ELds) <= 163840, "four emit waves per CU");

// Walk and describe the staged block into slot W; false if the block is off
// the lane-parallel form.
__device__ __forceinline__ bool front_fast(const View& V, uint32_t blen, uint32_t flags, pool::Slot<false>& W,
                                           const uint64_t agg[kNumComp], uint32_t* roff_o) {
  using namespace pool;
  const int l = lane_id();
  constexpr uint32_t kKv = uint32_t(Slot<false>::kKv);
  const bool vprefix = (flags & PBL_ROW_VALUE_PREFIX) && !(flags & PBL_ROW_RAW_KEYS);
  uint32_t roff, nres;
  if (rowc::init_checks(LdsRd{V}, blen, flags, &roff, &nres) != PBL_OK || roff == 0 || nres > kKv) return false;
  // lane l owns runs [r0, r1)
  const uint32_t R = (nres + kWave - 1) / kWave;
  const uint32_t r0 = min(uint32_t(l) * R, nres), r1 = min(r0 + R, nres);
  PAcc acc{0, 0, 0, 0};
  bool ok = true, bad = false, vbad = false, over = false;
  PRun RB;
  RB.n = 0;
  RB.pos = RB.e0 = RB.prev_kl = RB.prev_kind = RB.rw = 0;
  const bool single = R == 1;
  if (single) {
    if (r0 < nres) run_walk<false>(V, r0, nres, roff, flags, vprefix, RB, acc, ok, bad, vbad, over);
    if (over && ok)
      count_span<false>(V, RB.pos, RB.e0, RB.n, RB.prev_kl, RB.prev_kind, flags, vprefix, acc, ok, bad, vbad);
  } else {
    for (uint32_t r = r0; r < r1 && ok; r++) {
      uint32_t rw, e0;
      if (!run_bounds(V, r, nres, roff, &rw, &e0)) ok = false;
      else count_span<false>(V, rw & kRestartMask, e0, 0, 0, 0, flags, vprefix, acc, ok, bad, vbad);
    }
  }
  const uint32_t ic = dpp_incl_scan(acc.cnt), ik = dpp_incl_scan(acc.kb), iv = dpp_incl_scan(acc.vb);
  const uint32_t nkv = last_lane(ic), tkb = last_lane(ik), tvb = last_lane(iv);
  if (__ballot(bad || vbad || !ok) || nkv > kKv) return false;
  if (nkv != agg[0] || tkb != agg[1] || tvb != agg[2] || nres != agg[3]) return false;
  MState M{ic - acc.cnt, ic - acc.cnt, iv - acc.vb, 0, 0, 0};
  if (single) {
    if (r0 < nres) {
      park_meta<false>(W, V, RB, flags, M);
      if (over) span_meta<false>(W, V, RB.pos, RB.e0, RB.rw, RB.n, RB.prev_kl, RB.prev_kind, flags, vprefix, M);
    }
  } else {
    for (uint32_t r = r0; r < r1; r++) {
      uint32_t rw, e0;
      run_bounds(V, r, nres, roff, &rw, &e0);
      M.prev_sh = M.pp = M.ppsh = 0;
      span_meta<false>(W, V, rw & kRestartMask, e0, rw, 0, 0, 0, flags, vprefix, M);
    }
  }
  if (l < 5) W.vp[nkv + l] = tvb;
  *roff_o = roff;
  return true;
}

// The same description without the serial walk, for a block of at most
// kEntRec KVs: lane i takes entry i at the offset the size pass recorded
// (pos), decodes its header from the stage, and the wave derives the rest --
// value output offsets by a scan, the prefix parent (nearest earlier entry
// with a smaller shared length, entry_meta's chain) by one pass over the
// lanes, restart flags by a binary search of the restart table.  That search
// is slow_walk_t's restart pointer only for a strictly increasing table, so
// any other table (and any entry off the fast form's limits) returns false.
__device__ __forceinline__ bool front_par(const View& V, uint32_t blen, uint32_t flags, pool::Slot<false>& W,
                                          const uint64_t agg[kNumComp], uint32_t pos, uint32_t* roff_o) {
  using namespace pool;
  const int l = lane_id();
  const uint32_t nkv = uint32_t(agg[0]), nres = uint32_t(agg[3]);
  const uint32_t roff = blen - 4u * (1u + nres);  // (the size pass checked the table)
  const bool raw = (flags & PBL_ROW_RAW_KEYS) != 0;
  const bool me = uint32_t(l) < nkv;
  uint32_t sh = 0, un = 0, vl = 0, h = 0;
  bool ok = true;
  if (me) {
    ok = (l != 0 || pos == 0) && rowc::hdr2(V.ld8(pos), &sh, &un, &vl, &h) && sh + un <= kMaxKl && h <= 15;
    const uint32_t nxt = __shfl(pos, l + 1 < kWave ? l + 1 : l, kWave);
    ok = ok && pos + h + un + vl == (uint32_t(l) + 1 < nkv ? nxt : roff);
  }
  // the restart table strictly increasing (masked words)
  bool inc = true;
  for (uint32_t r = l; r + 1 < nres; r += kWave)
    inc = inc && (V.le32(roff + 4 * r) & kRestartMask) < (V.le32(roff + 4 * r + 4) & kRestartMask);
  if (__ballot(!ok || !inc)) return false;
  const uint32_t kl = sh + un;
  // prefix parent: the last lane t < l with sh_t < sh (itself when sh == 0)
  uint32_t par = uint32_t(l);
  for (uint32_t t = 0; t + 1 < nkv; t++) {
    const uint32_t sht = __builtin_amdgcn_readlane(sh, t);
    if (sh != 0 && t < uint32_t(l) && sht < sh) par = t;
  }
  // restart flags: offset pos in the table
  uint32_t fl = 0;
  if (me) {
    uint32_t lo = 0, hi = nres;
    while (lo < hi) {
      const uint32_t mid = (lo + hi) >> 1;
      if ((V.le32(roff + 4 * mid) & kRestartMask) < pos) lo = mid + 1;
      else hi = mid;
    }
    if (lo < nres) {
      const uint32_t rw = V.le32(roff + 4 * lo);
      if ((rw & kRestartMask) == pos) fl = PBL_KV_RESTART | ((rw >> 31) ? PBL_KV_RESTART_SAMEPFX : 0u);
    }
    if (!raw && kl < 8) fl |= PBL_KV_INVALID_KEY;
  }
  const uint32_t incl = dpp_incl_scan(me ? vl : 0u);
  if (me) {
    W.m0[l] = m_pack(pos + h, sh, kl, par, h, fl);
    W.vp[l] = (incl - vl) | ((pos + h + un) << 16);
  }
  if (l < 5) W.vp[nkv + l] = uint32_t(agg[2]);
  *roff_o = roff;
  return true;
}

// Values of the slot's KVs from the stage: values of at most 128 B 8 lanes per
// KV (8 KVs per pass), longer ones by the whole wave, four 16-B chunks per lane
// in flight; a value's last chunk ENDS at its end (overlapping the one before),
// so every store is a whole unaligned 16-B store of its own value's bytes.
__device__ __forceinline__ void values_from_stage(const uint32_t* vp, const View& V, uint32_t nkv,
                                                  gptr<uint8_t> vbytes) {
  using pool::st_out;
  const int l = lane_id();
  const uint32_t c = uint32_t(l) & 7u;
  for (uint32_t j0 = 0; j0 < nkv; j0 += 8) {
    const uint32_t j = j0 + (uint32_t(l) >> 3);
    const uint32_t a = j < nkv ? vp[j] : 0u, z = j < nkv ? vp[j + 1] : 0u;
    const uint32_t vo = a & 0xffffu, vl = (z & 0xffffu) - vo, vs = a >> 16;
    if (j >= nkv || vl > 128) continue;
    if (vl >= 16) {
      if (16 * c < vl) {
        const uint32_t q = 16 * c < vl - 16 ? 16 * c : vl - 16;
        const uint4 w = V.ld16(int32_t(vs + q));
        st_out((gptr<pool::u32x4_ug>)(vbytes + vo + q), pool::u32x4_ug{w.x, w.y, w.z, w.w});
      }
    } else {
      for (uint32_t o = c; o < vl; o += 8) vbytes[vo + o] = uint8_t(V.byte(vs + o));
    }
  }
  for (uint32_t j0 = 0; j0 < nkv; j0 += kWave) {
    const uint32_t j = j0 + uint32_t(l);
    const uint32_t a = j < nkv ? vp[j] : 0u, z = j < nkv ? vp[j + 1] : 0u;
    const uint32_t len = (z & 0xffffu) - (a & 0xffffu);
    for (uint64_t lm = __ballot(j < nkv && len > 128); lm; lm &= lm - 1) {
      const int sl = __builtin_ctzll(lm);
      const uint32_t vs = __shfl(a >> 16, sl, kWave), vl = __shfl(len, sl, kWave), vo = __shfl(a & 0xffffu, sl, kWave);
      for (uint32_t o0 = 16u * l; o0 < vl; o0 += 64u * kWave) {
        uint4 y[4];
#pragma unroll
        for (int k = 0; k < 4; k++) {
          const uint32_t o = o0 + 16u * kWave * k, q = o < vl - 16 ? o : vl - 16;
          y[k] = V.ld16(int32_t(vs + (o < vl ? q : 0u)));
        }
#pragma unroll
        for (int k = 0; k < 4; k++) {
          const uint32_t o = o0 + 16u * kWave * k, q = o < vl - 16 ? o : vl - 16;
          if (o < vl) st_out((gptr<pool::u32x4_ug>)(vbytes + vo + q), pool::u32x4_ug{y[k].x, y[k].y, y[k].z, y[k].w});
        }
      }
    }
  }
}

// The keys, per-KV arrays and restart words of a block front_par / front_fast
// described, at bases excl.  kPart: key_store's (0 all; 1 all but the long
// keys' own bytes; 2 those and the restart words).
template <int kPart>
__device__ __forceinline__ void emit_keys(const Args& A, uint32_t b, const View& V, const pool::Slot<false>& W,
                                          uint32_t roff, const uint64_t excl[kNumComp], const uint64_t agg[kNumComp]) {
  const int l = lane_id();
  const pbl_decode_out& O = A.out;
  const bool raw = (A.in.flags & PBL_ROW_RAW_KEYS) != 0;
  const uint32_t nkv = uint32_t(agg[0]), nres = uint32_t(agg[3]);
  if (O.restarts && kPart != 1)
    for (uint32_t r = l; r < nres; r += kWave) to_glb(O.restarts)[excl[3] + r] = V.le32(roff + 4 * r);
  uint32_t kcar = 0;
  for (uint32_t j0 = 0; j0 <= nkv; j0 += kWave) {
    pool::KBatch K;
    if (kPart != 2) pool::key_load<false, View>(W, V, raw, j0, nkv, K);
    pool::key_store<false, View, kPart>(W, V, A, b, j0, nkv, excl[0], excl[1], K, kcar);
  }
}

// PBL_RW_WAVES 2: a workgroup of two waves per block -- wave 0 stages,
// describes, then writes the keys and per-KV arrays while wave 1 writes the
// values (each phase a chain of LDS / issue latencies at one wave per SIMD;
// side by side they overlap).  3: a third wave takes the long keys' own bytes
// and the restart words from wave 0 (config 5 RI 16: a block's latency 18.8 K
// -> 16.9 K cycles, the rate unchanged, 1540 vs 1537 GiB/s).  1: one wave does
// all in turn (A/B: 1314 GiB/s).  Without the value stores the rate is 1752
// (diagnostic build): the value writes cost 11 %.
#ifndef PBL_RW_WAVES
#define PBL_RW_WAVES 2
#endif
constexpr int kRwWaves = PBL_RW_WAVES;
static_assert(kRwWaves >= 1 && kRwWaves <= 3, "emit waves per block: 1 to 3");

// One block's bases, status and extent: SCALAR loads (the constant address
// space: nothing in this kernel writes them).
template <class T>
using cptr = __attribute__((address_space(4))) const T*;
struct RDesc {
  uint64_t kv0, kv1, k0, k1, v0, v1, r0, r1, boff;
  uint32_t status, blen;
};
__device__ __forceinline__ RDesc load_desc(const Args& A, uint32_t b) {
  const pbl_decode_out& O = A.out;
  const uint32_t nb = A.in.n_blocks;
  const uint8_t* ws = reinterpret_cast<const uint8_t*>(O.workspace);
  RDesc d;
  d.kv0 = ((cptr<uint64_t>)O.blk_kv_base)[b];
  d.kv1 = ((cptr<uint64_t>)O.blk_kv_base)[b + 1];
  d.k0 = ((cptr<uint64_t>)O.blk_key_base)[b];
  d.k1 = ((cptr<uint64_t>)O.blk_key_base)[b + 1];
  d.v0 = ((cptr<uint64_t>)O.blk_val_base)[b];
  d.v1 = ((cptr<uint64_t>)O.blk_val_base)[b + 1];
  const cptr<uint64_t> rc = (cptr<uint64_t>)(ws + ws_rcnt_offset(nb));
  d.r0 = rc[b];
  d.r1 = rc[b + 1];
  d.status = ((cptr<uint32_t>)O.blk_status)[b];
  d.boff = ((cptr<uint64_t>)A.in.block_off)[b];
  d.blen = ((cptr<uint32_t>)A.in.block_len)[b];
  return d;
}

// One block of the emit (both waves).
__device__ __forceinline__ void emit_block(ELds& L, uint32_t* s_fast, const Args& A, uint32_t b, const RDesc& d) {
  const int l = lane_id();
  const bool w0 = kRwWaves == 1 || wave_id() == 0;
  const uint32_t nb = A.in.n_blocks, flags = A.in.flags;
  const pbl_decode_out& O = A.out;
  PSTAMP(A, b, 0, l == 0 && w0);
  const uint64_t excl[kNumComp] = {d.kv0, d.k0, d.v0, d.r0};
  const uint64_t agg[kNumComp] = {d.kv1 - d.kv0, d.k1 - d.k0, d.v1 - d.v0, d.r1 - d.r0};
  uint32_t status = d.status;
  if (status == PBL_OK && overflows(O, excl, agg)) status = PBL_OVERFLOW;
  const uint64_t boff = d.boff;
  const uint32_t blen = d.blen;
  const bool staged = status == PBL_OK && blen <= kMaxFastLen;
  const View V = lds_view(L.st.x, uint32_t(kPad + (boff & 15)));
  uint32_t fast = 0;
  if (w0) {
    const bool par = staged && agg[0] > 0 && agg[0] <= kEntRec;
    uint32_t pos = 0;
    if (staged) {  // (in flight under the metadata stores)
      pool::stage_dma(L.st, A.in.blocks, boff, blen);
      if (par && uint32_t(l) < agg[0])
        pos = to_glb(reinterpret_cast<const uint16_t*>(reinterpret_cast<const uint8_t*>(O.workspace) +
                                                       ws_ent_offset(nb)))[uint64_t(b) * kEntRec + l];
    }
    if (l == 0) {
      if (status != PBL_OK && O.key_off && excl[0] + b < O.kv_cap + nb) {
        to_glb(O.key_off)[excl[0] + b] = 0;
        to_glb(O.val_off)[excl[0] + b] = 0;
      }
      // (the bases are the scan's; the status, the counters and the totals)
      to_glb(O.blk_status)[b] = status;
      if (status != PBL_OK) {
        g_atomic_or(&O.totals->status_mask, 1u << status);
        g_atomic_add(&O.totals->n_bad_blocks, 1u);
      }
      if (b == nb - 1) {
        gptr<pbl_totals> T = to_glb(O.totals);
        T->n_kv = d.kv1;
        T->key_bytes = d.k1;
        T->val_bytes = d.v1;
        T->n_restarts = d.r1;
      }
    }
    PSTAMP(A, b, 1, l == 0);
    if (staged) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      wave_sync();
      PSTAMP(A, b, 2, l == 0);
      uint32_t roff = 0;
      if (PBL_RW_FAST && ((PBL_RW_PAR && par && front_par(V, blen, flags, L.sl, agg, pos, &roff)) ||
                          front_fast(V, blen, flags, L.sl, agg, &roff)))
        fast = roff + 1;
    }
    if (kRwWaves > 1 && l == 0) *s_fast = fast;
  }
  if (kRwWaves > 1) {
    __syncthreads();
    fast = *s_fast;
  }
  if (fast) {
    PSTAMP(A, b, 3, l == 0 && w0);
    if (w0) {
      if (kRwWaves == 3) emit_keys<1>(A, b, V, L.sl, fast - 1, excl, agg);
      else emit_keys<0>(A, b, V, L.sl, fast - 1, excl, agg);
      PSTAMP(A, b, 5, l == 0);
    }
    if (kRwWaves == 3 && wave_id() == 2) {
      emit_keys<2>(A, b, V, L.sl, fast - 1, excl, agg);
      PSTAMP(A, b, 7, l == 0);
    }
    if (kRwWaves == 1 || wave_id() == 1) {
      values_from_stage(L.sl.vp, V, uint32_t(agg[0]), to_glb(O.val_bytes) + excl[2]);
      PSTAMP(A, b, 6, l == 0);
    }
    PSTAMP(A, b, 4, l == 0 && w0);
  } else if (w0 && status == PBL_OK) {
    // the general walk: on the stage with the slot as its key buffer; a key
    // past the slot, or a block past the stage, from global memory with the
    // stage as the key buffer
    const uint8_t* g = A.in.blocks + boff;
    const uint64_t seq = A.in.synthetic_seq_num;
    if (l == 0) g_atomic_add(&O.totals->n_slow_blocks, 1u);
    SlowState ss;
    ss.status = PBL_UNSUPPORTED;
    if (staged) {
      wave_sync();
      slow_walk_t<SlowLds, PBL_RW_VALU>(SlowLds{V}, blen, flags, seq, to_lds_ptr(reinterpret_cast<uint8_t*>(&L.sl)),
                                        uint32_t(sizeof(L.sl)), kPassAll, O, b, excl, &ss);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      wave_sync();  // (the stage may become the key buffer below)
      PSTAMP(A, b, 3, l == 0);
    }
    if (ss.status == PBL_UNSUPPORTED)
      slow_walk_t<SlowGlb, PBL_BIG_U>(SlowGlb{to_glb(g), blen}, blen, flags, seq,
                                      to_lds_ptr(reinterpret_cast<uint8_t*>(L.st.x)), uint32_t(sizeof(L.st)),
                                      kPassAll, O, b, excl, &ss);
    PSTAMP(A, b, 4, l == 0);
    if (ss.status != PBL_OK && l == 0) {
      // the walk the size pass restated cannot disagree with it; if it ever
      // did, the block reports the walk's status
      to_glb(O.blk_status)[b] = ss.status;
      g_atomic_or(&O.totals->status_mask, 1u << ss.status);
      g_atomic_add(&O.totals->n_bad_blocks, 1u);
    }
  }
}

// One workgroup per block, in block order.  (Resident workgroups looping over
// blocks with the next block's descriptor prefetched measured slower: 1408 /
// 1310 GiB/s with static / ticketed assignment against 1475 on config 5 RI
// 16; the dispatcher's own refill hides a new workgroup's first round trip.)
__global__ void __launch_bounds__(kRwWaves * kWave) row_wave_emit_kernel(Args A) {
  __shared__ ELds L;
  __shared__ uint32_t s_fast;  // the block took the lane-parallel form (roff + 1), else 0
  const uint32_t b = blockIdx.x;
  emit_block(L, &s_fast, A, b, load_desc(A, b));
}

}  // namespace rwave
