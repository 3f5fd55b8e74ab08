// rowblk_res.hip.h — the row-format decode with every block RESIDENT in LDS
// from its walk to its last output byte: four waves per CU, each owning one
// 32 KiB stage and one metadata slot, and each prefetching its NEXT block into
// registers while it decodes the current one.
//
// Why: the staging-pool kernel (rowblk_pool.hip.h) releases a block's stage
// after the walk and re-reads its keys and values from global memory for the
// emit.  With eight 32 KiB blocks in flight per CU those re-reads miss the
// XCD's L2 (128 KiB per CU) and come back from beyond it: 1.93x the algorithmic
// traffic and two thirds of a block's time in dependent global round trips.
// Here every byte of a block is read from HBM exactly once, and the emit reads
// only LDS.  The HBM latency of the block read is hidden by the register
// prefetch (the block after the current one, 33 x 16 B per lane), not by more
// stages: LDS holds four blocks per CU, and the fifth and later blocks in
// flight sit in the prefetching waves' registers.
//
// A wave's loop (block `cur` already in its registers):
//
//   store     the registers -> the wave's stage (ds_write_b128), then the loads
//             of block `nxt` into the same registers, then the ticket of the
//             block after it (nxt2) and its descriptor
//   walk      Iter.Init checks; lane per restart run (rowblk_writer.go:147-155
//             cuts the prefix chain there), headers parked in registers; a DPP
//             scan places the runs; the block's aggregate is PUBLISHED, and the
//             look-back windows are issued at once
//   meta      per-entry metadata words and per-KV value offsets into the slot
//   resolve   the exclusive prefix (its windows landed during the metadata pass)
//   keys      lane per KV from the stage: offsets, trailer, flags, entry offset,
//             the user key merged from its own bytes and its prefix parent's
//   values    8 lanes per KV, 16-B chunks from the stage
//
// Deadlock freedom: a wave holds tickets cur < nxt < nxt2, and only cur is
// staged.  Take the smallest unpublished ticket m.  If m is some wave's cur,
// that wave walks and publishes it without waiting.  If m is some wave's nxt
// or nxt2, that wave's cur is smaller, hence published, and its look-back waits
// only on tickets below it, all published: it finishes, and m moves up to its
// stage.  Either way m gets published, for any residency.
//
// Blocks outside the fast-path limits take the wave-serial general walk
// (rowblk_general.hip.h) on the staged bytes; blocks past kMaxFastLen are sized
// and written by big_block_{sizes,values}_kernel around the launch (they are
// never prefetched).  Results are identical on every path.
//
// Semantics: cockroachdb/pebble sstable/rowblk/rowblk_iter.go — Init :241-276,
// readFirstKey :418-485, readEntry :333-416, decodeInternalKey :487-504, value
// prefix :1192-1199 (sstable/block/kv.go:14-41), decodeRestart :1092-1096,
// HideObsoletePoints :1168-1179.
#pragma once

namespace res {

using pool::GSrc;
using pool::KBatch;
using pool::MState;
using pool::PAcc;
using pool::PRun;
using pool::Slot;
using pool::Stage;
using pool::VSeg;
using pool::dpp_incl_scan;
using pool::last_lane;
using pool::st_out;
using pool::u32x4_ug;

#ifndef PBL_RES_WAVES
#define PBL_RES_WAVES 4
#endif
constexpr int kNW = PBL_RES_WAVES;  // waves = stages = slots per workgroup (one workgroup per CU)
constexpr int kTPBR = kNW * kWave;
// 16-B granules of a staged block (any 16-B phase of a <= 32 KiB block)
constexpr uint32_t kMaxGran = (kMaxFastLen + 15 + 15) / 16;  // 2049
constexpr int kPf = int((kMaxGran + kWave - 1) / kWave);      // prefetch registers per lane: 33
// s_waitcnt vmcnt(0) (gfx9 encoding, expcnt / lgkmcnt left at their maxima):
// through the builtin, the compiler's wait tracking sees it and knows the
// prefetch registers have landed.
constexpr unsigned kVmcnt0 = 0x0F70u;

template <bool kHide>
struct ResLds {
  Stage st[kNW];
  Slot<kHide> sl[kNW];
};
static_assert(sizeof(ResLds<true>) <= 163840 && sizeof(ResLds<false>) <= 163840, "one workgroup per CU");
static_assert(Slot<true>::kKv == 511 && Slot<false>::kKv == 511, "slot capacity");

// A block's descriptor (its ticket's block id, where it sits, and how long).
struct Desc {
  uint64_t boff;
  uint32_t b, blen;
};

// The next block in registers: lane l holds 16-B granules l, l + 64, ... of
// the block's 16-B aligned range.
struct Pf {
  u32x4 r[kPf];
};

__device__ __forceinline__ uint32_t n_gran(const Desc& D) {
  if (D.blen > kMaxFastLen) return 0;  // a big block: never staged
  return uint32_t((((D.boff + D.blen + 15) & ~uint64_t(15)) - (D.boff & ~uint64_t(15))) >> 4);
}

__device__ __forceinline__ void pf_issue(Pf& P, const uint8_t* blocks, const Desc& D) {
  const uint32_t l = lane_id(), n16 = n_gran(D);
  const gptr<const u32x4> src = (gptr<const u32x4>)to_glb(blocks + (D.boff & ~uint64_t(15)));
#pragma unroll
  for (int k = 0; k < kPf; k++) {
    const uint32_t g = uint32_t(kWave) * k + l;
    if (g < n16) P.r[k] = src[g];
  }
}

// Granule g of the block to x[1 + g] (the stage's front pad is one granule).
__device__ __forceinline__ void pf_store(Stage& S, const Pf& P, const Desc& D) {
  const uint32_t l = lane_id(), n16 = n_gran(D);
  const lptr<u32x4> dst = (lptr<u32x4>)to_lds_ptr(reinterpret_cast<u32x4*>(&S.x[1]));
#pragma unroll
  for (int k = 0; k < kPf; k++) {
    const uint32_t g = uint32_t(kWave) * k + l;
    if (g < n16) dst[g] = P.r[k];
  }
}

// Lane 0 takes a ticket; every lane gets it.
__device__ __forceinline__ uint32_t take_ticket(uint32_t* tick) {
  uint32_t t = 0;
  if (lane_id() == 0) t = g_atomic_add(tick, 1u);
  return __builtin_amdgcn_readfirstlane(t);
}

__device__ __forceinline__ Desc load_desc(const Args& A, const uint32_t* ids, uint32_t t, uint32_t nt) {
  Desc D;
  D.b = t;
  D.boff = 0;
  D.blen = 0;
  if (t < nt) {
    if (ids) D.b = __builtin_amdgcn_readfirstlane(to_glb(ids)[t]);
    D.boff = to_glb(A.in.block_off)[D.b];
    D.blen = to_glb(A.in.block_len)[D.b];
  }
  return D;
}

// ---- values from the stage: 8 lanes per KV, 16-B chunks ----------------------
// Lane c of a group copies its value's chunks c, c + 8, ...; a value's last
// chunk ENDS at the value's end (overlapping the one before it), so no store
// is partial.  kVG KVs per group per step, each step's LDS reads issued before
// the previous step's stores.  Values shorter than 16 B go byte by byte;
// values longer than kWaveVal are copied by the whole wave.
constexpr int kVG = pool::kVG;
constexpr uint32_t kWaveVal = pool::kWaveVal;
struct VBatchL {
  u32x4 x[kVG];
};

__device__ __forceinline__ void val_load_l(const uint32_t* vp, const View& V, uint32_t nkv, uint32_t j0, VBatchL& B) {
  const uint32_t jl = j0 + (uint32_t(lane_id()) >> 3);
#pragma unroll
  for (int u = 0; u < kVG; u++) {
    const VSeg S = pool::val_seg(vp, nkv, jl + 8 * u);
    const uint4 w = V.ld16(int32_t(S.has ? S.vs + S.q : 0u));
    B.x[u] = u32x4{w.x, w.y, w.z, w.w};
  }
}

__device__ __forceinline__ void val_store_l(const uint32_t* vp, uint32_t nkv, uint32_t j0, const VBatchL& B,
                                            const View& V, gptr<uint8_t> vbytes) {
  const uint32_t c = uint32_t(lane_id()) & 7u, jl = j0 + (uint32_t(lane_id()) >> 3);
#pragma unroll
  for (int u = 0; u < kVG; u++) {
    const VSeg S = pool::val_seg(vp, nkv, jl + 8 * u);
    if (S.has) st_out((gptr<u32x4_ug>)(vbytes + S.vo + S.q), u32x4_ug(B.x[u]));
    if (S.vl > 128 && S.vl <= kWaveVal) {
      for (uint32_t o = 16 * c + 128; o < S.vl; o += 128) {
        const uint32_t q = o < S.vl - 16 ? o : S.vl - 16;
        const uint4 w = V.ld16(int32_t(S.vs + q));
        st_out((gptr<u32x4_ug>)(vbytes + S.vo + q), u32x4_ug{w.x, w.y, w.z, w.w});
      }
    } else if (S.vl < 16) {
      for (uint32_t o = c; o < S.vl; o += 8) st_out(vbytes + S.vo + o, uint8_t(V.byte(S.vs + o)));
    }
  }
}

__device__ __forceinline__ void copy_values_lds(const uint32_t* vp, const View& V, uint32_t nkv, gptr<uint8_t> vbytes,
                                                VBatchL& B) {
  const int l = lane_id();
  for (uint32_t j0 = 0; j0 < nkv; j0 += 8 * kVG) {
    if (j0 + 8 * kVG < nkv) {
      VBatchL N;
      val_load_l(vp, V, nkv, j0 + 8 * kVG, N);
      val_store_l(vp, nkv, j0, B, V, vbytes);
      B = N;
    } else {
      val_store_l(vp, nkv, j0, B, V, vbytes);
    }
  }
  // long values: the whole wave, four 16-B chunks per lane per step
  for (uint32_t j0 = 0; j0 < nkv; j0 += kWave) {
    const uint32_t j = j0 + uint32_t(l);
    const uint32_t a = j < nkv ? vp[j] : 0u, z = j < nkv ? vp[j + 1] : 0u;
    const uint32_t len = (z & 0xffffu) - (a & 0xffffu);
    for (uint64_t lm = __ballot(j < nkv && len > kWaveVal); lm; lm &= lm - 1) {
      const int sl = __builtin_ctzll(lm);
      const uint32_t ls = __shfl(a >> 16, sl, kWave), ll = __shfl(len, sl, kWave), lo = __shfl(a & 0xffffu, sl, kWave);
      for (uint32_t o0 = 16u * l; o0 < ll; o0 += 64u * kWave) {
        uint4 y[4];
#pragma unroll
        for (int k = 0; k < 4; k++) {
          const uint32_t o = o0 + 16u * kWave * k, q = o < ll - 16 ? o : ll - 16;
          y[k] = V.ld16(int32_t(ls + (o < ll ? q : 0u)));
        }
#pragma unroll
        for (int k = 0; k < 4; k++) {
          const uint32_t o = o0 + 16u * kWave * k, q = o < ll - 16 ? o : ll - 16;
          if (o < ll) st_out((gptr<u32x4_ug>)(vbytes + lo + q), u32x4_ug{y[k].x, y[k].y, y[k].z, y[k].w});
        }
      }
    }
  }
}

// ---- one block ---------------------------------------------------------------
// Decode block D from stage S with slot W; on entry the stage holds the block.
// Publishes the block's aggregate as soon as the walk has sized it, issues the
// look-back windows right behind it, writes the metadata while they travel,
// then resolves and writes every output from LDS.  `nxt2` is loaded on the
// way (its ticket's descriptor, needed one iteration later).
template <bool kHide>
__device__ __forceinline__ void block_res(Stage& S, Slot<kHide>& W, const Desc& D, const Args& A) {
  const int l = lane_id();
  const uint32_t nb = A.in.n_blocks, flags = A.in.flags, b = D.b;
  const uint64_t boff = D.boff;
  const uint32_t blen = D.blen;
  const bool vprefix = (flags & PBL_ROW_VALUE_PREFIX) && !(flags & PBL_ROW_RAW_KEYS);
  const bool raw = (flags & PBL_ROW_RAW_KEYS) != 0;
  const pbl_decode_out& O = A.out;
  uint64_t* lb_state = reinterpret_cast<uint64_t*>(reinterpret_cast<uint8_t*>(O.workspace) + kWsHeader);
  constexpr uint32_t kKv = uint32_t(Slot<kHide>::kKv);

  if (blen > kMaxFastLen) {
    __builtin_amdgcn_s_waitcnt(kVmcnt0);
    pool::block_big(A, b, boff, blen);
    return;
  }
  const View V = lds_view(S.x, uint32_t(kPad + (boff & 15)));
  uint32_t roff, nres;
  uint32_t status = rowc::init_checks(LdsRd{V}, blen, flags, &roff, &nres);
  bool slow = status == PBL_OK && nres > kKv;
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
      if (r0 < nres) pool::run_walk<kHide>(V, r0, nres, roff, flags, vprefix, RB, acc, ok, bad, vbad, over);
      // a run longer than kRunBuf keeps its parked head and counts only its tail
      if (over && ok)
        pool::count_span<kHide>(V, RB.pos, RB.e0, RB.n, RB.prev_kl, RB.prev_kind, flags, vprefix, acc, ok, bad, vbad);
    } else {
      for (uint32_t r = r0; r < r1 && ok; r++) {
        uint32_t rw, e0;
        if (!pool::run_bounds(V, r, nres, roff, &rw, &e0)) ok = false;
        else pool::count_span<kHide>(V, rw & kRestartMask, e0, 0, 0, 0, flags, vprefix, acc, ok, bad, vbad);
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
      // the sizes are final: publish, start the look-back, then the metadata
      const uint64_t agg[kNumComp] = {nkv, tkb, tvb, nres};
      lb_publish(lb_state, nb, b, agg);
      published = true;
      if (b > 0) G.issue(LbPtrs(lb_state, nb), int64_t(b) - 1);
      PSTAMP(A, b, 2, l == 0);
      MState M{ie - (kHide ? acc.ne : acc.cnt), ic - acc.cnt, iv - acc.vb, 0, 0, 0};
      if (single) {
        if (r0 < nres) {
          pool::park_meta<kHide>(W, V, RB, flags, M);
          if (over) pool::span_meta<kHide>(W, V, RB.pos, RB.e0, RB.rw, RB.n, RB.prev_kl, RB.prev_kind, flags, vprefix, M);
        }
      } else {
        for (uint32_t r = r0; r < r1; r++) {
          uint32_t rw, e0;
          pool::run_bounds(V, r, nres, roff, &rw, &e0);
          M.prev_sh = M.pp = M.ppsh = 0;
          pool::span_meta<kHide>(W, V, rw & kRestartMask, e0, rw, 0, 0, 0, flags, vprefix, M);
        }
      }
      if (l < 5) W.vp[nkv + l] = tvb;
      PSTAMP(A, b, 3, l == 0);
    }
  }
  if (status == PBL_OK && slow) {
    __builtin_amdgcn_s_waitcnt(kVmcnt0);
    pool::block_slow(S, reinterpret_cast<uint8_t*>(W.m0), uint32_t(sizeof(W.m0)), A, b, boff, blen);
    return;
  }
  if (!published) {  // a failed or empty block: its (zero) aggregate
    const bool okb = status == PBL_OK;
    const uint64_t agg[kNumComp] = {okb ? nkv : 0, okb ? tkb : 0, okb ? tvb : 0, okb ? nres : 0};
    lb_publish(lb_state, nb, b, agg);
    if (b > 0) G.issue(LbPtrs(lb_state, nb), int64_t(b) - 1);
    if (l < 5) W.vp[l] = 0;  // (an empty block's lone N+1 offsets)
  }
  if (status != PBL_OK) nkv = tkb = tvb = nres = 0;
  wave_sync();  // the slot's metadata, written lane by lane, is read across lanes below

  // the first key batch, the first value step and the restart words: their LDS
  // reads overlap the look-back's round trip
  KBatch K;
  VBatchL VB;
  uint32_t rs0 = 0;
  const bool ok0 = status == PBL_OK;
  if (ok0) {
    pool::key_load<kHide, View>(W, V, raw, 0, nkv, K);
    val_load_l(W.vp, V, nkv, 0, VB);
    if (O.restarts && uint32_t(l) < nres) rs0 = V.le32(roff + 4 * l);
  }
  const uint64_t agg[kNumComp] = {nkv, tkb, tvb, nres};
  uint64_t excl[kNumComp];
  lb_finish(lb_state, nb, b, agg, excl, &O.totals->status_mask, G);
  __builtin_amdgcn_s_waitcnt(kVmcnt0);  // (every load of the iteration has landed)
  PSTAMP(A, b, 4, l == 0);
  uint32_t st2 = status;
  if (ok0 && overflows(O, excl, agg)) st2 = PBL_OVERFLOW;
  if (l == 0) {
    if (st2 != PBL_OK && O.key_off && excl[0] + b < O.kv_cap + nb) {
      to_glb(O.key_off)[excl[0] + b] = 0;
      to_glb(O.val_off)[excl[0] + b] = 0;
    }
    write_block_meta(O, b, nb, st2, excl, agg, false);
  }
  if (st2 != PBL_OK) return;

  // ---- keys and per-KV arrays: lane per KV, from the stage ---------------------
  const uint64_t kvb = excl[0], kbb = excl[1], vbb = excl[2], rbb = excl[3];
  if (O.restarts && uint32_t(l) < nres) to_glb(O.restarts)[rbb + l] = rs0;
  uint32_t kcar = 0;
  pool::key_store<kHide, View>(W, V, A, b, 0, nkv, kvb, kbb, K, kcar);
  for (uint32_t j0 = kWave * pool::kKU; j0 <= nkv; j0 += kWave * pool::kKU) {
    KBatch N;
    pool::key_load<kHide, View>(W, V, raw, j0, nkv, N);
    pool::key_store<kHide, View>(W, V, A, b, j0, nkv, kvb, kbb, N, kcar);
  }
  if (O.restarts)
    for (uint32_t r = kWave + l; r < nres; r += kWave) to_glb(O.restarts)[rbb + r] = V.le32(roff + 4 * r);
  PSTAMP(A, b, 5, l == 0);

  // ---- values, stage -> global -----------------------------------------------
  if (tvb) copy_values_lds(W.vp, V, nkv, to_glb(O.val_bytes) + vbb, VB);
  PSTAMP(A, b, 6, l == 0);
}

// The persistent kernel: one workgroup of kNW waves per CU; wave w owns stage
// w and slot w.  Per iteration the wave knows: `cur` (in its registers),
// `nxt` (descriptor), `t2` (a ticket).  The VMEM issue order inside an
// iteration is what keeps the registers' loads off the critical path:
//   ds_write cur -> stage, loads of nxt -> registers, descriptor of t2, the
//   ticket t3, [walk, publish, look-back windows, metadata], look-back wait
//   (the youngest loads, so everything above has landed by then), stores.
// No load is ever waited for behind a store.  `ids` (mixed batches): the
// ascending ids of the batch's row blocks, their count at workspace header
// word kWsRowCount (the colblk blocks' aggregates are published before this
// launch).  Null: every block.
template <bool kHide>
__global__ void __launch_bounds__(kTPBR, 1) rowblk_res_kernel(Args A, const uint32_t* ids) {
  __shared__ ResLds<kHide> L;
  const int w = wave_id();
  Stage& S = L.st[w];
  Slot<kHide>& W = L.sl[w];
  uint32_t* tick = reinterpret_cast<uint32_t*>(A.out.workspace);
  const uint32_t nt = ids ? __hip_atomic_load(to_glb(tick) + kWsRowCount, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                          : A.in.n_blocks;
  Pf P;
  uint32_t tc = take_ticket(tick);
  Desc cur = load_desc(A, ids, tc, nt);
  if (tc < nt) pf_issue(P, A.in.blocks, cur);
  uint32_t tn = take_ticket(tick);
  Desc nxt = load_desc(A, ids, tn, nt);
  uint32_t t2 = take_ticket(tick);
  __builtin_amdgcn_s_waitcnt(kVmcnt0);
  while (tc < nt) {
    PSTAMP(A, cur.b, 0, lane_id() == 0);
    pf_store(S, P, cur);
    wave_sync();
    PSTAMP(A, cur.b, 1, lane_id() == 0);
    if (tn < nt) pf_issue(P, A.in.blocks, nxt);
    const Desc nxt2 = load_desc(A, ids, t2, nt);
    uint32_t t3 = 0;
    if (lane_id() == 0) t3 = g_atomic_add(tick, 1u);  // (read after the look-back's wait)
    block_res<kHide>(S, W, cur, A);
    t3 = __builtin_amdgcn_readfirstlane(t3);
    wave_sync();  // (the stage and the slot are the next block's)
    tc = tn;
    cur = nxt;
    tn = t2;
    nxt = nxt2;
    t2 = t3;
  }
  __builtin_amdgcn_s_waitcnt(kVmcnt0);
}

}  // namespace res
