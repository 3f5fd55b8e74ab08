// colblk_pipe.hip.h — persistent, lagged-look-back form of the colblk decode
// (one 256-thread workgroup loops over tickets; 4 workgroups per CU).
//
// Iteration i of a workgroup, whole-workgroup phases:
//   parse  block a_i from slot[i&1]: header + column directory (lane 0), key
//          sizes and bounds checks (thread per row), block scan, and the
//          aggregate is PUBLISHED to the look-back state;
//   emit   block a_{i-1} from slot[(i-1)&1], parsed one phase earlier: its
//          exclusive prefix is resolved (normally without waiting: every
//          predecessor published at least a phase ago), then per-row arrays,
//          keys (built in LDS, leaving as aligned 16-B stores) and values
//          (one contiguous range, global -> global);
//   the head/tail of block a_{i+1}, loaded into registers at the start of the
//          iteration, goes to the slot the emit released.
// The look-back's wait is thus off the critical path (colblk_block.hip.h's
// one-block-per-workgroup form waits for it in-line).
//
// Semantics are those of colblk_block.hip.h (same helpers; DataBlockDecoder.Init
// sstable/colblk/data_block.go:1096-1109, DataBlockIter.Next :1662-1708).
#pragma once

namespace pbl {
namespace col {
namespace cpipe {

constexpr uint32_t kHeadBuf = kStage + 16;  // head bytes + the block's 16-B phase
constexpr uint32_t kTailBuf = kTail + 32;   // tail bytes + phase + partial granule
enum { kNone = 0, kFast = 1, kErr = 2 };

#ifdef PBL_STAMPS
// diagnostic build only: per-block phase timestamps past the look-back state
#define CSTAMP(A_, b_, i_)                                                                      \
  do {                                                                                          \
    if (threadIdx.x == 0)                                                                       \
      reinterpret_cast<uint64_t*>(reinterpret_cast<uint8_t*>((A_).out.workspace) +             \
                                  ws_bytes((A_).in.n_blocks))[uint64_t(b_) * 16 + (i_)] =       \
          __builtin_amdgcn_s_memtime();                                                         \
  } while (0)
#else
#define CSTAMP(A_, b_, i_) do {} while (0)
#endif

struct Slot {
  uint4 head4[kHeadBuf / 16];
  uint4 tail4[kTailBuf / 16];
  Desc d;
  uint64_t boff;
  uint64_t agg[kNumComp];
  uint32_t b, blen, nhead, tail_lo, shift, status, mode, tot0;
  uint32_t fast;    // header parsed and the key columns inside the staged head
  uint32_t schema;  // the block's format (PBL_FMT_COL_*)
};

struct CLds {
  Slot s[2];
  uint4 key4[(kKeyBuf + 2 * kKeyPad) / 16];
  // HideObsoletePoints: a chunk's visible rows, compacted: value source offset
  // (values column), output offset (from the chunk's value base), length
  uint32_t rv0[kChunk], rvo[kChunk], rvl[kChunk];
  uint64_t red[4];
  uint64_t bases[kNumComp];
  uint32_t scratch[16];
  uint32_t bad, nxt, st;
};
#ifndef PBL_COL_PIPE_WG
#define PBL_COL_PIPE_WG 4  // workgroups per CU (128 VGPRs): config 3 1423 against 1257 at 3 (166 VGPRs); round 2's form spilled 160 B/lane at 4
#endif
static_assert(sizeof(CLds) <= 163840 / PBL_COL_PIPE_WG, "pipelined colblk workgroups per CU");

__device__ __forceinline__ Src slot_src(const Slot& P, const Args& A) {
  return Src{(lds_cu8)to_lds(P.head4) + P.shift, (lds_cu8)to_lds(P.tail4) + P.shift,
             (glb_cu8)(A.in.blocks + P.boff), P.nhead, P.tail_lo, P.blen};
}

// 16 bytes of block E at block offset j (any alignment, [j, j + 16) inside the
// block): from the staged head or tail when they hold them, else global.
__device__ __forceinline__ uint4 slot_ld16(const Slot& E, const Args& A, uint32_t j) {
  if (j + 16 <= E.nhead) return lds_bytes16((lds_cu32)to_lds(E.head4), E.shift + j);
  if (j >= E.tail_lo && j + 16 <= E.blen) return lds_bytes16((lds_cu32)to_lds(E.tail4), E.shift + j - E.tail_lo);
  typedef u32x4 u32x4_ua __attribute__((aligned(1)));
  const u32x4 v = *(gptr<const u32x4_ua>)(to_glb(A.in.blocks) + E.boff + j);
  return make_uint4(v.x, v.y, v.z, v.w);
}

// Head / tail geometry of a block (same split as col_block).
__device__ __forceinline__ void geometry(uint32_t blen, uint32_t* nhead, uint32_t* tail_lo) {
  *nhead = blen < kStage ? blen : kStage;
  *tail_lo = blen > kTail ? ((blen - kTail) & ~15u) : 0;
}

// Raw 16-B aligned granules of the head and tail regions, held in registers
// (4 + 1 per thread cover 12 KiB + 16 B and 512 + 32 B).
struct ColPf {
  u32x4 h0, h1, h2, h3, tl;
  __device__ __forceinline__ void load(const uint8_t* blocks, uint64_t boff, uint32_t blen) {
    uint32_t nhead, tail_lo;
    geometry(blen, &nhead, &tail_lo);
    const uint64_t a0 = boff & ~uint64_t(15);
    const uint32_t nh = uint32_t(((boff + nhead + 15) & ~uint64_t(15)) - a0) >> 4;
    gptr<const u32x4> H = to_glb(reinterpret_cast<const u32x4*>(blocks + a0));
    const uint32_t t = threadIdx.x;
    h0 = H[t < nh ? t : nh - 1];
    h1 = H[t + 256 < nh ? t + 256 : nh - 1];
    h2 = H[t + 512 < nh ? t + 512 : nh - 1];
    h3 = H[t + 768 < nh ? t + 768 : nh - 1];
    const uint64_t b0 = (boff + tail_lo) & ~uint64_t(15);
    const uint32_t nt = uint32_t(((boff + blen + 15) & ~uint64_t(15)) - b0) >> 4;
    gptr<const u32x4> T = to_glb(reinterpret_cast<const u32x4*>(blocks + b0));
    tl = T[t < nt ? t : nt - 1];
  }
  __device__ __forceinline__ void store(Slot& P, uint64_t boff, uint32_t blen) const {
    uint32_t nhead, tail_lo;
    geometry(blen, &nhead, &tail_lo);
    const uint32_t nh = uint32_t(((boff + nhead + 15) & ~uint64_t(15)) - (boff & ~uint64_t(15))) >> 4;
    const uint64_t b0 = (boff + tail_lo) & ~uint64_t(15);
    const uint32_t nt = uint32_t(((boff + blen + 15) & ~uint64_t(15)) - b0) >> 4;
    lptr<u32x4> H = to_lds_ptr(reinterpret_cast<u32x4*>(P.head4));
    lptr<u32x4> T = to_lds_ptr(reinterpret_cast<u32x4*>(P.tail4));
    const uint32_t t = threadIdx.x;
    if (t < nh) H[t] = h0;
    if (t + 256 < nh) H[t + 256] = h1;
    if (t + 512 < nh) H[t + 512] = h2;
    if (t + 768 < nh) H[t + 768] = h3;
    if (t < nt) T[t] = tl;
  }
};

// Slot bookkeeping for block b (thread 0 computes; all threads see it after the
// caller's barrier).  Blocks whose start is not 8-B aligned are staged with the
// funnel shift instead (8-B column reads from LDS need 8-B alignment).
__device__ __forceinline__ void slot_setup(Slot& P, uint32_t b, uint64_t boff, uint32_t blen, const Args& A) {
  P.b = b;
  P.schema = A.in.block_format && b < A.in.n_blocks ? uint32_t(to_glb(A.in.block_format)[b]) : A.in.format;
  P.boff = boff;
  P.blen = blen;
  geometry(blen, &P.nhead, &P.tail_lo);
  P.shift = (boff & 7) == 0 ? uint32_t(boff & 15) : 0u;
  P.mode = kNone;
}
__device__ __forceinline__ void slot_stage_funnel(Slot& P, const Args& A) {
  const uint64_t a1 = (P.boff + P.blen + 15) & ~uint64_t(15);
  stage((lds_u4)to_lds(P.head4), A.in.blocks, P.boff, a1, 0, P.nhead);
  stage((lds_u4)to_lds(P.tail4), A.in.blocks, P.boff, a1, P.tail_lo, P.blen - P.tail_lo);
}

// Resolve block E.b's exclusive prefix and write its block metadata (one wave:
// wave 1, at the start of the iteration, concurrently with wave 0's header
// decode of the next block).  Leaves the bases and the status in L.
__device__ __forceinline__ void col_resolve(CLds& L, const Slot& E, const Args& A) {
  const uint32_t nb = A.in.n_blocks;
  const pbl_decode_out& O = A.out;
  uint8_t* ws = reinterpret_cast<uint8_t*>(O.workspace);
  uint64_t* lb_state = reinterpret_cast<uint64_t*>(ws + kWsHeader);
  const uint32_t b = E.b;
  const uint64_t agg[kNumComp] = {E.agg[0], E.agg[1], E.agg[2], E.agg[3]};
  uint64_t excl[kNumComp];
  lb_resolve(lb_state, nb, b, agg, excl, &O.totals->status_mask);
  if (lane_id() == 0) {
    uint32_t status = E.status;
    if (status == PBL_OK && overflows(O, excl, agg)) status = PBL_OVERFLOW;
    L.st = status;
#pragma unroll
    for (int c = 0; c < kNumComp; c++) L.bases[c] = excl[c];
    if (status != PBL_OK && O.key_off && excl[0] + b < O.kv_cap + nb) {
      to_glb(O.key_off)[excl[0] + b] = 0;
      to_glb(O.val_off)[excl[0] + b] = 0;
    }
    write_block_meta(O, b, nb, status, excl, agg, !E.fast);
  }
}

// ---- parse phase (whole workgroup) ------------------------------------------------
template <bool F, bool kHide>
__device__ __forceinline__ void col_parse_rows(CLds& L, Slot& P, const Args& A, uint32_t schema, const Src& S) {
  const int t = threadIdx.x;
  const uint32_t nb = A.in.n_blocks;
  uint8_t* ws = reinterpret_cast<uint8_t*>(A.out.workspace);
  uint64_t* lb_state = reinterpret_cast<uint64_t*>(ws + kWsHeader);
  const Desc& d = P.d;
  const bool hdr_ok = P.status == PBL_OK;
  const uint32_t rows = hdr_ok ? d.rows : 0;
  const uint32_t nch = (rows + kChunk - 1) / kChunk;
  uint32_t k0 = 0;
  uint64_t my_kb = 0, my_n = 0, my_vb = 0;
  bool my_bad = false;
  for (uint32_t c = 0; c < nch; c++) {
    const uint32_t r = c * kChunk + t;
    if (r < rows) {
      const RowParts p = row_parts<F>(S, d, schema, r);
      my_bad |= !p.ok || !value_ok(S, d, r);
      // HideObsoletePoints (data_block.go:1680-1697): the visible rows only
      if (!kHide || !row_obsolete(S, d, r)) {
        my_kb += p.klen;
        if (kHide) {
          my_n++;
          my_vb += row_voff(S, d, r + 1) - row_voff(S, d, r);
        }
      }
      if (c == 0) k0 = p.klen;
    }
  }
  if (my_bad) L.bad = 1;
  uint32_t excl0, tot0, de, dt;
  block_excl_scan2(k0, 0u, &excl0, &de, L.scratch, &tot0, &dt);
  uint64_t n_tot = rows, vb_tot = uint64_t(d.v_hi - d.v_lo);
  if (kHide) {
    n_tot = block_sum_u64(my_n, L.red);
    vb_tot = block_sum_u64(my_vb, L.red);
  }
  const uint64_t kb_tot = block_sum_u64(my_kb, L.red);  // (syncs; also orders L.bad)
  (void)excl0;
  if (t == 0 && P.status == PBL_OK) {
    if (L.bad) P.status = PBL_CORRUPT_BOUNDS;
    else if (kb_tot > 0xffffffffull || vb_tot > 0xffffffffull) P.status = PBL_UNSUPPORTED;
  }
  __syncthreads();
  const bool ok = P.status == PBL_OK;
  const uint64_t agg[kNumComp] = {ok ? n_tot : 0ull, ok ? kb_tot : 0ull, ok ? vb_tot : 0ull, 0ull};
  if (wave_id() == 0) lb_publish(lb_state, nb, P.b, agg);
  if (t == 0) {
#pragma unroll
    for (int c = 0; c < kNumComp; c++) P.agg[c] = agg[c];
    P.tot0 = tot0;
    P.mode = ok ? kFast : kErr;
  }
}

template <bool kSizeOnly = false, bool kHide = false>
__device__ __forceinline__ void col_parse(CLds& L, Slot& P, const Slot& E, const Args& A, uint32_t schema) {
  const Src S = slot_src(P, A);
  CSTAMP(A, P.b, 0);
  if (!kSizeOnly && wave_id() == 1 && E.mode != kNone) col_resolve(L, E, A);
  if (wave_id() == 0 && P.b < A.in.n_blocks) {
    const uint32_t st = parse_block_wave(S, schema, (A.in.flags & PBL_COL_TIERING) != 0, &P.d);
    if (lane_id() == 0) {
      L.bad = 0;
      P.status = st;
    }
  }
  __syncthreads();
  if (P.b >= A.in.n_blocks) return;
  if (threadIdx.x == 0) P.fast = P.status == PBL_OK && P.d.key_end <= P.nhead;
  CSTAMP(A, P.b, 1);
  if (P.status == PBL_OK && P.d.key_end <= P.nhead) col_parse_rows<true, kHide>(L, P, A, schema, S);
  else col_parse_rows<false, kHide>(L, P, A, schema, S);
  CSTAMP(A, P.b, 2);
}

// ---- emit phase (whole workgroup) --------------------------------------------------
// The values range of a block: 16-B chunks of the source (chunk k at range
// offset min(16 k, n - 16): the last one ends at the range's end), each read
// from the staged head or tail or from global memory and stored unaligned at
// the same offset of the output; kValU chunks per thread per step.  The first
// step is loaded at the start of the emit (ValStep), so its round trip runs
// under the key build and the per-row stores.
#ifndef PBL_COL_VALU
#define PBL_COL_VALU 4
#endif
#ifndef PBL_COL_VAL_EARLY
#define PBL_COL_VAL_EARLY 0  // (its 16 VGPRs spill at 4 workgroups per CU)
#endif
constexpr int kValU = PBL_COL_VALU;
struct ValStep {
  u32x4 x[kValU];
};
__device__ __forceinline__ void val_step_load(const Slot& E, const Args& A, uint32_t j0, uint32_t n, uint32_t k0,
                                              ValStep& V) {
  const uint32_t nch = (n + 15) >> 4;
#pragma unroll
  for (int u = 0; u < kValU; u++) {
    const uint32_t k = k0 + kTPB * u, q = 16 * k < n - 16 ? 16 * k : n - 16;
    uint4 w = make_uint4(0, 0, 0, 0);
    if (n >= 16 && k < nch) w = slot_ld16(E, A, j0 + q);
    V.x[u] = u32x4{w.x, w.y, w.z, w.w};
  }
}
__device__ __forceinline__ void val_step_store(uint8_t* vout, uint32_t n, uint32_t k0, const ValStep& V) {
  typedef u32x4 u32x4_ua __attribute__((aligned(1)));
  const uint32_t nch = (n + 15) >> 4;
#pragma unroll
  for (int u = 0; u < kValU; u++) {
    const uint32_t k = k0 + kTPB * u, q = 16 * k < n - 16 ? 16 * k : n - 16;
    if (n >= 16 && k < nch) __builtin_nontemporal_store(u32x4_ua(V.x[u]), (gptr<u32x4_ua>)(to_glb(vout) + q));
  }
}

template <bool F>
__device__ __forceinline__ void col_emit_rows(CLds& L, const Slot& E, const Args& A, uint32_t schema, const Src& S,
                                              bool prebuilt, uint32_t ex0, uint32_t tot0, const ValStep& V0) {
  const int t = threadIdx.x;
  const pbl_decode_out& O = A.out;
  const uint32_t b = E.b;
  const Desc& d = E.d;
  const uint32_t rows = d.rows;
  const uint32_t nch = (rows + kChunk - 1) / kChunk;
  const uint64_t kvb = L.bases[0], kbb = L.bases[1], vbb = L.bases[2];
  const gptr<uint32_t> key_off = to_glb(O.key_off), val_off = to_glb(O.val_off);
  const gptr<uint64_t> trailer = to_glb(O.trailer);
  const gptr<uint8_t> kv_flags = to_glb(O.kv_flags);
  const gptr<uint32_t> entry_off = to_glb(O.entry_off);

  // per-row arrays
  const UCol& vo = d.v_off;
  for (uint32_t r = t; r <= rows; r += kTPB) {
    const uint32_t v = vo.w ? uint32_t(S.le(vo.at + r * vo.w, vo.w)) : 0;
    val_off[kvb + b + r] = v - d.v_lo;
    if (r < rows) {
      trailer[kvb + r] = with_seq(u_at<F>(S, d.trailers, r), A.in.synthetic_seq_num, 0u);
      if (O.kv_flags) {
        uint8_t fl = 0;
        if (d.pc_at && ((S.le(d.pc_at + 8 * (r >> 6), 8) >> (r & 63)) & 1)) fl |= PBL_KV_PREFIX_CHANGED;
        if (d.obs_at && ((S.le(d.obs_at + 8 * (r >> 6), 8) >> (r & 63)) & 1)) fl |= PBL_KV_OBSOLETE;
        if (d.ext_at && ((S.le(d.ext_at + 8 * (r >> 6), 8) >> (r & 63)) & 1)) {
          const uint32_t v1 = vo.w ? uint32_t(S.le(vo.at + (r + 1) * vo.w, vo.w)) : 0;
          const bool vb = v1 > v && (S.byte(d.v_data + v) & 0xC0) == 0x80;
          fl |= vb ? PBL_KV_VALBLK_HANDLE : PBL_KV_BLOB_HANDLE;
        }
        kv_flags[kvb + r] = fl;
      }
      if (O.entry_off) entry_off[kvb + r] = r;
    }
  }

  CSTAMP(A, b, 5);
  // key bytes: chunks of 256 rows built in the LDS key buffer, copied out as
  // aligned 16-B granules (keys past the buffer go straight to global memory)
  lds_u8 kb8 = (lds_u8)to_lds(L.key4);
  uint32_t cbase = 0;
  if (prebuilt) {
    // single chunk, built in LDS while wave 0 resolved the look-back
    if (uint32_t(t) < rows) key_off[kvb + b + t] = ex0;
    const uint64_t lo = kbb, hi = kbb + tot0;
    const lds_cu32 W = (lds_cu32)to_lds(L.key4);
    for (uint64_t ga = (lo & ~uint64_t(15)) + 16ull * t; ga < hi; ga += 16ull * kTPB)
      store16(O.key_bytes, ga, lo, hi, lds_bytes16(W, uint32_t(kKeyPad + ga - lo)));
    cbase = tot0;
  }
  for (uint32_t c = 0; c < (prebuilt ? 0u : nch); c++) {
    const uint32_t r = c * kChunk + t;
    RowParts p;
    p.klen = 0;
    if (r < rows) p = row_parts<F>(S, d, schema, r);
    uint32_t ex, tot, de, dt;
    block_excl_scan2(p.klen, 0u, &ex, &de, L.scratch, &tot, &dt);
    if (r < rows) key_off[kvb + b + r] = cbase + ex;
    if (tot <= kKeyBuf) {
      if (r < rows) build_key<F>(S, d, schema, p, kb8, kKeyPad + ex);
      __syncthreads();
      const uint64_t lo = kbb + cbase, hi = lo + tot;
      const lds_cu32 W = (lds_cu32)to_lds(L.key4);
      for (uint64_t ga = (lo & ~uint64_t(15)) + 16ull * t; ga < hi; ga += 16ull * kTPB)
        store16(O.key_bytes, ga, lo, hi, lds_bytes16(W, uint32_t(kKeyPad + ga - lo)));
    } else if (r < rows) {
      build_key_global<F>(S, d, schema, p, O.key_bytes + kbb + cbase + ex);
    }
    cbase += tot;
    __syncthreads();
  }
  if (t == 0) key_off[kvb + b + rows] = cbase;
  CSTAMP(A, b, 6);

  // value bytes: one contiguous range (val_step_*), the first step loaded at
  // the start of the emit
  {
    const uint32_t j0 = d.v_data + d.v_lo, n = d.v_hi - d.v_lo;
    uint8_t* vout = O.val_bytes + vbb;
    if (n >= 16) {
      const uint32_t nch = (n + 15) >> 4;
      if (PBL_COL_VAL_EARLY) {
        val_step_store(vout, n, uint32_t(t), V0);
      } else {
        ValStep V;
        val_step_load(E, A, j0, n, uint32_t(t), V);
        val_step_store(vout, n, uint32_t(t), V);
      }
      for (uint32_t k0 = uint32_t(t) + kTPB * kValU; k0 < nch; k0 += kTPB * kValU) {
        ValStep V;
        val_step_load(E, A, j0, n, k0, V);
        val_step_store(vout, n, k0, V);
      }
    } else {
      for (uint32_t i = uint32_t(t); i < n; i += kTPB) to_glb(vout)[i] = uint8_t(S.byte(j0 + i));
    }
  }
  // KVMeta (decodeMeta, data_block.go:1633-1641): its own pass after the
  // copies, so the per-row loop above keeps its register budget
  if (O.tiering_span_id) {
    for (uint32_t r = t; r < rows; r += kTPB) {
      to_glb(O.tiering_span_id)[kvb + r] = u_at_any(S, d.span, r);
      to_glb(O.tiering_attr)[kvb + r] = u_at_any(S, d.attr, r);
    }
  }
  CSTAMP(A, b, 7);
}


// HideObsoletePoints fused into the pipeline's emit (data_block.go:1680-1697):
// chunk by chunk, a block scan of (visible, key length) and of the visible
// value lengths places every visible row; keys are built in LDS and leave as
// aligned 16-B granules, values are copied row by row (8 threads per row,
// 16-B chunks, the last one ending at the value's end) from the staged head
// and tail or from global memory.
template <bool F>
__device__ __forceinline__ void col_emit_rows_hide(CLds& L, const Slot& E, const Args& A, uint32_t schema,
                                                   const Src& S) {
  const int t = threadIdx.x;
  const pbl_decode_out& O = A.out;
  const uint32_t b = E.b;
  const Desc& d = E.d;
  const uint32_t rows = d.rows;
  const uint32_t nch = (rows + kChunk - 1) / kChunk;
  const uint64_t kvb = L.bases[0], kbb = L.bases[1], vbb = L.bases[2];
  typedef u32x4 u32x4_ua __attribute__((aligned(1)));
  lds_u8 kb8 = (lds_u8)to_lds(L.key4);
  uint32_t cn = 0, ck = 0, cv = 0;
  for (uint32_t c = 0; c < nch; c++) {
    const uint32_t r = c * kChunk + t;
    const bool vis = r < rows && !row_obsolete(S, d, r);
    RowParts p;
    p.klen = 0;
    uint32_t v0 = 0, v1 = 0;
    if (vis) {
      p = row_parts<F>(S, d, schema, r);
      v0 = row_voff(S, d, r);
      v1 = row_voff(S, d, r + 1);
    }
    uint32_t en, ek, ev, dz, tn, tk, tv, dt;
    block_excl_scan2(vis ? 1u : 0u, vis ? p.klen : 0u, &en, &ek, L.scratch, &tn, &tk);
    __syncthreads();
    block_excl_scan2(v1 - v0, 0u, &ev, &dz, L.scratch, &tv, &dt);
    if (vis) {
      const uint64_t i = kvb + cn + en;
      to_glb(O.key_off)[i + b] = ck + ek;
      to_glb(O.val_off)[i + b] = cv + ev;
      to_glb(O.trailer)[i] = with_seq(u_at<F>(S, d.trailers, r), A.in.synthetic_seq_num, 0u);
      if (O.kv_flags) {
        uint8_t fl = 0;
        if (d.pc_at && ((S.le(d.pc_at + 8 * (r >> 6), 8) >> (r & 63)) & 1)) fl |= PBL_KV_PREFIX_CHANGED;
        if (d.ext_at && ((S.le(d.ext_at + 8 * (r >> 6), 8) >> (r & 63)) & 1)) {
          const bool vb = v1 > v0 && (S.byte(d.v_data + v0) & 0xC0) == 0x80;
          fl |= vb ? PBL_KV_VALBLK_HANDLE : PBL_KV_BLOB_HANDLE;
        }
        to_glb(O.kv_flags)[i] = fl;
      }
      if (O.entry_off) to_glb(O.entry_off)[i] = r;
      L.rv0[en] = d.v_data + v0;
      L.rvo[en] = ev;
      L.rvl[en] = v1 - v0;
    }
    // keys
    if (tk <= kKeyBuf) {
      if (vis) build_key<F>(S, d, schema, p, kb8, kKeyPad + ek);
      __syncthreads();
      const uint64_t lo = kbb + ck, hi = lo + tk;
      const lds_cu32 W = (lds_cu32)to_lds(L.key4);
      for (uint64_t ga = (lo & ~uint64_t(15)) + 16ull * t; ga < hi; ga += 16ull * kTPB)
        store16(O.key_bytes, ga, lo, hi, lds_bytes16(W, uint32_t(kKeyPad + ga - lo)));
    } else {
      if (vis) build_key_global<F>(S, d, schema, p, O.key_bytes + kbb + ck + ek);
      __syncthreads();
    }
    // values: 8 threads per visible row
    const gptr<uint8_t> vout = to_glb(O.val_bytes) + vbb + cv;
    const uint32_t q8 = uint32_t(t) & 7u;
    for (uint32_t q = uint32_t(t) >> 3; q < tn; q += kTPB / 8) {
      const uint32_t src = L.rv0[q], o0 = L.rvo[q], len = L.rvl[q];
      if (len >= 16) {
        for (uint32_t o = 16 * q8; o < len; o += 128) {
          const uint32_t qq = o < len - 16 ? o : len - 16;
          const uint4 w = slot_ld16(E, A, src + qq);
          __builtin_nontemporal_store(u32x4_ua{w.x, w.y, w.z, w.w}, (gptr<u32x4_ua>)(vout + o0 + qq));
        }
      } else {
        for (uint32_t o = q8; o < len; o += 8) vout[o0 + o] = uint8_t(S.byte(src + o));
      }
    }
    if (O.tiering_span_id && vis) {  // KVMeta (decodeMeta, data_block.go:1633-1641)
      to_glb(O.tiering_span_id)[kvb + cn + en] = u_at_any(S, d.span, r);
      to_glb(O.tiering_attr)[kvb + cn + en] = u_at_any(S, d.attr, r);
    }
    cn += tn;
    ck += tk;
    cv += tv;
    __syncthreads();  // (the key buffer and the row arrays are the next chunk's)
  }
  if (t == 0) {
    to_glb(O.key_off)[kvb + b + cn] = ck;
    to_glb(O.val_off)[kvb + b + cn] = cv;
  }
}

// Emit (whole workgroup) of block E.b, whose prefix col_resolve left in L.
template <bool F, bool kHide>
__device__ __forceinline__ void col_emit_t(CLds& L, const Slot& E, const Args& A, uint32_t schema) {
  const uint32_t b = E.b;
  const int t = threadIdx.x;
  const Src S = slot_src(E, A);
  CSTAMP(A, b, 3);
  if (L.st != PBL_OK) return;
  if (kHide) {
    col_emit_rows_hide<F>(L, E, A, schema, S);
    return;
  }
  ValStep V0;  // the values' first step, in flight under the key build (PBL_COL_VAL_EARLY)
  if (PBL_COL_VAL_EARLY) val_step_load(E, A, E.d.v_data + E.d.v_lo, E.d.v_hi - E.d.v_lo, uint32_t(t), V0);
  // keys of a single-chunk block are built in LDS first (one scan + one barrier)
  const uint32_t rows = E.d.rows;
  const bool prebuilt = rows <= kChunk && E.tot0 <= kKeyBuf;
  RowParts p;
  p.klen = 0;
  uint32_t ex = 0, tot = 0;
  if (prebuilt) {
    if (uint32_t(t) < rows) p = row_parts<F>(S, E.d, schema, uint32_t(t));
    uint32_t de, dt;
    block_excl_scan2(p.klen, 0u, &ex, &de, L.scratch, &tot, &dt);
    if (uint32_t(t) < rows) build_key<F>(S, E.d, schema, p, (lds_u8)to_lds(L.key4), kKeyPad + ex);
    __syncthreads();
  }
  CSTAMP(A, b, 4);
  col_emit_rows<F>(L, E, A, schema, S, prebuilt, ex, tot, V0);
}

template <bool kHide>
__device__ __forceinline__ void col_emit(CLds& L, const Slot& E, const Args& A, uint32_t schema) {
  if (E.fast) col_emit_t<true, kHide>(L, E, A, schema);
  else col_emit_t<false, kHide>(L, E, A, schema);
}

// ---- the persistent kernel ----------------------------------------------------------
// kSizeOnly: parse and publish every block's aggregate, no resolve and no
// outputs.  kHide: HideObsoletePoints fused (PBL_ROW_HIDE_OBSOLETE).
template <class Q, bool kSizeOnly = false, bool kHide = false>
__device__ __forceinline__ void col_pipe_body(CLds& L, const Args& A, const Q& q) {
  const int t = threadIdx.x;
  const uint32_t nb = A.in.n_blocks;
  if (t == 0) {
    const uint32_t t0 = q.take();
    L.s[1].mode = kNone;
    L.s[1].b = nb;
    if (t0 < nb) {
      slot_setup(L.s[0], t0, to_glb(A.in.block_off)[t0], to_glb(A.in.block_len)[t0], A);
    } else {
      L.s[0].b = nb;
      L.s[0].mode = kNone;
    }
  }
  __syncthreads();
  if (L.s[0].b < nb) {
    if (L.s[0].shift == (L.s[0].boff & 15)) {
      ColPf pf;
      pf.load(A.in.blocks, L.s[0].boff, L.s[0].blen);
      pf.store(L.s[0], L.s[0].boff, L.s[0].blen);
    } else {
      slot_stage_funnel(L.s[0], A);
    }
  }
  __syncthreads();
  for (uint32_t i = 0;; i++) {
    Slot& P = L.s[i & 1];
    Slot& E = L.s[(i + 1) & 1];
    const uint32_t cb = P.b;
    if (cb >= nb && E.mode == kNone) break;
    // the next ticket is taken now (its latency overlaps the parse): tickets are
    // held for one iteration only, which keeps the look-back distance short
    if (t == 0) L.nxt = cb < nb ? q.take() : nb;
    ColPf pf;
    col_parse<kSizeOnly, kHide>(L, P, E, A, P.schema);  // (wave 1 first resolves E's prefix)
    __syncthreads();
    const uint32_t nx = L.nxt;
    uint64_t nx_off = 0;
    uint32_t nx_len = 0;
    if (nx < nb) {
      nx_off = to_glb(A.in.block_off)[nx];
      nx_len = to_glb(A.in.block_len)[nx];
    }
    const bool pf_on = nx < nb && (nx_off & 7) == 0;
    if (pf_on) pf.load(A.in.blocks, nx_off, nx_len);  // lands during the emit
    if (!kSizeOnly && E.mode != kNone) col_emit<kHide>(L, E, A, E.schema);
    __syncthreads();
    if (t == 0) slot_setup(E, nx < nb ? nx : nb, nx_off, nx_len, A);
    if (pf_on) pf.store(E, nx_off, nx_len);
    __syncthreads();
    if (nx < nb && !pf_on) slot_stage_funnel(E, A);
    __syncthreads();
  }
}

#ifndef PBL_COL_PIPE_BODY_ONLY  // (rowblk_decode.hip uses the body in the mixed pipeline)
template <bool kHide>
__global__ void __launch_bounds__(kTPB, PBL_COL_PIPE_WG) colblk_pipe_kernel(Args A) {
  __shared__ CLds L;
  col_pipe_body<TicketQueue, false, kHide>(L, A, TicketQueue{reinterpret_cast<uint32_t*>(A.out.workspace),
                                                              A.in.n_blocks});
}
#endif

}  // namespace cpipe
}  // namespace col
}  // namespace pbl
