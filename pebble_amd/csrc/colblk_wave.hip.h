// colblk_wave.hip.h — the colblk decode with one WAVE per block and no
// barrier, in two passes: the default for colblk batches (configs 3 and 5,
// and the colblk blocks of mixed batches).
//
// The single-pass forms place a block's outputs by a decoupled look-back, and
// with many blocks in flight the look-back convoys: a block waits for every
// predecessor back to the nearest inclusive prefix (the one-pass form of this
// kernel measured a 96 K-cycle median look-back of a 170 K-cycle block on
// config 5).  Here the placement is a separate scan:
//
//   sizes   colblk_wave_size_kernel: per block, the first kSizeStg bytes by
//           LDS-DMA (header, column directory, key columns, trailers,
//           prefixChanged, value offsets), DataBlockDecoder.Init + the
//           KeySeeker init lane per column (parse_block_wave), then lane per
//           row the key length and the bounds checks; the aggregate and
//           status go to blk_{kv,key,val}_base[b] / blk_status[b].  Nothing
//           waits.
//   scan    bases_scan_kernel<false>: the exclusive scan of those counts in
//           place (tiles of 1024 blocks, decoupled look-back across tiles),
//           totals at [n].
//   emit    colblk_wave_emit_kernel: per block, its final bases; the first
//           kStg bytes staged again, parsed again, then per-row arrays, keys
//           built in the wave's LDS key buffer (16-B segment copies, 16-B
//           stores out), the values range in 16-B chunks, kVU per lane in
//           flight, from the stage where it holds them, else global memory.
//
// A mixed batch (config 4) keeps its single pass over one look-back state: the
// size kernel publishes the colblk aggregates there (kList), the row kernel
// resolves through them, and the emit kernel (kList) resolves each colblk
// block's prefix afterwards -- every predecessor has published by then, so it
// never waits (the nearest inclusive prefix is the row block before it).
//
// Semantics are those of colblk_block.hip.h (DataBlockDecoder.Init
// sstable/colblk/data_block.go:1096-1109, DataBlockIter.Next :1662-1708,
// decodeMeta :1633-1641).  A block whose key region passes the stage reads
// it through the global reader (same results).
#pragma once

namespace pbl {
namespace col {
namespace cwave {

// Staged bytes: the size pass wants the key columns and the value offsets
// (config 3: ~4.7 KB); the emit also reads the first value bytes from the
// stage.  Measured (GiB/s, config 3 / config 5 colblk): size 2 / 4 / 6 KB with
// emit 6 KB 1440(pipeline) / 1513 / 1617 and 1259 / 1289 / 1283; emit 4 KB
// 1137 on config 5, 8 KB 1603 / 1337.
#ifndef PBL_CW_SSTAGE
#define PBL_CW_SSTAGE 6144
#endif
#ifndef PBL_CW_STAGE
#define PBL_CW_STAGE 6144  // emit stage, fixed-length batches
#endif
#ifndef PBL_CW_STAGE_VARLEN
#define PBL_CW_STAGE_VARLEN 8192  // emit stage, PBL_BATCH_VARLEN batches
#endif
#ifndef PBL_CW_KEYBUF
#define PBL_CW_KEYBUF 1536
#endif
#ifndef PBL_CW_VALU
#define PBL_CW_VALU 8  // 16-B value chunks per lane in flight (16: 782 against 809 on config 5)
#endif
#ifndef PBL_CW_WAVES
#define PBL_CW_WAVES 4  // waves per SIMD (one wave per workgroup; 5: within noise)
#endif
#ifndef PBL_CW_SWAVES
#define PBL_CW_SWAVES 5  // the size pass: 5 waves per SIMD (96 VGPRs, no scratch): config 3 / 5 colblk / 4 +1 %; 6 spills 36 B/lane
#endif
constexpr uint32_t kSizeStg = PBL_CW_SSTAGE;
constexpr uint32_t kKb = PBL_CW_KEYBUF;
constexpr int kVU = PBL_CW_VALU;

template <class T>
__device__ __forceinline__ void st_nt(gptr<T> p, T v) {  // outputs stream past the blocks' lines
  __builtin_nontemporal_store(v, p);
}

// The wave's LDS: the stage (block byte 0 at boff & 15; 32 B of slack past the
// end for lds_bytes16 and lds_copy), the key buffer, the block's descriptor.
template <uint32_t kS, uint32_t kK>
struct WLds {
  uint4 head4[(kS + 48) / 16];
  uint4 key4[(kK + 2 * kKeyPad) / 16];
  Desc d;
};

// Block b's first nst bytes into the stage by LDS-DMA (granule i of the 16-B
// aligned range at head4[i]; the ABI keeps every block readable up to its next
// 16-B boundary), one round trip.
__device__ __forceinline__ void cw_stage(uint4* head4, const uint8_t* blocks, uint64_t boff, uint32_t nst) {
  const int l = lane_id();
  const uint32_t sh = uint32_t(boff & 15);
  const gptr<const uint8_t> base = to_glb(blocks + (boff & ~uint64_t(15)));
  const uint32_t n16 = (sh + nst + 15) >> 4;
  for (uint32_t g0 = 0; g0 < n16; g0 += kWave)
    if (g0 + l < n16)
      __builtin_amdgcn_global_load_lds((gptr<const void>)(base + 16ull * (g0 + l)),
                                       (lptr<void>)to_lds_ptr(reinterpret_cast<void*>(&head4[g0])), 16, 0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  wave_sync();
}

// The block's reader: the stage for [0, nst) when the block is 8-B aligned
// (colblk blocks are, data_block.go:1097: the staged words keep every column's
// alignment), global memory for the rest.
__device__ __forceinline__ Src cw_src(const uint4* head4, const uint8_t* blocks, uint64_t boff, uint32_t blen,
                                      uint32_t nst) {
  const lds_cu8 h = (lds_cu8)to_lds(head4) + (boff & 15);
  return Src{h, h, (glb_cu8)(blocks + boff), (boff & 7) == 0 ? nst : 0u, 0xffffffffu, blen};
}

// Rows' key lengths and bounds checks (the size and the mixed emit passes):
// the block's aggregate {rows or visible rows, key bytes, value bytes, 0} and
// its status.
template <bool kHide>
__device__ __forceinline__ uint32_t cw_count(const Src& S, const Desc& d, uint32_t schema, uint32_t st, bool fast,
                                             uint64_t agg[kNumComp]) {
  const uint32_t rows = st == PBL_OK ? d.rows : 0;
  uint64_t kb = 0, nv = 0, vb = 0;
  bool bad = false;
  for (uint32_t r = lane_id(); r < rows; r += kWave) {
    const RowParts p = fast ? row_parts<true>(S, d, schema, r) : row_parts<false>(S, d, schema, r);
    bad |= !p.ok || !value_ok(S, d, r);
    if (!kHide || !row_obsolete(S, d, r)) {
      kb += p.klen;
      if (kHide) {
        nv++;
        vb += row_voff(S, d, r + 1) - row_voff(S, d, r);
      }
    }
  }
  kb = wave_sum(kb);
  if (kHide) {
    nv = wave_sum(nv);
    vb = wave_sum(vb);
  } else {
    nv = rows;
    vb = uint64_t(d.v_hi - d.v_lo);
  }
  if (st == PBL_OK) {
    if (__ballot(bad)) st = PBL_CORRUPT_BOUNDS;
    else if (kb > 0xffffffffull || vb > 0xffffffffull) st = PBL_UNSUPPORTED;
  }
  const bool ok = st == PBL_OK;
  agg[0] = ok ? nv : 0u;
  agg[1] = ok ? kb : 0u;
  agg[2] = ok ? vb : 0u;
  agg[3] = 0;
  return st;
}

// 16 bytes of the block at block offset j ([j, j + 16) inside the block): from
// the stage when it holds them, else global memory.
__device__ __forceinline__ uint4 blk16(const uint4* head4, uint32_t sh, uint32_t nst, gptr<const uint8_t> g,
                                       uint32_t j) {
  if (j + 16 <= nst) return lds_bytes16((lds_cu32)to_lds(head4), sh + j);
  typedef u32x4 u32x4_ua __attribute__((aligned(1)));
  const u32x4 v = *(gptr<const u32x4_ua>)(g + j);
  return make_uint4(v.x, v.y, v.z, v.w);
}

// Block b's outputs at bases excl (status OK, capacities checked).
template <bool F, class L_>
__device__ __forceinline__ void cw_emit(L_& L, const Args& A, uint32_t b, uint32_t schema, const Src& S, uint32_t sh,
                                        uint32_t nst, const uint64_t excl[kNumComp]) {
  const int l = lane_id();
  const pbl_decode_out& O = A.out;
  const Desc& d = L.d;
  const uint32_t rows = d.rows;
  const uint64_t kvb = excl[0], kbb = excl[1], vbb = excl[2];
  const gptr<const uint8_t> g = to_glb(A.in.blocks + A.in.block_off[b]);

  // ---- per-row arrays ----------------------------------------------------------
  const UCol& vo = d.v_off;
  for (uint32_t r = l; r <= rows; r += kWave) {
    const uint32_t v = vo.w ? uint32_t(S.le(vo.at + r * vo.w, vo.w)) : 0;
    st_nt(to_glb(O.val_off) + (kvb + b + r), v - d.v_lo);
    if (r < rows) {
      st_nt(to_glb(O.trailer) + (kvb + r), with_seq(u_at<F>(S, d.trailers, r), A.in.synthetic_seq_num, 0u));
      if (O.kv_flags) {
        uint8_t fl = 0;
        if (d.pc_at && ((S.le(d.pc_at + 8 * (r >> 6), 8) >> (r & 63)) & 1)) fl |= PBL_KV_PREFIX_CHANGED;
        if (d.obs_at && ((S.le(d.obs_at + 8 * (r >> 6), 8) >> (r & 63)) & 1)) fl |= PBL_KV_OBSOLETE;
        if (d.ext_at && ((S.le(d.ext_at + 8 * (r >> 6), 8) >> (r & 63)) & 1)) {
          const uint32_t v1 = vo.w ? uint32_t(S.le(vo.at + (r + 1) * vo.w, vo.w)) : 0;
          const bool vb = v1 > v && (S.byte(d.v_data + v) & 0xC0) == 0x80;
          fl |= vb ? PBL_KV_VALBLK_HANDLE : PBL_KV_BLOB_HANDLE;
        }
        st_nt(to_glb(O.kv_flags) + (kvb + r), fl);
      }
      if (O.entry_off) st_nt(to_glb(O.entry_off) + (kvb + r), r);
      if (O.tiering_span_id) {  // decodeMeta (data_block.go:1633-1641)
        st_nt(to_glb(O.tiering_span_id) + (kvb + r), u_at_any(S, d.span, r));
        st_nt(to_glb(O.tiering_attr) + (kvb + r), u_at_any(S, d.attr, r));
      }
    }
  }
  CSTAMP(A, b, 5);

  // ---- keys: 64 rows at a time, built in the key buffer -------------------------
  lds_u8 kb8 = (lds_u8)to_lds(L.key4);
  const lds_cu32 KW = (lds_cu32)to_lds(L.key4);
  constexpr uint32_t kKeyCap = uint32_t(sizeof(L.key4)) - 2 * kKeyPad;
  uint32_t cbase = 0;
  for (uint32_t r0 = 0; r0 < rows; r0 += kWave) {
    const uint32_t r = r0 + l;
    RowParts p;
    p.klen = 0;
    if (r < rows) p = row_parts<F>(S, d, schema, r);
    const uint32_t incl = wave_incl_scan(p.klen);
    const uint32_t tot = __shfl(incl, kWave - 1, kWave), ex = incl - p.klen;
    if (r < rows) st_nt(to_glb(O.key_off) + (kvb + b + r), cbase + ex);
    if (tot <= kKeyCap) {
      if (r < rows) build_key<F>(S, d, schema, p, kb8, kKeyPad + ex);
      wave_sync();
      const uint64_t lo = kbb + cbase, hi = lo + tot;
      for (uint64_t ga = (lo & ~uint64_t(15)) + 16ull * l; ga < hi; ga += 16ull * kWave)
        store16(O.key_bytes, ga, lo, hi, lds_bytes16(KW, uint32_t(kKeyPad + ga - lo)));
      wave_sync();  // (the buffer is the next chunk's)
    } else if (r < rows) {
      build_key_global<F>(S, d, schema, p, O.key_bytes + kbb + cbase + ex);
    }
    cbase += tot;
  }
  if (l == 0) st_nt(to_glb(O.key_off) + (kvb + b + rows), cbase);
  CSTAMP(A, b, 6);

  // ---- values: one contiguous range, 16-B chunks (the last ending at the end) --
  const uint32_t j0 = d.v_data + d.v_lo, n = d.v_hi - d.v_lo;
  const gptr<uint8_t> vout = to_glb(O.val_bytes) + vbb;
  typedef u32x4 u32x4_ua __attribute__((aligned(1)));
  if (n >= 16) {
    const uint32_t nch = (n + 15) >> 4;
    for (uint32_t k0 = l; k0 < nch; k0 += kWave * kVU) {
      uint4 x[kVU];
#pragma unroll
      for (int u = 0; u < kVU; u++) {
        const uint32_t k = k0 + kWave * u, q = 16 * k < n - 16 ? 16 * k : n - 16;
        x[u] = k < nch ? blk16(L.head4, sh, nst, g, j0 + q) : make_uint4(0, 0, 0, 0);
      }
#pragma unroll
      for (int u = 0; u < kVU; u++) {
        const uint32_t k = k0 + kWave * u, q = 16 * k < n - 16 ? 16 * k : n - 16;
        if (k < nch) __builtin_nontemporal_store(u32x4_ua{x[u].x, x[u].y, x[u].z, x[u].w}, (gptr<u32x4_ua>)(vout + q));
      }
    }
  } else {
    for (uint32_t i = l; i < n; i += kWave) vout[i] = uint8_t(S.byte(j0 + i));
  }
}

// ---- the size pass -------------------------------------------------------------
// kList: the colblk blocks of a mixed batch (the id list past its row ids;
// each aggregate is PUBLISHED to the look-back state); else every block of a
// colblk batch (aggregate and status to blk_{kv,key,val}_base[b] / blk_status[b]
// for bases_scan_kernel).  kHide: the visible rows, as
// col_emit_rows_hide places them.  Resident waves loop over the blocks.
struct SLds {
  uint4 head4[(kSizeStg + 48) / 16];
  Desc d;
};
template <bool kList, bool kHide>
__global__ void __launch_bounds__(kWave) __attribute__((amdgpu_waves_per_eu(PBL_CW_SWAVES)))
colblk_wave_size_kernel(Args A, const uint32_t* ids) {
  __shared__ SLds L;
  const int l = lane_id();
  const uint32_t nb = A.in.n_blocks;
  const pbl_decode_out& O = A.out;
  uint8_t* ws = reinterpret_cast<uint8_t*>(O.workspace);
  uint64_t* lb_state = reinterpret_cast<uint64_t*>(ws + kWsHeader);
  const uint32_t n_row = kList ? __hip_atomic_load(to_glb(reinterpret_cast<uint32_t*>(ws)) + kWsRowCount,
                                                   __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                               : 0u;
  for (uint32_t i = blockIdx.x; i < nb - n_row; i += gridDim.x) {
    const uint32_t b = kList ? to_glb(ids)[n_row + i] : i;
    const uint32_t schema = A.in.block_format ? uint32_t(to_glb(A.in.block_format)[b]) : A.in.format;
    const uint64_t boff = to_glb(A.in.block_off)[b];
    const uint32_t blen = to_glb(A.in.block_len)[b];
    const uint32_t nst = blen < kSizeStg ? blen : kSizeStg;
    cw_stage(L.head4, A.in.blocks, boff, nst);
    const Src S = cw_src(L.head4, A.in.blocks, boff, blen, nst);
    uint32_t st = parse_block_wave(S, schema, (A.in.flags & PBL_COL_TIERING) != 0, &L.d);
    wave_sync();
    uint64_t agg[kNumComp];
    st = cw_count<kHide>(S, L.d, schema, st, st == PBL_OK && S.nhead && L.d.key_end <= nst, agg);
    if (kList) {
      lb_publish(lb_state, nb, b, agg);
    } else if (l == 0) {
      to_glb(O.blk_kv_base)[b] = agg[0];
      to_glb(O.blk_key_base)[b] = agg[1];
      to_glb(O.blk_val_base)[b] = agg[2];
      to_glb(O.blk_status)[b] = st;
    }
    wave_sync();  // (the stage and the descriptor are the next block's)
  }
}

// ---- the emit pass ---------------------------------------------------------------
// kList = false: block b = the workgroup's, its bases from the scan, no
// look-back.  kList = true (mixed batches): the colblk id list; the block's
// aggregate is counted again and its prefix resolved by the look-back, which
// finds every predecessor published (the size pass and the row kernel ran
// before), so it never waits.
template <uint32_t kS, bool kList>
__global__ void __launch_bounds__(kWave) __attribute__((amdgpu_waves_per_eu(PBL_CW_WAVES)))
colblk_wave_emit_kernel(Args A, const uint32_t* ids) {
  __shared__ WLds<kS, kKb> L;
  const int l = lane_id();
  const uint32_t nb = A.in.n_blocks;
  const pbl_decode_out& O = A.out;
  uint8_t* ws = reinterpret_cast<uint8_t*>(O.workspace);
  uint32_t b = blockIdx.x;
  if (kList) {
    const uint32_t n_row = __hip_atomic_load(to_glb(reinterpret_cast<uint32_t*>(ws)) + kWsRowCount, __ATOMIC_RELAXED,
                                             __HIP_MEMORY_SCOPE_AGENT);
    if (blockIdx.x >= nb - n_row) return;
    b = to_glb(ids)[n_row + blockIdx.x];
  }
  CSTAMP(A, b, 0);
  const uint32_t schema = A.in.block_format ? uint32_t(to_glb(A.in.block_format)[b]) : A.in.format;
  const uint64_t boff = to_glb(A.in.block_off)[b];
  const uint32_t blen = to_glb(A.in.block_len)[b];
  const uint32_t nst = blen < kS ? blen : kS;
  uint64_t excl[kNumComp], agg[kNumComp];
  uint32_t st;
  if (!kList) {
    excl[0] = to_glb(O.blk_kv_base)[b];
    excl[1] = to_glb(O.blk_key_base)[b];
    excl[2] = to_glb(O.blk_val_base)[b];
    agg[0] = to_glb(O.blk_kv_base)[b + 1] - excl[0];
    agg[1] = to_glb(O.blk_key_base)[b + 1] - excl[1];
    agg[2] = to_glb(O.blk_val_base)[b + 1] - excl[2];
    excl[3] = agg[3] = 0;
    st = to_glb(O.blk_status)[b];
    if (st != PBL_OK) {  // (a failed block: its metadata only, no stage)
      if (l == 0) {
        if (O.key_off && excl[0] + b < O.kv_cap + nb) {
          to_glb(O.key_off)[excl[0] + b] = 0;
          to_glb(O.val_off)[excl[0] + b] = 0;
        }
        write_block_meta(O, b, nb, st, excl, agg, false);
      }
      return;
    }
  }
  cw_stage(L.head4, A.in.blocks, boff, nst);
  CSTAMP(A, b, 1);
  const Src S = cw_src(L.head4, A.in.blocks, boff, blen, nst);
  const uint32_t pst = parse_block_wave(S, schema, (A.in.flags & PBL_COL_TIERING) != 0, &L.d);
  wave_sync();
  const bool fast = pst == PBL_OK && S.nhead && L.d.key_end <= nst;
  if (kList) {
    uint64_t* lb_state = reinterpret_cast<uint64_t*>(ws + kWsHeader);
    st = cw_count<false>(S, L.d, schema, pst, fast, agg);
    lb_resolve(lb_state, nb, b, agg, excl, &O.totals->status_mask);
  }
  uint32_t status = st;
  if (st == PBL_OK && overflows(O, excl, agg)) status = PBL_OVERFLOW;
  if (l == 0) {
    if (status != PBL_OK && O.key_off && excl[0] + b < O.kv_cap + nb) {
      to_glb(O.key_off)[excl[0] + b] = 0;
      to_glb(O.val_off)[excl[0] + b] = 0;
    }
    write_block_meta(O, b, nb, status, excl, agg, !fast);
  }
  if (status != PBL_OK) return;
  CSTAMP(A, b, 4);
  const uint32_t sh = uint32_t(boff & 15);
  if (fast) cw_emit<true>(L, A, b, schema, S, sh, S.nhead, excl);
  else cw_emit<false>(L, A, b, schema, S, sh, S.nhead, excl);
  CSTAMP(A, b, 7);
}

// Exclusive scan, in place, of the per-block counts a size pass left in
// blk_{kv,key,val}_base[0, n): tiles of 1024 blocks per 256-thread workgroup
// in ticket order, each tile's aggregate published and its prefix resolved by
// the decoupled look-back (tf_scan_kernel's form); [n] gets the batch totals.
// kRst (row batches, rowblk_wave.hip.h): the restart counts at
// ws_rcnt_offset are scanned the same way (and copied to blk_rst_base when
// given); else (colblk: no restarts) blk_rst_base gets zeros.  (Each
// instantiation is launched from one translation unit only.)
constexpr uint32_t kScanTile = 1024;
template <bool kRst>
__global__ void __launch_bounds__(kTPB) bases_scan_kernel(Args A) {
  constexpr int kC = kRst ? 4 : 3;
  __shared__ uint32_t s_tile;
  __shared__ uint64_t s_wsum[kTPB / kWave][kC];
  __shared__ uint64_t s_excl[kC];
  const pbl_decode_out& O = A.out;
  uint8_t* ws = reinterpret_cast<uint8_t*>(O.workspace);
  uint32_t* hdr = reinterpret_cast<uint32_t*>(ws);
  uint64_t* lb_state = reinterpret_cast<uint64_t*>(ws + kWsHeader);
  const uint32_t nb = A.in.n_blocks, nt = (nb + kScanTile - 1) / kScanTile, t = threadIdx.x;
  uint64_t* const arr[4] = {O.blk_kv_base, O.blk_key_base, O.blk_val_base,
                            reinterpret_cast<uint64_t*>(ws + ws_rcnt_offset(nb))};
  for (;;) {
    if (t == 0) s_tile = g_atomic_add(hdr + 1, 1u);
    __syncthreads();
    const uint32_t tile = s_tile;
    __syncthreads();  // (s_tile is rewritten next iteration)
    if (tile >= nt) return;
    const uint32_t b0 = tile * kScanTile + 4 * t;
    uint64_t c[4][kC], s3[kC];
#pragma unroll
    for (int q = 0; q < kC; q++) s3[q] = 0;
#pragma unroll
    for (int k = 0; k < 4; k++) {
      const bool in = b0 + k < nb;
#pragma unroll
      for (int q = 0; q < kC; q++) {
        c[k][q] = in ? to_glb(arr[q])[b0 + k] : 0;
        s3[q] += c[k][q];
      }
    }
    uint64_t in3[kC];
#pragma unroll
    for (int q = 0; q < kC; q++) in3[q] = wave_incl_scan(s3[q]);
    if (lane_id() == kWave - 1)
      for (int q = 0; q < kC; q++) s_wsum[wave_id()][q] = in3[q];
    __syncthreads();
    uint64_t before[kC], agg[kNumComp] = {0, 0, 0, 0};
#pragma unroll
    for (int q = 0; q < kC; q++) before[q] = 0;
    for (int w = 0; w < kTPB / kWave; w++)
#pragma unroll
      for (int q = 0; q < kC; q++) {
        if (w < wave_id()) before[q] += s_wsum[w][q];
        agg[q] += s_wsum[w][q];
      }
    if (wave_id() == 0) {
      uint64_t excl[kNumComp];
      lb_publish(lb_state, nt, tile, agg);
      lb_resolve(lb_state, nt, tile, agg, excl, &O.totals->status_mask);
      if (lane_id() == 0)
        for (int q = 0; q < kC; q++) s_excl[q] = excl[q];
    }
    __syncthreads();
    uint64_t e[kC];
#pragma unroll
    for (int q = 0; q < kC; q++) e[q] = s_excl[q] + before[q] + in3[q] - s3[q];
#pragma unroll
    for (int k = 0; k < 4; k++) {
      const uint32_t b = b0 + k;
      if (b < nb) {
#pragma unroll
        for (int q = 0; q < kC; q++) to_glb(arr[q])[b] = e[q];
        if (O.blk_rst_base) to_glb(O.blk_rst_base)[b] = kRst ? e[kC - 1] : 0;
#pragma unroll
        for (int q = 0; q < kC; q++) e[q] += c[k][q];
      }
    }
    if (tile == nt - 1 && t == 0) {
#pragma unroll
      for (int q = 0; q < kC; q++) to_glb(arr[q])[nb] = s_excl[q] + agg[q];
      if (O.blk_rst_base) to_glb(O.blk_rst_base)[nb] = kRst ? s_excl[kC - 1] + agg[kC - 1] : 0;
    }
  }
}

}  // namespace cwave
}  // namespace col
}  // namespace pbl
