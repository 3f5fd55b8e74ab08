// rowblk_big.hip.h — what every row kernel shares besides the walk: the entry
// header decode, the Iter.Init checks, the diagnostic phase stamps, and the two
// passes for blocks past the 32 KiB LDS stage (big_block_sizes_kernel /
// big_block_sizes2_kernel before the decode launch, big_block_values_kernel
// after it for what the row kernel left).
//
// Semantics: cockroachdb/pebble sstable/rowblk/rowblk_iter.go — Init :241-276,
// readFirstKey :418-485, readEntry :333-416 (varints :345-398).
#pragma once

namespace rowc {

#ifdef PBL_STAMPS
// diagnostic build only: per-block phase timestamps (s_memtime) written past the
// look-back state in the workspace; never part of an output
#define PSTAMP(A_, b_, i_, lane0_)                                                             \
  do {                                                                                          \
    if (lane0_)                                                                                 \
      reinterpret_cast<uint64_t*>(reinterpret_cast<uint8_t*>((A_).out.workspace) +             \
                                  ws_bytes((A_).in.n_blocks))[uint64_t(b_) * 16 + (i_)] =       \
          __builtin_amdgcn_s_memtime();                                                         \
  } while (0)
// slot i_ = the wave's HW_ID (SIMD / CU / SE) and XCC_ID: where the roles run
#define PHWID(A_, b_, i_, lane0_)                                                              \
  do {                                                                                          \
    if (lane0_)                                                                                 \
      reinterpret_cast<uint64_t*>(reinterpret_cast<uint8_t*>((A_).out.workspace) +             \
                                  ws_bytes((A_).in.n_blocks))[uint64_t(b_) * 16 + (i_)] =       \
          uint64_t(__builtin_amdgcn_s_getreg(4 | (31 << 11))) |                                 \
          uint64_t(__builtin_amdgcn_s_getreg(20 | (15 << 11))) << 32;                           \
  } while (0)
#else
#define PSTAMP(A_, b_, i_, lane0_) do {} while (0)
#define PHWID(A_, b_, i_, lane0_) do {} while (0)
#endif

// Entry header (rowblk_iter.go:345-398: three uint32 varints) decoded without
// branches from the 8 bytes at the entry: each varint 1 or 2 bytes.  Returns
// false if any needs 3+ bytes (value >= 16384: the block takes the general path).
// Entry header: three uint32 varints decoded from one 8-byte window.  The
// common 1-2 byte form is decoded inline; a 3-byte varint (values of 16 KiB and
// more, config 5) takes hdr3 on the lanes that need it.  Anything longer takes
// the general path.
__device__ __forceinline__ bool hdr3(uint64_t w, uint32_t* sh, uint32_t* un, uint32_t* vl, uint32_t* h) {
  uint32_t p = 0, v[3];
  bool ok = true;
#pragma unroll
  for (int k = 0; k < 3; k++) {
    const uint32_t x = uint32_t(w >> (8 * p));  // p <= 6 here
    const uint32_t b0 = x & 0xff, b1 = (x >> 8) & 0xff, b2 = (x >> 16) & 0xff;
    const bool c0 = (b0 & 0x80) != 0, c1 = c0 && (b1 & 0x80) != 0;
    v[k] = c1 ? ((b0 & 0x7f) | ((b1 & 0x7f) << 7) | (b2 << 14)) : c0 ? ((b0 & 0x7f) | (b1 << 7)) : b0;
    ok = ok && !(c1 && (b2 & 0x80));
    p += c1 ? 3 : c0 ? 2 : 1;
  }
  *sh = v[0];
  *un = v[1];
  *vl = v[2];
  *h = p;
  // RunBuf packs unshared in 14 bits and the header length in 3
  return ok && p <= 7 && v[1] < 16384u;
}

__device__ __forceinline__ bool hdr2(uint64_t w, uint32_t* sh, uint32_t* un, uint32_t* vl, uint32_t* h) {
  if (__builtin_expect((uint32_t(w) & 0x808080u) == 0, 1)) {  // three 1-byte varints (values < 128)
    *sh = uint32_t(w) & 0xffu;
    *un = uint32_t(w >> 8) & 0xffu;
    *vl = uint32_t(w >> 16) & 0xffu;
    *h = 3;
    return true;
  }
  uint32_t p = 0, v[3];
  bool ok = true;
#pragma unroll
  for (int k = 0; k < 3; k++) {
    const uint32_t x = uint32_t(w >> (8 * p));
    const uint32_t b0 = x & 0xff, b1 = (x >> 8) & 0xff;
    const bool two = (b0 & 0x80) != 0;
    v[k] = two ? ((b0 & 0x7f) | (b1 << 7)) : b0;
    ok = ok && !(two && (b1 & 0x80));
    p += two ? 2 : 1;
  }
  *sh = v[0];
  *un = v[1];
  *vl = v[2];
  *h = p;
  if (__builtin_expect(!ok, 0)) ok = hdr3(w, sh, un, vl, h);
  return ok;
}

// Init checks (Init :248-256, readFirstKey :418-485) evaluated by every lane.
// Returns the status; *roff_o / *nres_o are set when it is PBL_OK.
template <class Rd>
__device__ __forceinline__ uint32_t init_checks(const Rd& rd, uint32_t blen, uint32_t flags, uint32_t* roff_o,
                                                uint32_t* nres_o) {
  *roff_o = 0;
  *nres_o = 0;
  if (blen < 4) return PBL_CORRUPT_BOUNDS;
  const uint32_t nw = rd.le32(blen - 4);
  if (nw == 0) return PBL_CORRUPT_NO_RESTARTS;
  if (nw >> 31) return PBL_CORRUPT_BOUNDS;
  const uint64_t need = 4ull * (1ull + nw);
  if (need > blen) return PBL_CORRUPT_BOUNDS;
  const uint32_t roff = blen - uint32_t(need);
  if (roff > 0 && !(flags & PBL_ROW_RAW_KEYS)) {
    if (rd.byte(0) != 0) return PBL_CORRUPT_FIRST_KEY;
    uint32_t un, vl;
    const uint32_t n1 = rd.varint(1, blen, &un);
    const uint32_t n2 = n1 ? rd.varint(1 + n1, blen, &vl) : 0;
    if (!n2) return PBL_CORRUPT_BOUNDS;
    if (un < 8) return PBL_CORRUPT_FIRST_KEY;
  }
  *roff_o = roff;
  *nres_o = nw;
  return PBL_OK;
}

#ifndef PBL_BIG_WIN
#define PBL_BIG_WIN 8  // blocks per sizes tier-1 workgroup (the values pass's form: 126 us at 8, 170 at 16)
#endif
#ifndef PBL_BIG_U
#define PBL_BIG_U 8  // value granules per lane in flight (16: within noise on config 5)
#endif
#ifndef PBL_BIG_KEYBUF
#define PBL_BIG_KEYBUF 8192
#endif
constexpr uint32_t kBigKeySmall = PBL_BIG_KEYBUF;  // the sizes tier-1 key buffer
constexpr int kWsBigRedo = 5;  // header u32 [5]: sizes tier-2 blocks (their ids in the redo area, ws_redo_offset)
constexpr int kWsBigPend = 6;  // header u32 [6]: blocks the row kernel did not write (ids at ws_pend_offset)

// Size pass for the blocks past the LDS stage (blen > kMaxFastLen), launched
// ahead of the row kernel on the same stream.  Their count walk reads global
// memory entry by entry; inside the pipeline it would hold back the look-back
// of every later ticket.  Here all of them walk at once and publish their
// aggregates, so the pipeline's parse_slow only resolves.  Same init checks and
// the same slow walk as parse_slow, so the aggregate is the one parse_slow
// computes.  Two tiers: tier 1 one one-wave
// workgroup per PBL_BIG_WIN-block window with a kBigKeySmall key buffer; a
// block whose walk needs more (PBL_UNSUPPORTED) is listed in the redo area and
// walked by tier 2 with the whole 32 KiB buffer.  (Tier 1 was one workgroup per
// 64 blocks, 4 per CU, with the 32 KiB buffer: config 5's 2195 big blocks took
// 59 us, two to three serial walks per wave; 33 us in windows, 16 us without
// one atomic per big block on a shared counter.)
__device__ __forceinline__ void big_block_publish(const Args& A, uint32_t b, const SlowState& ss) {
  const uint32_t nb = A.in.n_blocks;
  uint64_t* lb_state = reinterpret_cast<uint64_t*>(reinterpret_cast<uint8_t*>(A.out.workspace) + kWsHeader);
  const bool okk = ss.status == PBL_OK;
  const uint64_t agg[kNumComp] = {okk ? ss.nkv : 0, okk ? ss.kb : 0, okk ? ss.vb : 0, okk ? ss.nr : 0};
  lb_publish(lb_state, nb, b, agg);
  if (lane_id() == 0) {  // for parse_slow (write_block_meta replaces them)
    to_glb(A.out.blk_status)[b] = ss.status;
    to_glb(A.out.blk_kv_base)[b] = agg[0];
    to_glb(A.out.blk_key_base)[b] = agg[1];
    to_glb(A.out.blk_val_base)[b] = agg[2];
  }
}

// The count walk of a big block; a block failing Iter.Init's checks (zero
// restarts, a restart table past the block, a bad first entry) gets that
// status and a zero aggregate, which big_block_publish publishes like any other.
__device__ __forceinline__ void big_block_count(const Args& A, uint32_t b, lptr<uint8_t> keybuf, uint32_t keycap,
                                                SlowState* ss) {
  const uint32_t blen = A.in.block_len[b];
  const uint8_t* gblk = A.in.blocks + A.in.block_off[b];
  uint32_t roff, nres;
  const uint32_t st = init_checks(GlbRd{gblk}, blen, A.in.flags, &roff, &nres);
  if (st != PBL_OK) {
    ss->nkv = ss->kb = ss->vb = ss->nr = 0;
    ss->status = st;
    return;
  }
  const uint64_t dummy[kNumComp] = {0, 0, 0, 0};
  slow_walk_t<SlowGlb, 1>(SlowGlb{to_glb(gblk), blen}, blen, A.in.flags, A.in.synthetic_seq_num, keybuf, keycap, kPassCount,
                          A.out, b, dummy, ss);
}

__global__ void __launch_bounds__(kWave) big_block_sizes_kernel(Args A) {
  __shared__ uint4 keybuf4[kBigKeySmall / 16];
  const uint32_t nb = A.in.n_blocks;
  uint32_t* hdr = reinterpret_cast<uint32_t*>(A.out.workspace);
  uint32_t* redo = reinterpret_cast<uint32_t*>(reinterpret_cast<uint8_t*>(A.out.workspace) + ws_redo_offset(nb));
  for (uint64_t base = uint64_t(blockIdx.x) * PBL_BIG_WIN; base < nb; base += uint64_t(gridDim.x) * PBL_BIG_WIN) {
    const uint64_t bl = base + lane_id();
    // (row blocks only: a mixed batch's colblk blocks are the colblk pipeline's)
    uint64_t big = __ballot(lane_id() < PBL_BIG_WIN && bl < nb && to_glb(A.in.block_len)[bl] > kMaxFastLen &&
                            (!A.in.block_format || to_glb(A.in.block_format)[bl] == PBL_FMT_ROW));
    while (big) {
      const uint32_t b = uint32_t(base) + uint32_t(__builtin_ctzll(big));
      big &= big - 1;
      SlowState ss;
      big_block_count(A, b, to_lds_ptr(reinterpret_cast<uint8_t*>(keybuf4)), kBigKeySmall, &ss);
      if (ss.status == PBL_UNSUPPORTED) {  // a key past the small buffer (or a total past 4 GiB): tier 2
        if (lane_id() == 0) to_glb(redo)[g_atomic_add(hdr + kWsBigRedo, 1u)] = b;
        continue;
      }
      big_block_publish(A, b, ss);
    }
  }
}

__global__ void __launch_bounds__(kWave) big_block_sizes2_kernel(Args A) {
  __shared__ uint4 keybuf4[kLdsBlkBytes / 16];
  const uint32_t nb = A.in.n_blocks;
  const uint32_t* hdr = reinterpret_cast<const uint32_t*>(A.out.workspace);
  const uint32_t n = __hip_atomic_load(to_glb(hdr) + kWsBigRedo, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const uint32_t* redo = reinterpret_cast<const uint32_t*>(reinterpret_cast<uint8_t*>(A.out.workspace) +
                                                           ws_redo_offset(nb));
  for (uint32_t i = blockIdx.x; i < n; i += gridDim.x) {
    const uint32_t b = to_glb(redo)[i];
    SlowState ss;
    big_block_count(A, b, to_lds_ptr(reinterpret_cast<uint8_t*>(keybuf4)), uint32_t(kLdsBlkBytes), &ss);
    big_block_publish(A, b, ss);
  }
}

// Outputs of the blocks past the LDS stage.  The row kernel walks each one
// itself once its look-back has resolved the block's bases (block_big in
// rowblk_pool.hip.h: the wave's slot as the key buffer, the value copy hidden
// behind the other waves' work); the blocks it could not (a key past the slot)
// it lists, and this pass, launched after it on the same stream, walks them
// with the whole 32 KiB key buffer.  8 value granules per lane in flight.
__global__ void __launch_bounds__(kWave) big_block_values_kernel(Args A) {
  __shared__ uint4 keybuf4[kLdsBlkBytes / 16];
  const uint32_t nb = A.in.n_blocks;
  const uint32_t* hdr = reinterpret_cast<const uint32_t*>(A.out.workspace);
  const uint32_t n = __hip_atomic_load(to_glb(hdr) + kWsBigPend, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const uint32_t* pend = reinterpret_cast<const uint32_t*>(reinterpret_cast<const uint8_t*>(A.out.workspace) +
                                                           ws_pend_offset(nb));
  for (uint32_t i = blockIdx.x; i < n; i += gridDim.x) {
    const uint32_t b = to_glb(pend)[i];
    const uint32_t blen = A.in.block_len[b];
    const uint64_t bases[kNumComp] = {A.out.blk_kv_base[b], A.out.blk_key_base[b], A.out.blk_val_base[b],
                                      A.out.blk_rst_base ? A.out.blk_rst_base[b] : 0};
    SlowState ss;
    slow_walk_t<SlowGlb, PBL_BIG_U>(SlowGlb{to_glb(A.in.blocks + A.in.block_off[b]), blen}, blen, A.in.flags,
                                    A.in.synthetic_seq_num, to_lds_ptr(reinterpret_cast<uint8_t*>(keybuf4)),
                                    uint32_t(kLdsBlkBytes), kPassAll, A.out, b, bases, &ss);
  }
}

}  // namespace rowc
