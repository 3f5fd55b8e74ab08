// rowblk_global.hip.h — row batches whose blocks vary widely in length
// (PBL_BATCH_VARLEN, config 5: Zipf key and value lengths, ~13 KVs and a few
// large values per block) decoded without staging blocks in LDS, in three
// launches:
//
//   glb_sizes_kernel   one wave per block, many waves per CU (a 4 KiB LDS key
//                      buffer each): the wave-serial Iter.Next walk
//                      (rowblk_general.hip.h, count pass) straight from HBM;
//                      {status, n_kv, key bytes, value bytes, restarts} per
//                      block into the workspace.  A block whose key outgrows
//                      the buffer is left to glb_sizes_big_kernel (32 KiB).
//   glb_scan_kernel    tiles of 1024 blocks in ticket order, their prefixes
//                      by decoupled look-back: blk_*_base, per-block statuses
//                      (PBL_OVERFLOW past a capacity), totals
//   glb_values_kernel  one wave per block: the same walk writing every output
//                      at its base, values 16 B per lane, 8 granules in flight
//
// The LDS pipelines hold 4-5 blocks per CU and walk each block as a latency
// chain; these blocks have so few entries that the walk is short, and most of
// their bytes are values that move at copy rate once many blocks are in
// flight.  The size pass reads the headers and key bytes (the walk), the
// values pass the whole block.  Results are identical to every other path
// (same init checks and slow_walk).
//
// Semantics: cockroachdb/pebble sstable/rowblk/rowblk_iter.go (Init :241-276,
// readFirstKey :418-485, readEntry :333-416, Next :1145-1201).
#pragma once

namespace glb {

constexpr uint32_t kGKey = 4096;     // LDS key buffer of the common case
constexpr uint32_t kGTile = 1024;    // blocks per scan tile (256 threads x 4)
constexpr uint32_t kGBig = 0xffffffffu;      // workspace status: key past kGKey, for the 32 KiB pass
constexpr uint32_t kGBigDone = 0x80000000u;  // | status: sized by the 32 KiB pass (its values too)
#ifndef PBL_GLB_WAVES
#define PBL_GLB_WAVES 6  // waves per SIMD of the values walk (the size walk runs 8)
#endif
#ifndef PBL_GLB_VU
#define PBL_GLB_VU 2     // value granules per lane in flight in the values walk
#endif

__host__ __device__ inline uint32_t glb_tiles(uint32_t nb) { return (nb + kGTile - 1) / kGTile; }
// workspace: [0, 256) header (u32 [1] the tile ticket), the tiles' look-back
// state, then per block 4 u64 counts and a u32 status (all inside ws_bytes)
__host__ __device__ inline uint64_t glb_cnt_offset(uint32_t nb) {
  return (kWsHeader + uint64_t(2 + 2 * kNumComp) * glb_tiles(nb) * 8ull + 15) & ~15ull;
}
__host__ __device__ inline uint64_t glb_st_offset(uint32_t nb) { return glb_cnt_offset(nb) + 32ull * nb; }

__device__ __forceinline__ void glb_size_block(const Args& A, uint32_t b, lptr<uint8_t> kbuf, uint32_t keycap,
                                               bool big_pass) {
  const uint32_t flags = A.in.flags;
  uint8_t* ws = reinterpret_cast<uint8_t*>(A.out.workspace);
  const gptr<uint64_t> cnt = to_glb(reinterpret_cast<uint64_t*>(ws + glb_cnt_offset(A.in.n_blocks)));
  const gptr<uint32_t> sts = to_glb(reinterpret_cast<uint32_t*>(ws + glb_st_offset(A.in.n_blocks)));
  const uint32_t blen = to_glb(A.in.block_len)[b];
  const uint8_t* gblk = A.in.blocks + to_glb(A.in.block_off)[b];
  uint32_t roff, nres;
  uint32_t st = pipe::init_checks(GlbRd{gblk}, blen, flags, &roff, &nres);
  SlowState ss{0, 0, 0, 0, st};
  if (st == PBL_OK) {
    uint64_t dummy[kNumComp] = {0, 0, 0, 0};
    slow_walk_t<SlowGlb, 1>(SlowGlb{to_glb(gblk), blen}, blen, flags, A.in.synthetic_seq_num, kbuf, keycap,
                            kPassCount, A.out, b, dummy, &ss);
    st = ss.status;
    if (st == PBL_UNSUPPORTED && !big_pass) st = kGBig;
  }
  const bool ok = st == PBL_OK;
  if (lane_id() == 0) {
    cnt[4ull * b + 0] = ok ? ss.nkv : 0;
    cnt[4ull * b + 1] = ok ? ss.kb : 0;
    cnt[4ull * b + 2] = ok ? ss.vb : 0;
    cnt[4ull * b + 3] = ok ? ss.nr : 0;
    sts[b] = big_pass ? (st | kGBigDone) : st;
  }
}

__global__ void __launch_bounds__(kWave) __attribute__((amdgpu_waves_per_eu(8)))
glb_sizes_kernel(Args A) {
  __shared__ uint4 kb4[kGKey / 16];
  for (uint32_t b = blockIdx.x; b < A.in.n_blocks; b += gridDim.x) {
    glb_size_block(A, b, to_lds_ptr(reinterpret_cast<uint8_t*>(kb4)), kGKey, false);
    wave_sync();
  }
}

// The blocks glb_sizes_kernel left (a key past 4 KiB), with a 32 KiB buffer.
__global__ void __launch_bounds__(kWave) glb_sizes_big_kernel(Args A) {
  __shared__ uint4 kb4[kLdsBlkBytes / 16];
  const uint32_t nb = A.in.n_blocks;
  const gptr<uint32_t> sts =
      to_glb(reinterpret_cast<uint32_t*>(reinterpret_cast<uint8_t*>(A.out.workspace) + glb_st_offset(nb)));
  for (uint64_t base = uint64_t(blockIdx.x) * kWave; base < nb; base += uint64_t(gridDim.x) * kWave) {
    const uint64_t bl = base + lane_id();
    uint64_t m = __ballot(bl < nb && sts[bl] == kGBig);
    while (m) {
      const uint32_t b = uint32_t(base) + uint32_t(__builtin_ctzll(m));
      m &= m - 1;
      glb_size_block(A, b, to_lds_ptr(reinterpret_cast<uint8_t*>(kb4)), uint32_t(kLdsBlkBytes), true);
      wave_sync();
    }
  }
}

// Tiles in ticket order: exclusive prefixes of the per-block counts (decoupled
// look-back over the tiles' aggregates), per-block statuses and metadata.
__global__ void __launch_bounds__(kTPB) glb_scan_kernel(Args A) {
  __shared__ uint32_t s_tile;
  __shared__ uint64_t s_wsum[kTPB / kWave][kNumComp];
  __shared__ uint64_t s_excl[kNumComp];
  uint8_t* ws = reinterpret_cast<uint8_t*>(A.out.workspace);
  uint32_t* hdr = reinterpret_cast<uint32_t*>(ws);
  uint64_t* lb_state = reinterpret_cast<uint64_t*>(ws + kWsHeader);
  const uint32_t nb = A.in.n_blocks, nt = glb_tiles(nb), t = threadIdx.x;
  const gptr<const uint64_t> cnt = to_glb(reinterpret_cast<const uint64_t*>(ws + glb_cnt_offset(nb)));
  const gptr<const uint32_t> sts = to_glb(reinterpret_cast<const uint32_t*>(ws + glb_st_offset(nb)));
  const pbl_decode_out& O = A.out;
  for (;;) {
    if (t == 0) s_tile = g_atomic_add(hdr + 1, 1u);
    __syncthreads();
    const uint32_t tile = s_tile;
    __syncthreads();  // (s_tile is rewritten next iteration)
    if (tile >= nt) return;
    const uint32_t b0 = tile * kGTile + 4 * t;
    uint64_t c[4][kNumComp], s4[kNumComp] = {0, 0, 0, 0};
#pragma unroll
    for (int k = 0; k < 4; k++)
#pragma unroll
      for (int q = 0; q < kNumComp; q++) {
        c[k][q] = b0 + k < nb ? cnt[4ull * (b0 + k) + q] : 0;
        s4[q] += c[k][q];
      }
    uint64_t in4[kNumComp];
#pragma unroll
    for (int q = 0; q < kNumComp; q++) in4[q] = wave_incl_scan(s4[q]);
    if (lane_id() == kWave - 1)
      for (int q = 0; q < kNumComp; q++) s_wsum[wave_id()][q] = in4[q];
    __syncthreads();
    uint64_t before[kNumComp] = {0, 0, 0, 0}, agg[kNumComp] = {0, 0, 0, 0};
    for (int w = 0; w < kTPB / kWave; w++)
#pragma unroll
      for (int q = 0; q < kNumComp; q++) {
        if (w < wave_id()) before[q] += s_wsum[w][q];
        agg[q] += s_wsum[w][q];
      }
    if (wave_id() == 0) {
      uint64_t excl[kNumComp];
      lb_publish(lb_state, nt, tile, agg);
      lb_resolve(lb_state, nt, tile, agg, excl, &O.totals->status_mask);
      if (lane_id() == 0)
        for (int q = 0; q < kNumComp; q++) s_excl[q] = excl[q];
    }
    __syncthreads();
    uint64_t e[kNumComp];
#pragma unroll
    for (int q = 0; q < kNumComp; q++) e[q] = s_excl[q] + before[q] + in4[q] - s4[q];
#pragma unroll
    for (int k = 0; k < 4; k++) {
      const uint32_t b = b0 + k;
      if (b < nb) {
        uint32_t st = sts[b] & ~kGBigDone;
        if (st == PBL_OK && overflows(O, e, c[k])) st = PBL_OVERFLOW;
        if (st != PBL_OK && O.key_off && e[0] + b < O.kv_cap + nb) {
          to_glb(O.key_off)[e[0] + b] = 0;
          to_glb(O.val_off)[e[0] + b] = 0;
        }
        write_block_meta(O, b, nb, st, e, c[k], true);  // (every block takes the general walk: n_slow_blocks)
#pragma unroll
        for (int q = 0; q < kNumComp; q++) e[q] += c[k][q];
      }
    }
  }
}

__global__ void __launch_bounds__(kWave) __attribute__((amdgpu_waves_per_eu(PBL_GLB_WAVES)))
glb_values_kernel(Args A) {
  __shared__ uint4 kb4[kGKey / 16];
  const uint32_t nb = A.in.n_blocks;
  const gptr<const uint32_t> sts =
      to_glb(reinterpret_cast<const uint32_t*>(reinterpret_cast<uint8_t*>(A.out.workspace) + glb_st_offset(nb)));
  for (uint32_t b = blockIdx.x; b < nb; b += gridDim.x) {
    if (to_glb(A.out.blk_status)[b] != PBL_OK || sts[b] != PBL_OK) continue;
    const uint32_t blen = to_glb(A.in.block_len)[b];
    const uint64_t bases[kNumComp] = {to_glb(A.out.blk_kv_base)[b], to_glb(A.out.blk_key_base)[b],
                                      to_glb(A.out.blk_val_base)[b],
                                      A.out.blk_rst_base ? to_glb(A.out.blk_rst_base)[b] : 0};
    SlowState ss;
    slow_walk_t<SlowGlb, PBL_GLB_VU>(SlowGlb{to_glb(A.in.blocks + to_glb(A.in.block_off)[b]), blen}, blen,
                            A.in.flags, A.in.synthetic_seq_num, to_lds_ptr(reinterpret_cast<uint8_t*>(kb4)), kGKey, kPassAll,
                            A.out, b, bases, &ss);
    wave_sync();
  }
}

// The values of the blocks sized by glb_sizes_big_kernel.
__global__ void __launch_bounds__(kWave) glb_values_big_kernel(Args A) {
  __shared__ uint4 kb4[kLdsBlkBytes / 16];
  const uint32_t nb = A.in.n_blocks;
  const gptr<const uint32_t> sts =
      to_glb(reinterpret_cast<const uint32_t*>(reinterpret_cast<uint8_t*>(A.out.workspace) + glb_st_offset(nb)));
  for (uint64_t base = uint64_t(blockIdx.x) * kWave; base < nb; base += uint64_t(gridDim.x) * kWave) {
    const uint64_t bl = base + lane_id();
    // (the blocks glb_sizes_big_kernel sized: kGBigDone | PBL_OK; the metadata
    // status tells whether they fit the capacities)
    uint64_t m = __ballot(bl < nb && to_glb(A.out.blk_status)[bl] == PBL_OK && sts[bl] == kGBigDone);
    while (m) {
      const uint32_t b = uint32_t(base) + uint32_t(__builtin_ctzll(m));
      m &= m - 1;
      const uint32_t blen = to_glb(A.in.block_len)[b];
      const uint64_t bases[kNumComp] = {to_glb(A.out.blk_kv_base)[b], to_glb(A.out.blk_key_base)[b],
                                        to_glb(A.out.blk_val_base)[b],
                                        A.out.blk_rst_base ? to_glb(A.out.blk_rst_base)[b] : 0};
      SlowState ss;
      slow_walk_t<SlowGlb, 8>(SlowGlb{to_glb(A.in.blocks + to_glb(A.in.block_off)[b]), blen}, blen, A.in.flags,
                              A.in.synthetic_seq_num, to_lds_ptr(reinterpret_cast<uint8_t*>(kb4)),
                              uint32_t(kLdsBlkBytes), kPassAll, A.out, b, bases, &ss);
      wave_sync();
    }
  }
}

}  // namespace glb
