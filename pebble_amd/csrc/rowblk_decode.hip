// rowblk_decode.hip — gfx950 decoder for Pebble row-oriented data blocks: the
// C-ABI entry points (pbl_decode_batch, pbl_size_batch, the offset concat),
// the launchers, and the helpers every row kernel shares.
//
// Kernels:
//   rowblk_pool_kernel   (rowblk_pool.hip.h) the staging-pool kernel
//   big_block_*_kernel   (rowblk_big.hip.h) blocks past the 32 KiB LDS stage
//   row_wave_*_kernel    (rowblk_wave.hip.h) PBL_BATCH_VARLEN batches in two
//                        passes (sizes, bases_scan_kernel<true>, outputs)
//   mixed_*              row + colblk batches (config 4): the ids split by
//                        format, the colblk sizes, the row kernel over the row
//                        ids, the colblk pipeline over the colblk ids
//
// Semantics follow cockroachdb/pebble sstable/rowblk/rowblk_iter.go:
//   Init :241-276 (numRestarts, restarts offset), readFirstKey :418-485,
//   readEntry :333-416 (3 uint32 varints, fullKey = fullKey[:shared]+unshared),
//   decodeInternalKey :487-504 (LE64 trailer & TrailerObsoleteMask, <8 B =>
//   InternalKeyKindInvalid), value prefix :1192-1199 (block/kv.go:14-41),
//   decodeRestart :1092-1096, RawIter.readEntry :1784-1794 (PBL_ROW_RAW_KEYS).
// Blocks whose restart table is inconsistent with a per-run walk, or that do
// not fit the fast path's limits, take the general path (rowblk_general.hip.h):
// a wave-serial restatement of Iter.First/Next, bit-identical by construction.
#include <algorithm>
#include <atomic>

#include "common.hip.h"
#include "colblk_block.hip.h"

namespace pbl {
namespace row {

constexpr int kPad = 16;                  // LDS front pad: segment gathers may start up to 15 B early
constexpr int kLdsBlkBytes = kPad + 32768 + 32;  // block staging (any 16-B phase of a <=32 KiB block)
constexpr uint32_t kMaxFastLen = 32768;   // blocks up to this length take the LDS path
constexpr uint32_t kRestartMask = 0x7fffffffu;
constexpr uint64_t kTrailerObsoleteMask = ((((uint64_t)1 << 56) - 1) << 8) | 191u;
constexpr uint64_t kKindInvalid = kKindInvalidTrailer;

// Unaligned LDS access.  gfx950 runs in unaligned access mode (the HSA
// runtime's default), where one ds_read_b128 / b64 / b32 serves any byte
// address: a 16-byte gather is one instruction instead of five dword reads
// and four alignbytes.  Measured on config 2 (same box, A/B): unaligned 16-byte
// gathers +2.7 % (992 vs 965 GiB/s), unaligned 8-byte header reads in the
// parse walk -1.5 %; so gathers are unaligned and ld8/le32 stay dword reads
// (PBL_LDS_UA8 / PBL_LDS_UA16 switch each form for A/B builds).
typedef u32x4 u32x4_u __attribute__((aligned(1)));
typedef u32x2 u32x2_u __attribute__((aligned(1)));
typedef uint32_t u32_u __attribute__((aligned(1)));
#ifndef PBL_LDS_UA8
#define PBL_LDS_UA8 0
#endif
#ifndef PBL_LDS_UA16
#define PBL_LDS_UA16 1
#endif

// 16 bytes at LDS byte address a (any alignment)
__device__ inline uint4 lds_gather16(lptr<const uint32_t> W, uint32_t a) {
#if !PBL_LDS_UA16
  uint32_t q = a >> 2, r = a & 3;
  uint32_t x0 = W[q], x1 = W[q + 1], x2 = W[q + 2], x3 = W[q + 3], x4 = W[q + 4];
  return make_uint4(__builtin_amdgcn_alignbyte(x1, x0, r), __builtin_amdgcn_alignbyte(x2, x1, r),
                    __builtin_amdgcn_alignbyte(x3, x2, r), __builtin_amdgcn_alignbyte(x4, x3, r));
#else
  const u32x4 v = *(lptr<const u32x4_u>)(reinterpret_cast<lptr<const uint8_t>>(W) + a);
  return make_uint4(v.x, v.y, v.z, v.w);
#endif
}

// Read-only view of the staged block: its base offset lives in a register.
struct View;
__device__ __forceinline__ View lds_view(const void* lds, uint32_t base);
struct View {
  lptr<const uint8_t> B;   // LDS bytes (array start)
  lptr<const uint32_t> W;  // LDS words (array start)
  uint32_t base;      // byte index of block byte 0 (kPad + shift)
  __device__ inline uint32_t byte(uint32_t i) const { return B[base + i]; }
  // 8 block bytes [i, i+8) as a little-endian u64
  __device__ inline uint64_t ld8(uint32_t i) const {
#if !PBL_LDS_UA8
    uint32_t a = base + i, q = a >> 2, r = a & 3;
    uint32_t x0 = W[q], x1 = W[q + 1], x2 = W[q + 2];
    uint32_t lo = __builtin_amdgcn_alignbyte(x1, x0, r);
    uint32_t hi = __builtin_amdgcn_alignbyte(x2, x1, r);
    return uint64_t(hi) << 32 | lo;
#else
    const u32x2 v = *(lptr<const u32x2_u>)(B + base + i);
    return uint64_t(v.y) << 32 | v.x;
#endif
  }
  __device__ inline uint32_t le32(uint32_t i) const {
#if !PBL_LDS_UA8
    uint32_t a = base + i, q = a >> 2, r = a & 3;
    return __builtin_amdgcn_alignbyte(W[q + 1], W[q], r);
#else
    return *(lptr<const u32_u>)(B + base + i);
#endif
  }
  // 16 block bytes starting at block offset i (i may be up to 15 below 0)
  __device__ inline uint4 ld16(int32_t i) const { return lds_gather16(W, uint32_t(int32_t(base) + i)); }
};

__device__ __forceinline__ View lds_view(const void* lds, uint32_t base) {
  return View{to_lds_ptr(reinterpret_cast<const uint8_t*>(lds)), to_lds_ptr(reinterpret_cast<const uint32_t*>(lds)),
              base};
}

// mask of the low n bytes of a word, n clamped to [0, 4]
__device__ inline uint32_t low_bytes(int n) {
  n = n < 0 ? 0 : n;
  return n >= 4 ? 0xffffffffu : (1u << (8 * n)) - 1u;
}
// byte mask of bytes [a, b) within the 4-byte word k of a 16-byte granule
__device__ inline uint32_t word_mask(int k, uint32_t a, uint32_t b) {
  return low_bytes(int(b) - 4 * k) & ~low_bytes(int(a) - 4 * k);
}
__device__ inline void merge16(uint4& w, const uint4& v, uint32_t a, uint32_t b) {
  uint32_t m;
  m = word_mask(0, a, b); w.x = (w.x & ~m) | (v.x & m);
  m = word_mask(1, a, b); w.y = (w.y & ~m) | (v.y & m);
  m = word_mask(2, a, b); w.z = (w.z & ~m) | (v.z & m);
  m = word_mask(3, a, b); w.w = (w.w & ~m) | (v.w & m);
}

// varint from LDS (rowblk_iter.go:2020-2038); returns bytes used, 0 if it runs past `end`
__device__ inline uint32_t lds_varint(const View& V, uint32_t p, uint32_t end, uint32_t* v) {
  uint32_t r = 0;
#pragma unroll
  for (int i = 0; i < 5; i++) {
    if (p + i >= end) return 0;
    uint32_t b = V.byte(p + i);
    if (i == 4) { *v = r | (b << 28); return 5; }
    if (b < 128) { *v = r | (b << (7 * i)); return i + 1; }
    r |= (b & 0x7f) << (7 * i);
  }
  return 0;
}

#include "rowblk_general.hip.h"

struct LdsRd {  // staged block through the View
  View V;
  __device__ uint32_t byte(uint32_t i) const { return V.byte(i); }
  __device__ uint32_t le32(uint32_t i) const { return V.le32(i); }
  __device__ uint32_t varint(uint32_t p, uint32_t end, uint32_t* v) const { return lds_varint(V, p, end, v); }
};
struct GlbRd {  // unstaged block in global memory
  const uint8_t* g;
  __device__ uint32_t byte(uint32_t i) const { return g[i]; }
  __device__ uint32_t le32(uint32_t i) const { return g_le32(g + i); }
  __device__ uint32_t varint(uint32_t p, uint32_t end, uint32_t* v) const { return g_varint(g + p, g + end, v); }
};

#include "rowblk_big.hip.h"
#include "rowblk_pool.hip.h"
#include "rowblk_wave.hip.h"

}  // namespace row
}  // namespace pbl

#define PBL_COL_PIPE_BODY_ONLY
#include "colblk_pipe.hip.h"
#include "colblk_wave.hip.h"

namespace pbl {
namespace row {

// ---- mixed row + colblk batches (config 4) ------------------------------------
// The batch's block ids are split by format into two ascending lists
// (mixed_split_*); every block's outputs are placed by ONE look-back state
// indexed by the block id, so every block's exclusive prefix is over the batch
// order, as in the single-format kernels.

__global__ void __launch_bounds__(kTPB) mixed_split_count_kernel(Args A, uint32_t* counts) {
  const uint32_t nb = A.in.n_blocks;
  const uint32_t c0 = blockIdx.x * kSplitChunk;
  uint32_t k = 0;
  for (uint32_t i = c0 + threadIdx.x; i < nb && i < c0 + kSplitChunk; i += kTPB)
    k += to_glb(A.in.block_format)[i] == PBL_FMT_ROW;
  __shared__ uint32_t red[kTPB / kWave];
  k = wave_sum(k);
  if (lane_id() == 0) red[wave_id()] = k;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t s = 0;
    for (int w = 0; w < kTPB / kWave; w++) s += red[w];
    counts[blockIdx.x] = s;
  }
}

__global__ void __launch_bounds__(kTPB) mixed_split_scatter_kernel(Args A, const uint32_t* counts, uint32_t n_chunks,
                                                                   uint32_t* ids) {
  const uint32_t nb = A.in.n_blocks;
  const uint32_t c = blockIdx.x;
  __shared__ uint32_t sc[kTPB];
  __shared__ uint32_t base_row, base_col;
  if (threadIdx.x == 0) {
    uint32_t before = 0, total = 0;
    for (uint32_t i = 0; i < n_chunks; i++) {
      const uint32_t x = to_glb(counts)[i];
      if (i < c) before += x;
      total += x;
    }
    base_row = before;
    base_col = total + (c * kSplitChunk - before);  // col ids follow all row ids
    if (c == 0) to_glb(reinterpret_cast<uint32_t*>(A.out.workspace))[kWsRowCount] = total;
  }
  __syncthreads();
  // in-order compaction of the chunk, kTPB ids at a time
  for (uint32_t i0 = c * kSplitChunk; i0 < nb && i0 < (c + 1) * kSplitChunk; i0 += kTPB) {
    const uint32_t i = i0 + threadIdx.x;
    const bool live = i < nb && i < (c + 1) * kSplitChunk;
    const uint32_t isrow = live && to_glb(A.in.block_format)[i] == PBL_FMT_ROW;
    sc[threadIdx.x] = isrow;
    __syncthreads();
    // inclusive scan (Hillis-Steele over kTPB entries)
    for (uint32_t d = 1; d < kTPB; d <<= 1) {
      const uint32_t v = threadIdx.x >= d ? sc[threadIdx.x - d] : 0u;
      __syncthreads();
      sc[threadIdx.x] += v;
      __syncthreads();
    }
    const uint32_t incl = sc[threadIdx.x], nrow = sc[kTPB - 1];
    const uint32_t nlive = (nb - i0 < kTPB ? nb - i0 : kTPB);
    if (live) {
      if (isrow) to_glb(ids)[base_row + incl - 1] = i;
      else to_glb(ids)[base_col + (threadIdx.x - (incl - isrow))] = i;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      base_row += nrow;
      base_col += nlive - nrow;
    }
    __syncthreads();
  }
}

// Mixed batches: launches over the split id lists.  (1) the colblk sizes are
// published (colblk_wave_size_kernel<true>, colblk_wave.hip.h); (2) the row
// kernel runs over the row list, its look-back walking through the colblk
// aggregates; (3) the colblk blocks' outputs (mixed_col_kernel below with
// HideObsoletePoints, else the wave form's emit): every predecessor has
// published, so their look-backs end at the row block before them.
// Deadlock-free: (2) waits only on aggregates published by (1) or by its own
// resident waves in ticket order, (3) never waits.
constexpr int kWsColTick2 = 4;  // header u32 [4]: the colblk queue of launch (3)

// (3) with HideObsoletePoints: the colblk pipeline's fused form over the
// colblk list (the visible rows, as colblk_wave_size_kernel<true, true>
// counted them).
template <bool kHide>
__global__ void __launch_bounds__(kTPB, PBL_COL_PIPE_WG) mixed_col_kernel(Args A, const uint32_t* ids) {
  __shared__ col::cpipe::CLds L;
  const uint32_t nb = A.in.n_blocks;
  uint32_t* hdr = reinterpret_cast<uint32_t*>(A.out.workspace);
  const uint32_t n_row = __hip_atomic_load(to_glb(hdr) + kWsRowCount, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  col::cpipe::col_pipe_body<ListQueue, false, kHide>(L, A, ListQueue{hdr + kWsColTick2, ids + n_row, nb - n_row, nb});
}

// KVMeta{} for the row blocks' KVs (rowblk.Iter has no meta columns) when the
// caller asked for the tiering arrays: one wave per block, after the decode
// (a block that did not decode has no KV range).
__global__ void __launch_bounds__(kWave) row_meta_zero_kernel(Args A) {
  const pbl_decode_out& O = A.out;
  const uint32_t nb = A.in.n_blocks;
  for (uint32_t b = blockIdx.x; b < nb; b += gridDim.x) {
    const uint32_t fmt = A.in.block_format ? uint32_t(to_glb(A.in.block_format)[b]) : A.in.format;
    if (fmt != PBL_FMT_ROW || to_glb(O.blk_status)[b] != PBL_OK) continue;
    const uint64_t k0 = to_glb(O.blk_kv_base)[b], k1 = to_glb(O.blk_kv_base)[b + 1];
    for (uint64_t k = k0 + lane_id(); k < k1; k += kWave) {
      to_glb(O.tiering_span_id)[k] = 0;
      to_glb(O.tiering_attr)[k] = 0;
    }
  }
}

// Size pass epilogue: a block that decoded reports PBL_OK, not the forced
// overflow of the pass.
__global__ void size_fixup_kernel(uint32_t* blk_status, pbl_totals* totals, uint32_t n) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i == 0) __hip_atomic_fetch_and(&totals->status_mask, ~(1u << PBL_OVERFLOW), __ATOMIC_RELAXED,
                                     __HIP_MEMORY_SCOPE_AGENT);
  if (i < n && blk_status[i] == PBL_OVERFLOW) {
    blk_status[i] = PBL_OK;
    g_atomic_add(&totals->n_bad_blocks, ~0u);  // (-1)
  }
}

__global__ void rebase_kernel(uint64_t* kvb, uint64_t* kb, uint64_t* vb, uint64_t* rb, uint32_t n,
                              uint64_t dkv, uint64_t dk, uint64_t dv, uint64_t dr) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i > n) return;
  kvb[i] += dkv;
  kb[i] += dk;
  vb[i] += dv;
  if (rb) rb[i] += dr;
}

__global__ void offset_concat_kernel(uint64_t* kvb, uint64_t* kb, uint64_t* vb, uint64_t* rb, uint32_t n,
                                     const uint64_t* rank_totals, uint32_t rank) {
  uint64_t d[4] = {0, 0, 0, 0};
  for (uint32_t r = 0; r < rank; r++)
    for (int c = 0; c < 4; c++) d[c] += rank_totals[4 * r + c];
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i <= n; i += gridDim.x * blockDim.x) {
    kvb[i] += d[0];
    kb[i] += d[1];
    vb[i] += d[2];
    if (rb) rb[i] += d[3];
  }
}

}  // namespace row
}  // namespace pbl

namespace pbl {

namespace {
constexpr int kMaxDevices = 64;
std::atomic<int> g_cus[kMaxDevices];
std::atomic<int> g_per_cu[kMaxDevices][kKNum];
}  // namespace

uint64_t persistent_grid(hipStream_t st, PersistentKernel k, const void* fn, uint64_t n_units, int* cus_out,
                         int block_threads) {
  int dev = -1;
  if (st ? hipStreamGetDevice(st, &dev) != hipSuccess : hipGetDevice(&dev) != hipSuccess) return 0;
  if (dev < 0 || dev >= kMaxDevices) return 0;
  int cus = g_cus[dev].load(std::memory_order_relaxed);
  int per_cu = g_per_cu[dev][k].load(std::memory_order_relaxed);
  if (cus <= 0 || per_cu <= 0) {
    // the occupancy query answers for the current device: switch to the
    // stream's device for it and back
    int cur = -1;
    if (hipGetDevice(&cur) != hipSuccess) return 0;
    if (cur != dev && hipSetDevice(dev) != hipSuccess) return 0;
    const bool ok = hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess &&
                    hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fn, block_threads, 0) == hipSuccess;
    if (cur != dev) (void)hipSetDevice(cur);
    if (!ok) return 0;
    cus = cus > 0 ? cus : 1;
    per_cu = per_cu > 0 ? per_cu : 1;
    g_cus[dev].store(cus, std::memory_order_relaxed);
    g_per_cu[dev][k].store(per_cu, std::memory_order_relaxed);
  }
  if (cus_out) *cus_out = cus;
  uint64_t grid = uint64_t(cus) * uint64_t(per_cu);
  if (grid > n_units) grid = n_units;
  return grid ? grid : 1;
}

}  // namespace pbl

namespace {
// The big row blocks' passes (rowblk_big.hip.h): sizes before the row kernel
// (tier 1 a workgroup per PBL_BIG_WIN-block window, tier 2 over the blocks it
// listed); after it, the outputs of the blocks the row kernel did not write.
void launch_big_sizes(const pbl::Args& a, hipStream_t st, uint32_t small) {
  const uint32_t g1 = (a.in.n_blocks + PBL_BIG_WIN - 1) / PBL_BIG_WIN;
  hipLaunchKernelGGL(pbl::row::rowc::big_block_sizes_kernel, dim3(g1), dim3(pbl::kWave), 0, st, a);
  hipLaunchKernelGGL(pbl::row::rowc::big_block_sizes2_kernel, dim3(small), dim3(pbl::kWave), 0, st, a);
}

void launch_big_values(const pbl::Args& a, hipStream_t st, uint32_t small) {
  hipLaunchKernelGGL(pbl::row::rowc::big_block_values_kernel, dim3(small), dim3(pbl::kWave), 0, st, a);
}

// Row batches on the staging-pool kernel (rowblk_pool.hip.h), with the same
// big-block passes around it.
int launch_row_pool(const pbl::Args& a, hipStream_t st, bool values) {
  const uint32_t nb = a.in.n_blocks;
  const bool hide = (a.in.flags & PBL_ROW_HIDE_OBSOLETE) && !(a.in.flags & PBL_ROW_RAW_KEYS);
  const void* fn = hide ? reinterpret_cast<const void*>(pbl::row::pool::rowblk_pool_kernel<true>)
                        : reinterpret_cast<const void*>(pbl::row::pool::rowblk_pool_kernel<false>);
  int cus = 0;
  const uint64_t grid = pbl::persistent_grid(st, pbl::kKRowPool, fn,
                                             (uint64_t(nb) + pbl::row::pool::kNW - 1) / pbl::row::pool::kNW, &cus,
                                             pbl::row::pool::kTPBP);
  if (!grid) return PBL_DEVICE_ERROR;
  const uint32_t small = uint32_t(std::min<uint64_t>(nb, uint64_t(cus > 0 ? cus : 1) * 4));
  launch_big_sizes(a, st, small);
  if (hide)
    hipLaunchKernelGGL(pbl::row::pool::rowblk_pool_kernel<true>, dim3(uint32_t(grid)), dim3(pbl::row::pool::kTPBP), 0,
                       st, a, static_cast<const uint32_t*>(nullptr));
  else
    hipLaunchKernelGGL(pbl::row::pool::rowblk_pool_kernel<false>, dim3(uint32_t(grid)), dim3(pbl::row::pool::kTPBP),
                       0, st, a, static_cast<const uint32_t*>(nullptr));
  if (values) launch_big_values(a, st, small);
  return hipGetLastError() == hipSuccess ? PBL_OK : PBL_DEVICE_ERROR;
}

// Mixed batches: the ids split by format, the colblk sizes, the row kernel
// over the row ids (with the big row blocks' size / value passes around it),
// then the colblk blocks.
int launch_mixed(const pbl_block_batch* batch, const pbl::Args& a, hipStream_t st, bool values) {
  // HideObsoletePoints: colblk rows by their isObsolete bit, row entries by
  // their trailer's obsolete bit unless the keys are raw
  const bool hide = (batch->flags & PBL_ROW_HIDE_OBSOLETE) != 0;
  const bool hide_rows = hide && !(batch->flags & PBL_ROW_RAW_KEYS);
  const uint32_t nb = batch->n_blocks;
  uint8_t* ws = reinterpret_cast<uint8_t*>(a.out.workspace);
  uint32_t* ids = reinterpret_cast<uint32_t*>(ws + pbl::ws_ids_offset(nb));
  uint32_t* counts = ids + nb;
  const uint32_t nch = (nb + pbl::kSplitChunk - 1) / pbl::kSplitChunk;
  hipLaunchKernelGGL(pbl::row::mixed_split_count_kernel, dim3(nch), dim3(pbl::kTPB), 0, st, a, counts);
  hipLaunchKernelGGL(pbl::row::mixed_split_scatter_kernel, dim3(nch), dim3(pbl::kTPB), 0, st, a,
                     static_cast<const uint32_t*>(counts), nch, ids);
  int cus = 0;
  const void* cfn = hide ? reinterpret_cast<const void*>(pbl::row::mixed_col_kernel<true>)
                         : reinterpret_cast<const void*>(pbl::row::mixed_col_kernel<false>);
  const uint64_t g_c = pbl::persistent_grid(st, hide ? pbl::kKMixedColHide : pbl::kKMixedCol, cfn, nb, &cus);
  if (!g_c) return PBL_DEVICE_ERROR;
  const uint32_t small = uint32_t(std::min<uint64_t>(nb, uint64_t(cus > 0 ? cus : 1) * 4));
  const uint32_t* cids = static_cast<const uint32_t*>(ids);
  launch_big_sizes(a, st, small);
  // (3) the colblk sizes, published (the staged wave form, colblk_wave.hip.h)
  const uint32_t g_cs = uint32_t(std::min<uint64_t>(nb, uint64_t(cus > 0 ? cus : 1) * 4 * PBL_CW_SWAVES));
  if (hide)
    hipLaunchKernelGGL((pbl::col::cwave::colblk_wave_size_kernel<true, true>), dim3(g_cs), dim3(pbl::kWave), 0, st, a,
                       cids);
  else
    hipLaunchKernelGGL((pbl::col::cwave::colblk_wave_size_kernel<true, false>), dim3(g_cs), dim3(pbl::kWave), 0, st,
                       a, cids);
  // the row blocks on the staging-pool kernel, over the row id list
  const void* pfn = hide_rows ? reinterpret_cast<const void*>(pbl::row::pool::rowblk_pool_kernel<true>)
                              : reinterpret_cast<const void*>(pbl::row::pool::rowblk_pool_kernel<false>);
  const uint64_t g_p = pbl::persistent_grid(st, pbl::kKRowPool, pfn,
                                            (uint64_t(nb) + pbl::row::pool::kNW - 1) / pbl::row::pool::kNW, &cus,
                                            pbl::row::pool::kTPBP);
  if (!g_p) return PBL_DEVICE_ERROR;
  if (hide_rows)
    hipLaunchKernelGGL(pbl::row::pool::rowblk_pool_kernel<true>, dim3(uint32_t(g_p)), dim3(pbl::row::pool::kTPBP), 0,
                       st, a, cids);
  else
    hipLaunchKernelGGL(pbl::row::pool::rowblk_pool_kernel<false>, dim3(uint32_t(g_p)), dim3(pbl::row::pool::kTPBP), 0,
                       st, a, cids);
  // (5) the colblk blocks: with HideObsoletePoints the pipeline's fused form;
  // else the wave form's emit over the colblk list, whose look-back finds
  // every predecessor published (the row kernel has finished)
#ifndef PBL_MIX_COL_WAVE
#define PBL_MIX_COL_WAVE 1
#endif
  if (hide)
    hipLaunchKernelGGL(pbl::row::mixed_col_kernel<true>, dim3(uint32_t(g_c)), dim3(pbl::kTPB), 0, st, a, cids);
  else if (PBL_MIX_COL_WAVE)
    hipLaunchKernelGGL((pbl::col::cwave::colblk_wave_emit_kernel<PBL_CW_STAGE, true>), dim3(nb), dim3(pbl::kWave), 0,
                       st, a, cids);
  else
    hipLaunchKernelGGL(pbl::row::mixed_col_kernel<false>, dim3(uint32_t(g_c)), dim3(pbl::kTPB), 0, st, a, cids);
  if (values) launch_big_values(a, st, small);
  return hipGetLastError() == hipSuccess ? PBL_OK : PBL_DEVICE_ERROR;
}

// Variable-length row batches: the two-pass form (rowblk_wave.hip.h).
int launch_row_wave(const pbl::Args& a, hipStream_t st) {
  const uint32_t nb = a.in.n_blocks;
  int dev = 0, cus = 256;
  if (hipStreamGetDevice(st, &dev) != hipSuccess ||
      hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
    return PBL_DEVICE_ERROR;
  namespace cw = pbl::col::cwave;
  const uint32_t nt = (nb + cw::kScanTile - 1) / cw::kScanTile;
  hipLaunchKernelGGL(pbl::row::rwave::row_wave_size_kernel, dim3((nb + pbl::kWave - 1) / pbl::kWave),
                     dim3(pbl::kWave), 0, st, a);
  hipLaunchKernelGGL(pbl::row::rwave::row_wave_dense_kernel, dim3(std::min<uint32_t>(nb, uint32_t(cus) * 8)),
                     dim3(pbl::kWave), 0, st, a);
  hipLaunchKernelGGL(cw::bases_scan_kernel<true>, dim3(std::min<uint32_t>(nt, uint32_t(cus) * 2)), dim3(pbl::kTPB), 0,
                     st, a);
  hipLaunchKernelGGL(pbl::row::rwave::row_wave_emit_kernel, dim3(nb), dim3(pbl::row::rwave::kRwWaves * pbl::kWave), 0,
                     st, a);
  return hipGetLastError() == hipSuccess ? PBL_OK : PBL_DEVICE_ERROR;
}

// A single-format row batch: the staging-pool kernel, or with
// PBL_BATCH_VARLEN the two-pass form (PBL_KERNEL_POOL forces the pool).
int launch_row(const pbl::Args& a, hipStream_t st, bool values) {
  const uint32_t f = a.in.flags;
  if ((f & PBL_BATCH_VARLEN) && !(f & PBL_KERNEL_POOL) && pbl::row::rwave::sizes_without_keys(f))
    return launch_row_wave(a, st);
  return launch_row_pool(a, st, values);
}
}  // namespace

extern "C" {

int pbl_abi_version(void) { return PBL_ABI_VERSION; }

uint64_t pbl_workspace_bytes(uint32_t n_blocks) { return pbl::ws_alloc_bytes(n_blocks); }

int pbl_decode_batch_colblk(const pbl_block_batch* batch, pbl_decode_out* out, void* stream);

int pbl_decode_batch(const pbl_block_batch* batch, pbl_decode_out* out, void* stream) {
  if (!batch || !out || (batch->synthetic_seq_num >> 56)) return PBL_INVALID_ARG;  // (base.SeqNumMax)
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (!out->totals || !out->blk_kv_base || !out->blk_key_base || !out->blk_val_base || !out->blk_status)
    return PBL_INVALID_ARG;
  if (hipMemsetAsync(out->totals, 0, sizeof(pbl_totals), st) != hipSuccess) return PBL_DEVICE_ERROR;
  if (batch->n_blocks == 0) return PBL_OK;
  if (!batch->blocks || !batch->block_off || !batch->block_len || !out->trailer || !out->key_off ||
      !out->val_off || !out->key_bytes || !out->val_bytes || !out->workspace ||
      out->workspace_bytes < pbl::ws_alloc_bytes(batch->n_blocks) || (!out->tiering_span_id != !out->tiering_attr))
    return PBL_INVALID_ARG;
  if (!batch->block_format && batch->format != PBL_FMT_ROW) return pbl_decode_batch_colblk(batch, out, stream);
  if (hipMemsetAsync(out->workspace, 0, pbl::ws_bytes(batch->n_blocks), st) != hipSuccess)
    return PBL_DEVICE_ERROR;
  pbl::Args a;
  a.in = *batch;
  a.out = *out;
  const int rc = batch->block_format ? launch_mixed(batch, a, st, true) : launch_row(a, st, true);
  if (rc != PBL_OK || !out->tiering_span_id) return rc;
  const uint32_t g = batch->n_blocks < 8192 ? batch->n_blocks : 8192;
  hipLaunchKernelGGL(pbl::row::row_meta_zero_kernel, dim3(g), dim3(pbl::kWave), 0, st, a);
  return hipGetLastError() == hipSuccess ? PBL_OK : PBL_DEVICE_ERROR;
}

int pbl_size_batch(const pbl_block_batch* batch, pbl_decode_out* out, void* stream) {
  if (!batch || !out || (batch->synthetic_seq_num >> 56)) return PBL_INVALID_ARG;
  if (!out->totals || !out->blk_kv_base || !out->blk_key_base || !out->blk_val_base || !out->blk_status)
    return PBL_INVALID_ARG;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (batch->n_blocks == 0) return pbl_decode_batch(batch, out, stream);
  if (!batch->blocks || !batch->block_off || !batch->block_len || !out->workspace ||
      out->workspace_bytes < pbl::ws_alloc_bytes(batch->n_blocks))
    return PBL_INVALID_ARG;
  // the decode with every per-KV pointer NULL and zero capacities: each block
  // takes its overflow branch (sizes computed and published, nothing written);
  // the fixup then reports the statuses the decode would have had
  pbl_decode_out o = *out;
  o.trailer = nullptr;
  o.kv_flags = nullptr;
  o.entry_off = nullptr;
  o.key_off = nullptr;
  o.val_off = nullptr;
  o.key_bytes = nullptr;
  o.val_bytes = nullptr;
  o.restarts = nullptr;
  o.tiering_span_id = nullptr;
  o.tiering_attr = nullptr;
  o.kv_cap = o.key_cap = o.val_cap = o.rst_cap = 0;
  if (hipMemsetAsync(o.totals, 0, sizeof(pbl_totals), st) != hipSuccess) return PBL_DEVICE_ERROR;
  if (hipMemsetAsync(o.workspace, 0, pbl::ws_bytes(batch->n_blocks), st) != hipSuccess) return PBL_DEVICE_ERROR;
  pbl::Args a;
  a.in = *batch;
  a.out = o;
  int rc = PBL_OK;
  if (!batch->block_format && batch->format != PBL_FMT_ROW) {
    rc = pbl_decode_batch_colblk(batch, &o, stream);
  } else {
    // the launch sequence of pbl_decode_batch (whose checks require output
    // pointers), minus the big-block value pass
    rc = batch->block_format ? launch_mixed(batch, a, st, false) : launch_row(a, st, false);
  }
  if (rc != PBL_OK) return rc;
  hipLaunchKernelGGL(pbl::row::size_fixup_kernel, dim3((batch->n_blocks + 255) / 256), dim3(256), 0, st,
                     o.blk_status, o.totals, batch->n_blocks);
  return hipGetLastError() == hipSuccess ? PBL_OK : PBL_DEVICE_ERROR;
}

size_t pbl_struct_layout(uint64_t* out, size_t cap) {
#define PBL_OFF(T, f) uint64_t(offsetof(T, f))
  const uint64_t v[] = {
      sizeof(pbl_block_batch), PBL_OFF(pbl_block_batch, blocks), PBL_OFF(pbl_block_batch, block_off),
      PBL_OFF(pbl_block_batch, block_len), PBL_OFF(pbl_block_batch, n_blocks), PBL_OFF(pbl_block_batch, format),
      PBL_OFF(pbl_block_batch, flags), PBL_OFF(pbl_block_batch, reserved), PBL_OFF(pbl_block_batch, block_format),
      PBL_OFF(pbl_block_batch, synthetic_seq_num),
      sizeof(pbl_totals), PBL_OFF(pbl_totals, n_kv), PBL_OFF(pbl_totals, key_bytes), PBL_OFF(pbl_totals, val_bytes),
      PBL_OFF(pbl_totals, n_restarts), PBL_OFF(pbl_totals, status_mask), PBL_OFF(pbl_totals, n_bad_blocks),
      PBL_OFF(pbl_totals, n_slow_blocks), PBL_OFF(pbl_totals, pad),
      sizeof(pbl_decode_out), PBL_OFF(pbl_decode_out, trailer), PBL_OFF(pbl_decode_out, kv_flags),
      PBL_OFF(pbl_decode_out, entry_off), PBL_OFF(pbl_decode_out, key_off), PBL_OFF(pbl_decode_out, val_off),
      PBL_OFF(pbl_decode_out, key_bytes), PBL_OFF(pbl_decode_out, val_bytes), PBL_OFF(pbl_decode_out, restarts),
      PBL_OFF(pbl_decode_out, blk_kv_base), PBL_OFF(pbl_decode_out, blk_key_base),
      PBL_OFF(pbl_decode_out, blk_val_base), PBL_OFF(pbl_decode_out, blk_rst_base),
      PBL_OFF(pbl_decode_out, blk_status), PBL_OFF(pbl_decode_out, totals), PBL_OFF(pbl_decode_out, kv_cap),
      PBL_OFF(pbl_decode_out, key_cap), PBL_OFF(pbl_decode_out, val_cap), PBL_OFF(pbl_decode_out, rst_cap),
      PBL_OFF(pbl_decode_out, workspace), PBL_OFF(pbl_decode_out, workspace_bytes),
      PBL_OFF(pbl_decode_out, tiering_span_id), PBL_OFF(pbl_decode_out, tiering_attr),
      sizeof(pbl_transforms), PBL_OFF(pbl_transforms, synthetic_seq_num),
      PBL_OFF(pbl_transforms, hide_obsolete_points), PBL_OFF(pbl_transforms, split), PBL_OFF(pbl_transforms, prefix),
      PBL_OFF(pbl_transforms, suffix), PBL_OFF(pbl_transforms, prefix_len), PBL_OFF(pbl_transforms, suffix_len),
      PBL_OFF(pbl_transforms, blocks),
      sizeof(pbl_footer), PBL_OFF(pbl_footer, table_format), PBL_OFF(pbl_footer, checksum_type),
      PBL_OFF(pbl_footer, metaindex_off), PBL_OFF(pbl_footer, metaindex_len), PBL_OFF(pbl_footer, index_off),
      PBL_OFF(pbl_footer, index_len), PBL_OFF(pbl_footer, footer_off), PBL_OFF(pbl_footer, footer_len),
      PBL_OFF(pbl_footer, attributes), PBL_OFF(pbl_footer, reserved),
      sizeof(pbl_index_out), PBL_OFF(pbl_index_out, handle_off), PBL_OFF(pbl_index_out, handle_len),
      PBL_OFF(pbl_index_out, props_off), PBL_OFF(pbl_index_out, props_len), PBL_OFF(pbl_index_out, blk_base),
      PBL_OFF(pbl_index_out, blk_status), PBL_OFF(pbl_index_out, cap),
      sizeof(pbl_kv_out), PBL_OFF(pbl_kv_out, key_off), PBL_OFF(pbl_kv_out, key_len), PBL_OFF(pbl_kv_out, val_off),
      PBL_OFF(pbl_kv_out, val_len), PBL_OFF(pbl_kv_out, blk_base), PBL_OFF(pbl_kv_out, blk_status),
      PBL_OFF(pbl_kv_out, cap),
      sizeof(pbl_value_out), PBL_OFF(pbl_value_out, val_off), PBL_OFF(pbl_value_out, val_bytes),
      PBL_OFF(pbl_value_out, blk_val_base), PBL_OFF(pbl_value_out, blk_status), PBL_OFF(pbl_value_out, val_cap),
      sizeof(pbl_kv), PBL_OFF(pbl_kv, user_key), PBL_OFF(pbl_kv, user_key_len), PBL_OFF(pbl_kv, trailer),
      PBL_OFF(pbl_kv, value), PBL_OFF(pbl_kv, value_len), PBL_OFF(pbl_kv, kv_flags), PBL_OFF(pbl_kv, reserved),
      sizeof(pbl_kv_meta), PBL_OFF(pbl_kv_meta, tiering_span_id), PBL_OFF(pbl_kv_meta, tiering_attribute)};
#undef PBL_OFF
  const size_t n = sizeof(v) / sizeof(v[0]);
  for (size_t i = 0; i < n && i < cap && out; i++) out[i] = v[i];
  return n;
}

int pbl_rebase_blocks(pbl_decode_out* out, uint32_t n_blocks, uint64_t kv_base, uint64_t key_base,
                      uint64_t val_base, uint64_t rst_base, void* stream) {
  if (!out || !out->blk_kv_base || !out->blk_key_base || !out->blk_val_base) return PBL_INVALID_ARG;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  uint32_t n = n_blocks + 1;
  hipLaunchKernelGGL(pbl::row::rebase_kernel, dim3((n + 255) / 256), dim3(256), 0, st, out->blk_kv_base,
                     out->blk_key_base, out->blk_val_base, out->blk_rst_base, n_blocks, kv_base, key_base,
                     val_base, rst_base);
  return hipGetLastError() == hipSuccess ? PBL_OK : PBL_DEVICE_ERROR;
}

int pbl_offset_concat(pbl_decode_out* out, uint32_t n_blocks, const uint64_t* rank_totals, uint32_t rank,
                      void* stream) {
  if (!out || !rank_totals || !out->blk_kv_base || !out->blk_key_base || !out->blk_val_base)
    return PBL_INVALID_ARG;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  uint32_t n = n_blocks + 1;
  uint32_t grid = (n + 255) / 256;
  if (grid > 1024) grid = 1024;
  hipLaunchKernelGGL(pbl::row::offset_concat_kernel, dim3(grid), dim3(256), 0, st, out->blk_kv_base,
                     out->blk_key_base, out->blk_val_base, out->blk_rst_base, n_blocks, rank_totals, rank);
  return hipGetLastError() == hipSuccess ? PBL_OK : PBL_DEVICE_ERROR;
}

}  // extern "C"
