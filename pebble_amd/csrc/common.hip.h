// common.hip.h — shared device helpers for the gfx950 block decoders:
// wave/block scans and the decoupled look-back that places every block's
// outputs in ONE pass (no separate size pass).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/pebble_amd.h"

namespace pbl {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));  // native 16-B vector
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));  // native 8-B vector

constexpr int kTPB = 256;   // threads per workgroup (4 waves); one workgroup per block
constexpr int kWave = 64;
constexpr int kNumComp = 4; // look-back components: n_kv, key bytes, value bytes, restarts
#ifndef PBL_LB_WIN
#define PBL_LB_WIN 2
#endif
// Look-back windows (of 64 predecessors) loaded per round trip.  Fewer windows
// mean more round trips on a long walk but a smaller, lower-pressure resolve
// (it is inlined into every persistent kernel): measured on the MI355X (config
// 2 / 3 / 4 GiB/s) 8 windows 972 / 1199 / 857, 4: 999 / - / -, 2: 1036 / 1270
// / 893, 1: 1035 / 1228 / -.
constexpr int kLbWin = PBL_LB_WIN;

// ---- workspace layout ------------------------------------------------------
// [0,256): ticket counter (u32 [0]), big-block count (u32 [1], row pipeline), pad.  Then
//   rec[n_blocks]             one 16-B record per block {w0, w1}, each 8-B half
//                             self-tagged with a 3-bit state (top bits):
//                               w0 = Agg | packed aggregate (4 counts), or
//                               w0 = Wide (aggregate too wide: in wide[]), or
//                               w0 = Pfx | (n_kv:31 | key:30), w1 = Pfx | (val:37 | rst:24)
//                                    (packed INCLUSIVE prefix), or
//                               w0 = PfxWide (inclusive prefix too wide: in pfx[])
//   pfx[kNumComp][n_blocks]   wide inclusive prefixes {state | value}
//   wide[kNumComp][n_blocks]  wide aggregates {state | value}
// All written and read with agent-scope relaxed 8-byte atomics (sc1): each word
// carries its own state, so a reader that sees a record before the words it
// announces simply polls those (no fences; MI355X_MICROARCH.md "Valid forms",
// R2 granules).  A resolve normally costs ONE round trip: the windows of
// predecessor records carry packed inclusive prefixes, so the nearest one ends
// the walk without a second fetch.
constexpr uint64_t kKindInvalidTrailer = 191u;  // base.InternalKeyKindInvalid, seq 0

// blockiter.SyntheticSeqNum fused into the decode (pbl_block_batch.
// synthetic_seq_num, 0 = unset): SetSeqNum on every decodable key after the
// obsolete bit is masked (rowblk_iter.go:1168-1191; colblk data_block.go:
// 1693-1695).  An invalid row key keeps the Invalid trailer (its kind byte has
// bit 7 set, which no masked trailer has); raw-key batches carry no seqnums.
__device__ __forceinline__ uint64_t with_seq(uint64_t tr, uint64_t seq, uint32_t flags) {
  return (seq && !(flags & PBL_ROW_RAW_KEYS) && tr != kKindInvalidTrailer) ? (seq << 8) | (tr & 0xff) : tr;
}

constexpr uint64_t kWsHeader = 256;
constexpr int kWsColTick = 2;   // header u32 [2]: the colblk queue's ticket counter (mixed batches)
constexpr int kWsRowCount = 3;  // header u32 [3]: row-format blocks in a mixed batch
constexpr uint32_t kSplitChunk = 4096;  // blocks per chunk of the mixed-batch split
constexpr int kStShift = 61;
constexpr uint64_t kStAgg = 1ull << kStShift;
constexpr uint64_t kStWide = 2ull << kStShift;
constexpr uint64_t kStPfx = 3ull << kStShift;
constexpr uint64_t kStPfxWide = 4ull << kStShift;
constexpr uint64_t kStMask = 7ull << kStShift;
constexpr uint64_t kValMask = (1ull << kStShift) - 1;
// packed aggregate fields (w0 of an Agg record): n_kv 14 | key bytes 18 | value bytes 18 | restarts 11
constexpr int kPkBits[kNumComp] = {14, 18, 18, 11};
constexpr int kPkShift[kNumComp] = {0, 14, 32, 50};
// packed inclusive prefix: w0 = n_kv 31 | key 30, w1 = val 37 | rst 24
constexpr int kPfBits[kNumComp] = {31, 30, 37, 24};

__host__ __device__ inline uint64_t ws_bytes(uint32_t n_blocks) {
  return kWsHeader + uint64_t(2 + 2 * kNumComp) * n_blocks * 8ull;
}
// Two-pass forms (a size pass, the bases scan, then the outputs): per-block
// restart counts, scanned in place into restart bases ([n_blocks] = total).
// The last n_blocks + 1 words of the look-back area, which the scan's own
// per-tile look-back (n_blocks / 1024 records) never reaches.
__host__ __device__ inline uint64_t ws_rcnt_offset(uint32_t n_blocks) {
  return ws_bytes(n_blocks) - 8ull * (n_blocks + 1);
}
#ifdef PBL_STAMPS
constexpr uint64_t kStampWords = 16;  // diagnostic build: per-block phase stamps
#else
constexpr uint64_t kStampWords = 0;
#endif
// Past the look-back state (and the diagnostic stamps): a mixed batch's block
// ids split by format (row ids ascending, then colblk ids ascending) and the
// split's per-chunk row counts.  Not cleared per launch.
__host__ __device__ inline uint64_t ws_ids_offset(uint32_t n_blocks) {
  return ws_bytes(n_blocks) + kStampWords * 8ull * n_blocks;
}
// Then the big row blocks' lists (rowblk_big.hip.h): the sizes pass's tier-2
// list (count at header word 5); the blocks the row kernel's own walk left
// (count at word 6), for the values pass.
__host__ __device__ inline uint64_t ws_redo_offset(uint32_t n_blocks) {
  return ws_ids_offset(n_blocks) + 4ull * n_blocks + 4ull * (n_blocks / kSplitChunk + 1) + 8;
}
__host__ __device__ inline uint64_t ws_pend_offset(uint32_t n_blocks) { return ws_redo_offset(n_blocks) + 4ull * n_blocks; }
// Then the entry offsets of the two-pass row form (rowblk_wave.hip.h): the
// first kEntRec entries' block offsets per block, u16 (blocks <= 32 KiB).
constexpr uint32_t kEntRec = 64;
__host__ __device__ inline uint64_t ws_ent_offset(uint32_t n_blocks) {
  return (ws_pend_offset(n_blocks) + 4ull * n_blocks + 15) & ~uint64_t(15);
}
__host__ __device__ inline uint64_t ws_alloc_bytes(uint32_t n_blocks) {
  return ws_ent_offset(n_blocks) + 2ull * kEntRec * n_blocks;
}


// Address-space-typed pointers.  A generic pointer compiles to FLAT
// instructions, which count against BOTH vmcnt and lgkmcnt: an LDS read issued
// after a FLAT store or load then waits for that global access (HBM latency)
// before it can be consumed.  Every hot-path access goes through one of these.
template <class T>
using gptr = __attribute__((address_space(1))) T*;
template <class T>
using lptr = __attribute__((address_space(3))) T*;
template <class T>
__device__ __forceinline__ gptr<T> to_glb(T* p) {
  return (gptr<T>)p;
}
template <class T>
__device__ __forceinline__ lptr<T> to_lds_ptr(T* p) {
  return (lptr<T>)p;
}

// device-scope atomics on global memory (global_atomic_*, never FLAT)
__device__ inline uint32_t g_atomic_add(uint32_t* p, uint32_t v) {
  return __hip_atomic_fetch_add(to_glb(p), v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ inline uint32_t g_atomic_or(uint32_t* p, uint32_t v) {
  return __hip_atomic_fetch_or(to_glb(p), v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// A persistent kernel's source of blocks.  take() returns a block id, or
// n_blocks when the queue is drained.  TicketQueue: tickets are block ids (the
// single-format kernels); ListQueue: tickets index an id list (a mixed batch's
// per-format list).  Separate types keep the list indirection out of the
// single-format kernels' code.
struct TicketQueue {
  uint32_t* tick;
  uint32_t n_blocks;
  __device__ uint32_t take() const {
    const uint32_t t = g_atomic_add(tick, 1u);
    return t < n_blocks ? t : n_blocks;
  }
};
struct ListQueue {
  uint32_t* tick;
  const uint32_t* ids;
  uint32_t n;         // tickets in this queue
  uint32_t n_blocks;  // the sentinel
  __device__ uint32_t take() const {
    const uint32_t t = g_atomic_add(tick, 1u);
    return t < n ? to_glb(ids)[t] : n_blocks;
  }
};

__device__ inline uint64_t ld_agent(const uint64_t* p) {
  return __hip_atomic_load(to_glb(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ inline void st_agent(uint64_t* p, uint64_t v) {
  __hip_atomic_store(to_glb(p), v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ inline int lane_id() { return threadIdx.x & (kWave - 1); }
__device__ inline int wave_id() { return threadIdx.x >> 6; }

// In-wave ordering of LDS traffic between lanes (no workgroup barrier).
__device__ inline void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

template <typename T>
__device__ inline T wave_incl_scan(T v) {
  const int l = lane_id();
#pragma unroll
  for (int d = 1; d < kWave; d <<= 1) {
    T o = __shfl_up(v, d, kWave);
    if (l >= d) v += o;
  }
  return v;
}
template <typename T>
__device__ inline T wave_sum(T v) {
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) v += __shfl_xor(v, d, kWave);
  return v;
}

// Block-wide exclusive scan of two u32 sequences (one value each per thread).
// `scratch` must hold 2*(kTPB/kWave) u32.  Caller must __syncthreads() before
// reusing scratch.
__device__ inline void block_excl_scan2(uint32_t a, uint32_t b, uint32_t* ea, uint32_t* eb,
                                        uint32_t* scratch, uint32_t* tot_a, uint32_t* tot_b) {
  uint32_t ia = wave_incl_scan(a), ib = wave_incl_scan(b);
  const int w = wave_id(), l = lane_id();
  if (l == kWave - 1) { scratch[w] = ia; scratch[4 + w] = ib; }
  __syncthreads();
  uint32_t pa = 0, pb = 0, ta = 0, tb = 0;
#pragma unroll
  for (int i = 0; i < kTPB / kWave; i++) {
    uint32_t sa = scratch[i], sb = scratch[4 + i];
    if (i < w) { pa += sa; pb += sb; }
    ta += sa; tb += sb;
  }
  *ea = pa + ia - a;
  *eb = pb + ib - b;
  *tot_a = ta;
  *tot_b = tb;
}

// Stage n16 16-byte granules src[0, n16) (global, 16-B aligned) into LDS
// dst[0, n16) by LDS-DMA (global_load_lds_dwordx4: no registers, every granule
// in flight at once), then wait for them.  One wave; lanes past n16 are masked
// off (nothing lands past the stage).  A register round trip per granule
// (load, wait, ds_write) serialises the block's HBM latency instead.
__device__ inline void lds_stage16(lptr<u32x4> dst, gptr<const u32x4> src, uint32_t n16) {
  const uint32_t l = lane_id();
  for (uint32_t g0 = 0; g0 < n16; g0 += kWave) {
    if (g0 + l < n16)
      __builtin_amdgcn_global_load_lds((gptr<const void>)(src + (g0 + l)), (lptr<void>)(dst + g0), 16, 0, 0);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  wave_sync();
}

// Decoupled look-back (single-pass scan across blocks), in two halves so a
// workgroup can publish its aggregate as soon as it is known and resolve its
// exclusive prefix later.  Tickets are handed out in launch order, so every
// predecessor is resident and publishes its aggregate before it waits: no
// deadlock for any residency.  Both halves run on one wave of the workgroup
// that owns virtual block `v`; `st` is the workspace after its header.
__device__ inline bool agg_packable(const uint64_t agg[kNumComp]) {
  return agg[0] < (1ull << kPkBits[0]) && agg[1] < (1ull << kPkBits[1]) && agg[2] < (1ull << kPkBits[2]) &&
         agg[3] < (1ull << kPkBits[3]);
}
__device__ inline bool pfx_packable(const uint64_t p[kNumComp]) {
  return p[0] < (1ull << kPfBits[0]) && p[1] < (1ull << kPfBits[1]) && p[2] < (1ull << kPfBits[2]) &&
         p[3] < (1ull << kPfBits[3]);
}

struct LbPtrs {
  uint64_t* rec;   // [2 * n_blocks]
  uint64_t* pfx;   // [kNumComp * n_blocks]
  uint64_t* wide;  // [kNumComp * n_blocks]
  __device__ LbPtrs(uint64_t* st, uint32_t n_blocks)
      : rec(st), pfx(st + 2ull * n_blocks), wide(st + 2ull * n_blocks + uint64_t(kNumComp) * n_blocks) {}
};

// Store block v's inclusive prefix `p` (lanes 0-3 of the calling wave).
__device__ inline void lb_store_pfx(const LbPtrs& P, uint32_t n_blocks, uint32_t v, const uint64_t p[kNumComp]) {
  const int l = lane_id();
  if (pfx_packable(p)) {
    if (l == 0) {
      // w1 first: a reader that sees w0's Pfx before w1's polls w1
      st_agent(P.rec + 2ull * v + 1, kStPfx | p[2] | (p[3] << kPfBits[2]));
      st_agent(P.rec + 2ull * v, kStPfx | p[0] | (p[1] << kPfBits[0]));
    }
  } else {
    if (l < kNumComp) {
      const uint64_t x = l == 0 ? p[0] : l == 1 ? p[1] : l == 2 ? p[2] : p[3];
      st_agent(P.pfx + uint64_t(l) * n_blocks + v, kStPfxWide | (x & kValMask));
    }
    if (l == 0) st_agent(P.rec + 2ull * v, kStPfxWide);
  }
}

__device__ inline void lb_publish(uint64_t* st, uint32_t n_blocks, uint32_t v, const uint64_t agg[kNumComp]) {
  const int l = lane_id();
  const LbPtrs P(st, n_blocks);
  if (v == 0) {  // block 0: its inclusive prefix IS its aggregate
    lb_store_pfx(P, n_blocks, v, agg);
    return;
  }
  if (agg_packable(agg)) {
    if (l == 0) {
      uint64_t packed = 0;
      for (int c = 0; c < kNumComp; c++) packed |= agg[c] << kPkShift[c];
      st_agent(P.rec + 2ull * v, kStAgg | packed);
    }
  } else {
    // wide aggregates go to their own slots (the record announces them)
    if (l < kNumComp) {
      const uint64_t a = l == 0 ? agg[0] : l == 1 ? agg[1] : l == 2 ? agg[2] : agg[3];
      st_agent(P.wide + uint64_t(l) * n_blocks + v, kStWide | (a & kValMask));
    }
    if (l == 0) st_agent(P.rec + 2ull * v, kStWide);
  }
}

// Poll one word until its state is `want` (single lane); returns the payload.
__device__ inline uint64_t lb_poll(uint64_t* p, uint64_t want, uint32_t* spins, bool* timed_out) {
  uint64_t x;
  while (((x = ld_agent(p)) & kStMask) != want) {
    if (++*spins > (1u << 22)) { *timed_out = true; return 0; }
    __builtin_amdgcn_s_sleep(2);
  }
  return x & kValMask;
}

// The 4 component words at src[q * n + idx] in one round trip (loads issued
// together), each polled on its own only if it is not ready yet.
__device__ inline void lb_fetch4(uint64_t* src, uint32_t n_blocks, int64_t idx, uint64_t want, uint64_t c[kNumComp],
                                 uint32_t* spins, bool* timed_out) {
  uint64_t x[kNumComp];
#pragma unroll
  for (int q = 0; q < kNumComp; q++) x[q] = ld_agent(src + uint64_t(q) * n_blocks + idx);
#pragma unroll
  for (int q = 0; q < kNumComp; q++)
    c[q] = (x[q] & kStMask) == want ? (x[q] & kValMask)
                                    : lb_poll(src + uint64_t(q) * n_blocks + idx, want, spins, timed_out);
}

// Windows of predecessor records loaded in one round trip: lane l of window k
// holds rec[top - 64k - l] (w0 and w1).
template <int W>
struct LbWindows {
  uint64_t w0[W], w1[W];
  int64_t top;
  __device__ inline void issue(const LbPtrs& P, int64_t top_) {
    top = top_;
    const int l = lane_id();
#pragma unroll
    for (int k = 0; k < W; k++) {
      const int64_t idx = top - kWave * k - l;
      w0[k] = idx >= 0 ? ld_agent(P.rec + 2 * idx) : kStPfx;  // (index -1 acts as a zero prefix)
      w1[k] = idx >= 0 ? ld_agent(P.rec + 2 * idx + 1) : kStPfx;
    }
  }
};

// Consume loaded windows: accumulate per-lane partial sums into acc.  Returns
// true when the walk reached an inclusive prefix; otherwise *next_top is where
// to continue and *wait_idx >= 0 names a predecessor that has not published.
template <int W>
__device__ inline bool lb_consume(const LbPtrs& P, uint32_t n_blocks, const LbWindows<W>& G, uint64_t acc[kNumComp],
                                  int64_t* next_top, int64_t* wait_idx, uint32_t* spins, bool* timed_out) {
  const int l = lane_id();
  int64_t top = G.top;
  *wait_idx = -1;
#pragma unroll
  for (int k = 0; k < W; k++) {
    const int64_t idx = G.top - kWave * k - l;
    const uint64_t state = G.w0[k] & kStMask;
    const bool is_pfx = state == kStPfx || state == kStPfxWide;
    const uint64_t pfxm = __ballot(is_pfx);
    const uint64_t notready = __ballot(state == 0);
    const int first = pfxm ? __builtin_ctzll(pfxm) : 64;
    const uint64_t need = first >= 63 ? ~0ull : ((2ull << first) - 1);
    if (notready & need) {
      *wait_idx = G.top - kWave * k - __builtin_ctzll(notready & need);
      *next_top = top;
      return false;
    }
    uint64_t c[kNumComp] = {0, 0, 0, 0};
    if (l < first && state == kStAgg) {
#pragma unroll
      for (int q = 0; q < kNumComp; q++) c[q] = (G.w0[k] >> kPkShift[q]) & ((1ull << kPkBits[q]) - 1);
    }
    if (l < first && state == kStWide) lb_fetch4(P.wide, n_blocks, idx, kStWide, c, spins, timed_out);
    if (l == first && idx >= 0) {
      if (state == kStPfx) {
        uint64_t w1 = G.w1[k];
        if ((w1 & kStMask) != kStPfx) w1 = kStPfx | lb_poll(P.rec + 2 * idx + 1, kStPfx, spins, timed_out);
        c[0] = G.w0[k] & ((1ull << kPfBits[0]) - 1);
        c[1] = (G.w0[k] >> kPfBits[0]) & ((1ull << kPfBits[1]) - 1);
        c[2] = w1 & ((1ull << kPfBits[2]) - 1);
        c[3] = (w1 >> kPfBits[2]) & ((1ull << kPfBits[3]) - 1);
      } else {
        lb_fetch4(P.pfx, n_blocks, idx, kStPfxWide, c, spins, timed_out);
      }
    }
    // per-lane partial sums; the cross-lane reduction happens once, at the end
#pragma unroll
    for (int q = 0; q < kNumComp; q++) acc[q] += c[q];
    if (first < 64) return true;
    top -= kWave;
  }
  *next_top = top;
  return false;
}

// Finish a resolve whose first windows (from v-1 down) are already loaded.
template <int W>
__device__ inline void lb_finish(uint64_t* st, uint32_t n_blocks, uint32_t v, const uint64_t agg[kNumComp],
                                 uint64_t excl[kNumComp], uint32_t* timeout_flag, const LbWindows<W>& first_win) {
  const int l = lane_id();
  const LbPtrs P(st, n_blocks);
  uint64_t acc[kNumComp] = {0, 0, 0, 0};
  uint32_t spins = 0;
  bool timed_out = false;
  int64_t top = int64_t(v) - 1, wait_idx = -1;
  bool done = v == 0 || lb_consume(P, n_blocks, first_win, acc, &top, &wait_idx, &spins, &timed_out);
  // a lane polling a wide record may have timed out on its own: leave together
  if (__ballot(timed_out)) timed_out = true;
  while (!done && !timed_out) {
    if (wait_idx >= 0) {
      // Poll the missing predecessor from ONE lane (a whole-window re-read per
      // poll would flood this CU's memory queue), then re-read the windows.
      if (l == 0) {
        while ((ld_agent(P.rec + 2 * wait_idx) & kStMask) == 0) {
          if (++spins > (1u << 22)) { timed_out = true; break; }
          __builtin_amdgcn_s_sleep(2);
        }
      }
      if (__shfl(timed_out ? 1 : 0, 0, kWave)) { timed_out = true; break; }
    }
    LbWindows<W> G;
    G.issue(P, top);
    done = lb_consume(P, n_blocks, G, acc, &top, &wait_idx, &spins, &timed_out);
    if (__ballot(timed_out)) timed_out = true;
  }
  if (timed_out && l == 0) g_atomic_or(timeout_flag, 1u << PBL_TIMEOUT);
#pragma unroll
  for (int q = 0; q < kNumComp; q++) excl[q] = wave_sum(acc[q]);
  if (v > 0) {
    uint64_t p[kNumComp];
#pragma unroll
    for (int q = 0; q < kNumComp; q++) p[q] = excl[q] + agg[q];
    lb_store_pfx(P, n_blocks, v, p);
  }
}

template <int W = kLbWin>
__device__ inline void lb_resolve(uint64_t* st, uint32_t n_blocks, uint32_t v, const uint64_t agg[kNumComp],
                                  uint64_t excl[kNumComp], uint32_t* timeout_flag) {
  LbWindows<W> G;
  if (v > 0) G.issue(LbPtrs(st, n_blocks), int64_t(v) - 1);
  lb_finish(st, n_blocks, v, agg, excl, timeout_flag, G);
}

__device__ inline void lookback(uint64_t* st, uint32_t n_blocks, uint32_t v, const uint64_t agg[kNumComp],
                                uint64_t excl[kNumComp], uint32_t* timeout_flag) {
  lb_publish(st, n_blocks, v, agg);
  lb_resolve(st, n_blocks, v, agg, excl, timeout_flag);
}

// ---- shared by the row and colblk decoders --------------------------------
struct Args {
  pbl_block_batch in;
  pbl_decode_out out;
};

// Store 16 bytes (w) covering global bytes [ga, ga+16) of which only [lo, hi)
// belong to this block: one dwordx4 store when whole, byte stores at the edges.
// PBL_STORE16_NT: whole granules as non-temporal stores (the outputs stream
// past the L2 lines of blocks still being read).
#ifndef PBL_STORE16_NT
#define PBL_STORE16_NT 1  // measured: config 3 1275 vs 1250 GiB/s
#endif
__device__ inline void store16(uint8_t* base_, uint64_t ga, uint64_t lo, uint64_t hi, uint4 w) {
  const gptr<uint8_t> base = to_glb(base_);
  if (ga >= lo && ga + 16 <= hi) {
#if PBL_STORE16_NT
    __builtin_nontemporal_store(u32x4{w.x, w.y, w.z, w.w}, (gptr<u32x4>)(base + ga));
#else
    *(gptr<u32x4>)(base + ga) = u32x4{w.x, w.y, w.z, w.w};
#endif
    return;
  }
#pragma unroll
  for (int i = 0; i < 16; i++) {
    uint32_t word = i < 4 ? w.x : i < 8 ? w.y : i < 12 ? w.z : w.w;
    if (ga + i >= lo && ga + i < hi) base[ga + i] = uint8_t(word >> (8 * (i & 3)));
  }
}

// Per-block results and batch totals, written by lane 0 of wave 0.
__device__ inline void write_block_meta(const pbl_decode_out& O, uint32_t b, uint32_t nb, uint32_t status,
                                        const uint64_t excl[kNumComp], const uint64_t agg[kNumComp],
                                        bool slow) {
  to_glb(O.blk_kv_base)[b] = excl[0];
  to_glb(O.blk_key_base)[b] = excl[1];
  to_glb(O.blk_val_base)[b] = excl[2];
  if (O.blk_rst_base) to_glb(O.blk_rst_base)[b] = excl[3];
  to_glb(O.blk_status)[b] = status;
  gptr<pbl_totals> T = to_glb(O.totals);
  if (slow) g_atomic_add(&O.totals->n_slow_blocks, 1u);
  if (status != PBL_OK) {
    g_atomic_or(&O.totals->status_mask, 1u << status);
    g_atomic_add(&O.totals->n_bad_blocks, 1u);
  }
  if (b == nb - 1) {
    to_glb(O.blk_kv_base)[nb] = excl[0] + agg[0];
    to_glb(O.blk_key_base)[nb] = excl[1] + agg[1];
    to_glb(O.blk_val_base)[nb] = excl[2] + agg[2];
    if (O.blk_rst_base) to_glb(O.blk_rst_base)[nb] = excl[3] + agg[3];
    T->n_kv = excl[0] + agg[0];
    T->key_bytes = excl[1] + agg[1];
    T->val_bytes = excl[2] + agg[2];
    T->n_restarts = excl[3] + agg[3];
  }
}

// (a size pass, pbl_size_batch, passes key_off = NULL: every block "overflows",
// so sizes are computed and nothing is written)
__device__ inline bool overflows(const pbl_decode_out& O, const uint64_t excl[kNumComp],
                                 const uint64_t agg[kNumComp]) {
  return !O.key_off || excl[0] + agg[0] > O.kv_cap || excl[1] + agg[1] > O.key_cap || excl[2] + agg[2] > O.val_cap ||
         (O.restarts && excl[3] + agg[3] > O.rst_cap);
}

// ---- host side: persistent-grid sizing ----------------------------------------
// The device of a launch is the device of its stream (hipStreamGetDevice), not
// the calling thread's current device.  The CU count and each persistent
// kernel's resident workgroups per CU are hardware properties of that device:
// they are queried once and cached (the library's only process-wide state, and
// immutable once written; racing first calls store the same values).
enum PersistentKernel { kKColPipe = 0, kKMixedCol = 1, kKRowPool = 2, kKColPipeHide = 3, kKMixedColHide = 4, kKNum = 5 };

// Resident grid for `fn` on the stream's device (never more than n_units, at
// least 1); 0 on a runtime error.
uint64_t persistent_grid(hipStream_t st, PersistentKernel k, const void* fn, uint64_t n_units, int* cus_out,
                         int block_threads = kTPB);

}  // namespace pbl
