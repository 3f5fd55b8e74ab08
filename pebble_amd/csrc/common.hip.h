// common.hip.h — shared device helpers for the gfx950 block decoders:
// wave/block scans and the decoupled look-back that places every block's
// outputs in ONE pass (no separate size pass).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/pebble_amd.h"

namespace pbl {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));  // native 16-B vector

constexpr int kTPB = 256;   // threads per workgroup (4 waves); one workgroup per block
constexpr int kWave = 64;
constexpr int kNumComp = 4; // look-back components: n_kv, key bytes, value bytes, restarts
constexpr int kLbWin = 4;   // look-back windows (of 64 predecessors) loaded per round trip

// ---- workspace layout ------------------------------------------------------
// [0,256): ticket counter (+ pad).  Then kNumComp arrays of n_blocks u64
// granules {state:2 | value:62} written and read with agent-scope relaxed
// atomics (8-byte sc1 accesses: the data IS the flag, no fences needed —
// MI355X_MICROARCH.md "Valid forms", R2 granules).
constexpr uint64_t kWsHeader = 256;
constexpr uint64_t kStateAgg = 1ull << 62;
constexpr uint64_t kStatePfx = 2ull << 62;
constexpr uint64_t kValMask = (1ull << 62) - 1;

__host__ __device__ inline uint64_t ws_bytes(uint32_t n_blocks) {
  return kWsHeader + uint64_t(kNumComp) * n_blocks * 8ull;
}
#ifdef PBL_STAMPS
constexpr uint64_t kStampWords = 16;  // diagnostic build: per-block phase stamps
#else
constexpr uint64_t kStampWords = 0;
#endif
__host__ __device__ inline uint64_t ws_alloc_bytes(uint32_t n_blocks) {
  return ws_bytes(n_blocks) + kStampWords * 8ull * n_blocks;
}

__device__ inline uint64_t ld_agent(const uint64_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ inline void st_agent(uint64_t* p, uint64_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
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

// Decoupled look-back (single-pass scan across blocks), in two halves so a
// workgroup can publish its aggregate as soon as it is known and resolve its
// exclusive prefix later (after overlapping independent work).  Tickets are
// handed out in launch order, so every predecessor is already resident and
// publishes its aggregate before it waits: no deadlock for any residency.
// Both halves are executed by wave 0 of the workgroup that owns virtual block `v`.
__device__ inline void lb_publish(uint64_t* st, uint32_t n_blocks, uint32_t v, const uint64_t agg[kNumComp]) {
  const int l = lane_id();
  if (l < kNumComp) {
    uint64_t a = l == 0 ? agg[0] : l == 1 ? agg[1] : l == 2 ? agg[2] : agg[3];
    st_agent(st + uint64_t(l) * n_blocks + v, (v == 0 ? kStatePfx : kStateAgg) | (a & kValMask));
  }
}

// All components are walked back together, kLbWin windows of 64 predecessors
// per round trip.  Returns exclusive prefixes and publishes the inclusive ones.
__device__ inline void lb_resolve(uint64_t* st, uint32_t n_blocks, uint32_t v, const uint64_t agg[kNumComp],
                                  uint64_t excl[kNumComp], uint32_t* timeout_flag) {
  const int l = lane_id();
  uint64_t acc[kNumComp];
  int64_t top[kNumComp];
  bool done[kNumComp];
#pragma unroll
  for (int c = 0; c < kNumComp; c++) { acc[c] = 0; top[c] = int64_t(v) - 1; done[c] = v == 0; }
  uint32_t spins = 0;
  while (!(done[0] && done[1] && done[2] && done[3])) {
    uint64_t g[kNumComp][kLbWin];
#pragma unroll
    for (int c = 0; c < kNumComp; c++)
#pragma unroll
      for (int k = 0; k < kLbWin; k++) {
        int64_t idx = top[c] - kWave * k - l;
        g[c][k] = (!done[c] && idx >= 0) ? ld_agent(st + uint64_t(c) * n_blocks + idx) : kStatePfx;
      }
    int64_t wait_word = -1;  // a word that was not ready yet
#pragma unroll
    for (int c = 0; c < kNumComp; c++) {
      bool stop = done[c];
#pragma unroll
      for (int k = 0; k < kLbWin; k++) {
        if (stop) continue;
        uint64_t state = g[c][k] >> 62;
        uint64_t pfx = __ballot(state == 2);
        uint64_t notready = __ballot(state == 0);
        int first = pfx ? __builtin_ctzll(pfx) : 64;
        uint64_t need = first >= 63 ? ~0ull : ((2ull << first) - 1);
        if (notready & need) {
          if (wait_word < 0)
            wait_word = int64_t(c) * n_blocks + (top[c] - kWave * k - __builtin_ctzll(notready & need));
          stop = true;
          continue;
        }
        acc[c] += wave_sum((l <= first) ? (g[c][k] & kValMask) : 0ull);
        if (first < 64) { done[c] = true; stop = true; }
        else top[c] -= kWave;
      }
    }
    if (wait_word >= 0) {
      // Poll the missing predecessor from ONE lane (a whole-window re-read per
      // poll would flood this CU's memory queue), then re-read the window.
      bool timed_out = false;
      if (l == 0) {
        while ((ld_agent(st + wait_word) >> 62) == 0) {
          if (++spins > (1u << 22)) { timed_out = true; break; }
          __builtin_amdgcn_s_sleep(2);
        }
      }
      if (__shfl(timed_out ? 1 : 0, 0, kWave)) {
        if (l == 0) atomicOr(timeout_flag, 1u << PBL_TIMEOUT);
        break;
      }
    }
  }
#pragma unroll
  for (int c = 0; c < kNumComp; c++) excl[c] = acc[c];
  if (l < kNumComp && v > 0) {
    uint64_t e = l == 0 ? excl[0] : l == 1 ? excl[1] : l == 2 ? excl[2] : excl[3];
    uint64_t a = l == 0 ? agg[0] : l == 1 ? agg[1] : l == 2 ? agg[2] : agg[3];
    st_agent(st + uint64_t(l) * n_blocks + v, kStatePfx | ((e + a) & kValMask));
  }
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
__device__ inline void store16(uint8_t* base, uint64_t ga, uint64_t lo, uint64_t hi, uint4 w) {
  if (ga >= lo && ga + 16 <= hi) {
    *reinterpret_cast<uint4*>(base + ga) = w;
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
  O.blk_kv_base[b] = excl[0];
  O.blk_key_base[b] = excl[1];
  O.blk_val_base[b] = excl[2];
  if (O.blk_rst_base) O.blk_rst_base[b] = excl[3];
  O.blk_status[b] = status;
  if (slow) atomicAdd(&O.totals->n_slow_blocks, 1u);
  if (status != PBL_OK) {
    atomicOr(&O.totals->status_mask, 1u << status);
    atomicAdd(&O.totals->n_bad_blocks, 1u);
  }
  if (b == nb - 1) {
    O.blk_kv_base[nb] = excl[0] + agg[0];
    O.blk_key_base[nb] = excl[1] + agg[1];
    O.blk_val_base[nb] = excl[2] + agg[2];
    if (O.blk_rst_base) O.blk_rst_base[nb] = excl[3] + agg[3];
    O.totals->n_kv = excl[0] + agg[0];
    O.totals->key_bytes = excl[1] + agg[1];
    O.totals->val_bytes = excl[2] + agg[2];
    O.totals->n_restarts = excl[3] + agg[3];
  }
}

__device__ inline bool overflows(const pbl_decode_out& O, const uint64_t excl[kNumComp],
                                 const uint64_t agg[kNumComp]) {
  return excl[0] + agg[0] > O.kv_cap || excl[1] + agg[1] > O.key_cap || excl[2] + agg[2] > O.val_cap ||
         (O.restarts && excl[3] + agg[3] > O.rst_cap);
}

}  // namespace pbl
