// snappy_dec.hip.h — the snappy block decoder of snappy2_kernel (physical.hip),
// written against a small set of wave primitives (lptr / gptr, lane_id,
// wave_sync, __shfl, __ballot, readfirstlane, alignbyte) so that
// scripts/snappy_emu.cpp can run the same code on the host with 64 threads in
// lockstep.  Included by physical.hip inside namespace pbl::phys, after
// kSnIn / kSnQ and the SN_T / SN_ACC stamp macros.
#pragma once

constexpr uint32_t kSnBkShift = 7, kSnBk = 65536u >> kSnBkShift;  // output buckets (sn_buckets)
struct Snap2Lds {
  alignas(16) uint32_t in[(kSnIn + 64) / 4];  // compressed bytes at their 16-B phase (+ slack)
  uint64_t q[kSnQ];               // dst | len << 16 | (src or offset) << 32 | copy << 63
  uint32_t r[kSnQ];               // copies: where their bytes are (see sn_resolve)
  uint16_t bk[kSnBk];             // output buckets -> element (sn_buckets)
};

// bytes [a, a + 16) of the staged LDS words, any alignment
__device__ __forceinline__ uint4 sn_lds16(lptr<const uint32_t> W, uint32_t a) {
  const uint32_t q = a >> 2, r = a & 3;
  const uint32_t x0 = W[q], x1 = W[q + 1], x2 = W[q + 2], x3 = W[q + 3], x4 = W[q + 4];
  return make_uint4(__builtin_amdgcn_alignbyte(x1, x0, r), __builtin_amdgcn_alignbyte(x2, x1, r),
                    __builtin_amdgcn_alignbyte(x3, x2, r), __builtin_amdgcn_alignbyte(x4, x3, r));
}
__device__ __forceinline__ uint64_t sn_lds8(lptr<const uint32_t> W, uint32_t a) {
  const uint32_t q = a >> 2, r = a & 3;
  const uint32_t x0 = W[q], x1 = W[q + 1], x2 = W[q + 2];
  return uint64_t(__builtin_amdgcn_alignbyte(x2, x1, r)) << 32 | __builtin_amdgcn_alignbyte(x1, x0, r);
}

typedef u32x4 sn_u32x4_u __attribute__((aligned(1)));
typedef uint64_t sn_u64_u __attribute__((aligned(1)));
typedef uint32_t sn_u32_u __attribute__((aligned(1)));
typedef uint16_t sn_u16_u __attribute__((aligned(1)));
// bytes [0, n) of w (n <= 16) to p, nothing past n
__device__ __forceinline__ void sn_store_n(gptr<uint8_t> p, const uint4& w, uint32_t n) {
  if (n == 16) {
    *(gptr<sn_u32x4_u>)p = u32x4{w.x, w.y, w.z, w.w};
    return;
  }
  uint64_t lo = uint64_t(w.x) | uint64_t(w.y) << 32, hi = uint64_t(w.z) | uint64_t(w.w) << 32;
  uint32_t o = 0;
  if (n & 8) { *(gptr<sn_u64_u>)p = lo; lo = hi; o = 8; }
  if (n & 4) { *(gptr<sn_u32_u>)(p + o) = uint32_t(lo); lo >>= 32; o += 4; }
  if (n & 2) { *(gptr<sn_u16_u>)(p + o) = uint16_t(lo); lo >>= 16; o += 2; }
  if (n & 1) *(p + o) = uint8_t(lo);
}

__device__ __forceinline__ void sn_fence() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}

// One element at the start of w (the 8 input bytes from its tag on, zero past
// the input): header bytes h, output length len, copy offset off (copies).
// Unvalidated; the callers check it against the input and output left.
struct SnElem {
  uint32_t h, len, off;
  bool lit;
};
__device__ __forceinline__ SnElem sn_elem(uint64_t w) {
  const uint32_t t = uint32_t(w) & 0xff, kind = t & 3, ext = uint32_t(w >> 8);
  SnElem e;
  e.lit = kind == 0;
  if (kind == 0) {
    uint32_t x = t >> 2;
    e.h = 1;
    if (x >= 60) {
      const uint32_t nb = x - 59;
      e.h = 1 + nb;
      x = ext & (nb == 4 ? 0xffffffffu : (1u << (8 * nb)) - 1u);
    }
    e.len = x + 1;  // (x = 2^32 - 1 wraps to 0: rejected)
    e.off = 0;
  } else if (kind == 1) {
    e.h = 2;
    e.len = 4 + ((t >> 2) & 7);
    e.off = ((t & 0xe0) << 3) | (ext & 0xff);
  } else {
    e.h = kind == 2 ? 3 : 5;
    e.len = 1 + (t >> 2);
    e.off = kind == 2 ? (ext & 0xffff) : ext;
  }
  return e;
}
// snappy.Decode's ErrCorrupt cases for the element at input offset s (n input
// bytes) and output offset d (D output bytes)
__device__ __forceinline__ bool sn_elem_ok(const SnElem& e, uint32_t s, uint32_t n, uint32_t d, uint32_t D) {
  if (e.h > n - s || e.len > D - d) return false;
  return e.lit ? (e.len != 0 && e.len <= n - s - e.h) : (e.off != 0 && e.off <= d);
}
__device__ __forceinline__ uint64_t sn_qent(const SnElem& e, uint32_t s, uint32_t d) {
  return e.lit ? uint64_t(d) | uint64_t(e.len) << 16 | uint64_t(s + e.h) << 32
               : uint64_t(d) | uint64_t(e.len) << 16 | uint64_t(e.off) << 32 | (1ull << 63);
}

// The whole wave: queue the elements starting at input offset *s (output
// offset *d) until the queue or the input is full.  Returns the count; *ok
// clears on a corrupt element.  The LDS words are read by every lane at one
// address and made uniform with readfirstlane, so the walk's arithmetic and
// branches are scalar; lane 0 writes the queue.
__device__ __forceinline__ uint32_t sn_parse(lptr<const uint32_t> W, uint32_t ib, lptr<uint64_t> Q, uint32_t n,
                                             uint32_t D, uint32_t* s_io, uint32_t* d_io, bool* ok) {
  uint32_t s = *s_io, d = *d_io, c = 0;
  const bool l0 = lane_id() == 0;
  while (s < n && c < kSnQ) {
    const uint32_t a = ib + s, q = a >> 2, r = 8 * (a & 3);
    // (readfirstlane returns int: through uint32_t, no sign extension)
    const uint64_t x01 = uint64_t(uint32_t(__builtin_amdgcn_readfirstlane(W[q]))) |
                         uint64_t(uint32_t(__builtin_amdgcn_readfirstlane(W[q + 1]))) << 32;
    const uint32_t x2 = uint32_t(__builtin_amdgcn_readfirstlane(W[q + 2]));
    const uint64_t w = (x01 >> r) | (r ? uint64_t(x2) << (64 - r) : 0ull);  // bytes [a, a + 8)
    const SnElem e = sn_elem(w);
    if (!sn_elem_ok(e, s, n, d, D)) { *ok = false; break; }
    if (l0) Q[c] = sn_qent(e, s, d);
    c++;
    s += e.h + (e.lit ? e.len : 0u);
    d += e.len;
  }
  *s_io = s;
  *d_io = d;
  return c;
}

constexpr uint32_t kSnWalkMin = 64;  // smaller blocks: sn_decode walks them itself

// Copy sources by pointer jumping.  R[j] of copy j holds a position whose
// final bytes equal the copy's: first its output position o - off; each round
// finds the element whose output holds that range and replaces it by the same
// range of that element's source -- a literal's input bytes (kSnRes | input
// offset: resolved, copied with the literals), or a copy's own R (an output
// position, strictly lower) -- so a chain of copies of copies collapses in log
// rounds.  A range that straddles elements or lies before this round's queue
// stops (kSnStop | output position).  Unresolved copies then run in output
// order, a group at a time, each reading the final output at its position;
// since chains collapse towards their roots, a group can take every copy whose
// position range ends below the group's first output.  Races between lanes are
// benign: every value R[k] takes is a valid source of copy k's bytes.
// Overlapping copies (off < len) keep o - off and repeat their period.
constexpr uint32_t kSnRes = 1u << 31, kSnStop = 1u << 30, kSnPos = 0xffffu;
__device__ __forceinline__ uint32_t sn_dst(uint64_t e) { return uint32_t(e) & 0xffffu; }
__device__ __forceinline__ uint32_t sn_len(uint64_t e) { return uint32_t(e >> 16) & 0xffffu; }
__device__ __forceinline__ uint32_t sn_src(uint64_t e) { return uint32_t(e >> 32) & 0x7fffffffu; }
// Buckets of the round's output: BK[c] = the element holding output offset
// d0 + c * 2^kSnBkShift.
__device__ __forceinline__ void sn_buckets(lptr<const uint64_t> QR, lptr<uint16_t> BK, uint32_t qc, uint32_t d0) {
  const uint32_t lane = lane_id();
  for (uint32_t i0 = 0; i0 < qc; i0 += kWave) {
    const uint32_t j = i0 + lane;
    uint32_t c0 = 0, c1 = 0;
    if (j < qc) {
      const uint64_t e = QR[j];
      const uint32_t r = sn_dst(e) - d0, m = (1u << kSnBkShift) - 1;
      c0 = (r + m) >> kSnBkShift;
      c1 = (r + sn_len(e) + m) >> kSnBkShift;
      if (c1 - c0 <= 4)
        for (uint32_t c = c0; c < c1; c++) BK[c] = uint16_t(j);
    }
    for (uint64_t wm = __ballot(c1 - c0 > 4); wm; wm &= wm - 1) {
      const int sl = __builtin_ctzll(wm);
      const uint32_t a = __shfl(c0, sl, kWave), z = __shfl(c1, sl, kWave);
      for (uint32_t c = a + lane; c < z; c += kWave) BK[c] = uint16_t(i0 + uint32_t(sl));
    }
  }
  wave_sync();
}
__device__ __forceinline__ void sn_resolve(lptr<const uint64_t> QR, lptr<uint32_t> R, lptr<const uint16_t> BK,
                                           uint32_t qc, uint32_t d0) {
  const uint32_t lane = lane_id();
  for (uint32_t j = lane; j < qc; j += kWave) {
    const uint64_t e = QR[j];
    if (e >> 63) {
      const uint32_t o = sn_dst(e), len = sn_len(e), off = sn_src(e);
      R[j] = (off < len ? kSnStop : 0u) | (o - off);
    }
  }
  wave_sync();
  for (int round = 0; round < 12; round++) {
    bool open = false;
    for (uint32_t j = lane; j < qc; j += kWave) {
      const uint64_t e = QR[j];
      if (!(e >> 63)) continue;
      const uint32_t rj = R[j];
      if (rj & (kSnRes | kSnStop)) continue;
      const uint32_t len = sn_len(e);
      uint32_t nr = kSnStop | rj;
      if (rj >= d0) {
        uint32_t k = BK[(rj - d0) >> kSnBkShift];
        while (k + 1 < qc && sn_dst(QR[k + 1]) <= rj) k++;
        const uint64_t ek = QR[k];
        const uint32_t dk = sn_dst(ek);
        if (rj + len <= dk + sn_len(ek)) {
          if (!(ek >> 63)) {
            nr = kSnRes | (sn_src(ek) + (rj - dk));
          } else {
            const uint32_t rk = R[k];
            if (rk & kSnRes) {
              nr = rk + (rj - dk);
            } else {
              nr = (rk & kSnPos) + (rj - dk);  // (< rj: another round)
              open = true;
            }
          }
        }
      }
      R[j] = nr;
    }
    if (!__ballot(open)) break;
    wave_sync();
  }
  wave_sync();
}

// One snappy block (those the walk does not cover): compressed bytes staged at byte ib of W (n bytes, the
// uvarint header included), D decoded bytes to dst.  Uniform result: false = corrupt.
__device__ bool sn_decode(Snap2Lds& S, uint32_t ib, uint32_t n, uint32_t used, uint32_t D, gptr<uint8_t> dst,
                          uint32_t g_sn_b = 0) {
  const uint32_t lane = lane_id();
  (void)g_sn_b;
  lptr<const uint32_t> W = to_lds_ptr(static_cast<const uint32_t*>(S.in));
  lptr<uint64_t> Q = to_lds_ptr(S.q);
  const lptr<const uint64_t> QR = to_lds_ptr(static_cast<const uint64_t*>(S.q));
  lptr<uint32_t> R = to_lds_ptr(S.r);
  lptr<uint16_t> BK = to_lds_ptr(S.bk);
  uint32_t s = used, d = 0;
  bool ok = true;
  while (s < n) {
    const uint32_t dr = d;  // the round's first output offset
    SN_T(t0);
    const uint32_t qc = sn_parse(W, ib, Q, n, D, &s, &d, &ok);
    if (!ok) return false;
    wave_sync();
    SN_ACC(1, t0);
    SN_T(t1);
    sn_buckets(QR, BK, qc, dr);
    sn_resolve(QR, R, to_lds_ptr(static_cast<const uint16_t*>(S.bk)), qc, dr);
    SN_ACC(6, t1);
    SN_T(t1b);
    // literals and resolved copies: lane per element, from the staged input
    for (uint32_t i0 = 0; i0 < qc; i0 += kWave) {
      const uint32_t i = i0 + lane;
      uint64_t e = 0;
      uint32_t len = 0, src = 0;
      if (i < qc) {
        e = QR[i];
        len = uint32_t(e >> 16) & 0xffffu;
        src = uint32_t(e >> 32) & 0x7fffffffu;
        if (e >> 63) {
          const uint32_t ri = R[i];
          if (ri & kSnRes) src = ri & ~kSnRes;
          else len = 0;
        }
      }
      const uint32_t o = uint32_t(e) & 0xffffu;
      if (len && len <= 256)
        for (uint32_t c = 0; c < len; c += 16) {
          const uint32_t k = len - c < 16 ? len - c : 16u;
          sn_store_n(dst + o + c, sn_lds16(W, ib + src + c), k);
        }
      for (uint64_t m = __ballot(len > 256); m; m &= m - 1) {
        const int sl = __builtin_ctzll(m);
        const uint32_t lo = __shfl(o, sl, kWave), ls = __shfl(src, sl, kWave), ll = __shfl(len, sl, kWave);
        for (uint32_t c = 16 * lane; c < ll; c += 16 * kWave) {
          const uint32_t k = ll - c < 16 ? ll - c : 16u;
          sn_store_n(dst + lo + c, sn_lds16(W, ib + ls + c), k);
        }
      }
    }
    sn_fence();
    SN_ACC(2, t1b);
    SN_T(t2);
    // copies: groups of independent ones, lane per copy
    uint32_t i = 0;
    while (i < qc) {
      const uint32_t j = i + lane;
      uint64_t e = 0;
      if (j < qc) e = QR[j];
      const bool isc = j < qc && (e >> 63) && !(R[j] & kSnRes);  // (resolved copies are done)
      const uint64_t cm = __ballot(isc);
      if (!cm) {  // (no pending copy among the next 64)
        i += kWave;
        continue;
      }
      const int first = __builtin_ctzll(cm);
      const uint32_t o = uint32_t(e) & 0xffffu, len = uint32_t(e >> 16) & 0xffffu,
                     off = uint32_t(e >> 32) & 0x7fffffffu;
      const uint32_t d0 = __builtin_amdgcn_readlane(o, first);
      // final bytes at [P, P + len) (an overlapping copy: its period [o - off, o))
      const bool ovl = off < len;
      const uint32_t P = ovl ? o - off : (isc ? R[j] & kSnPos : 0u);
      const bool indep = isc && (ovl ? o <= d0 : P + len <= d0);
      const uint64_t stop = first == 63 ? 0ull : (__ballot(isc && !indep) & ~((2ull << first) - 1));
      const uint32_t end = stop ? uint32_t(__builtin_ctzll(stop)) : uint32_t(kWave);  // lanes [first, end) run
      if (isc && uint32_t(lane) >= uint32_t(first) && uint32_t(lane) < end) {
        const gptr<const uint8_t> sp = dst + P;
        if (!ovl || off >= 16) {  // (an overlapping copy: each chunk's source is written before it)
          for (uint32_t c = 0; c < len; c += 16) {
            const u32x4 v = *(gptr<const sn_u32x4_u>)(sp + c);
            sn_store_n(dst + o + c, make_uint4(v.x, v.y, v.z, v.w), len - c < 16 ? len - c : 16u);
          }
        } else {
          // the period: bytes [o - off, o), final
          uint8_t per[16];
          for (uint32_t k = 0; k < off; k++) per[k] = sp[k];
          for (uint32_t k = 0; k < len; k++) dst[o + k] = per[k % off];
        }
      }
      sn_fence();
      i += end;
#ifdef PBL_SNAP_STAMPS
      if (lane == 0 && g_sn_b < 65536) g_snap_stamps[8 * g_sn_b + 5] += 1;  // groups
#endif
    }
    SN_ACC(3, t2);
  }
#ifdef PBL_SNAP_STAMPS
  if (lane == 0 && g_sn_b < 65536) g_snap_stamps[8 * g_sn_b + 4] += 1;  // rounds
#endif
  return d == D;
}


// ==== snappy4: the blocks the walk covers (sn4_walkable) ======================
// snappy_walk_kernel walks each block's element chain on one lane (64 blocks
// per wave: the chain's latency becomes throughput), validates every element
// and leaves, in the block's own output region, which the decode overwrites
// afterwards:
//   out[0, 16)             {ok, elements, D, n}
//   out[16, 16 + 4 nw)     the tag bitmap: bit i of word w = an element's tag
//                          at input offset 32 w + i (nw = ceil(n / 32))
// snappy4_kernel then decodes a block per wave with nothing staged: the tag
// offsets come from the bitmap (a popcount scan), every element decodes on its
// own lane from the input in HBM, output offsets by a scan of the lengths; an
// output-start bitmap with per-word counts finds the element holding any
// output offset with one LDS round trip, so the copy-chain pointer jumping
// (sn_resolve's scheme) runs with each lane's copies in registers.  20 KB of
// LDS: 8 blocks per CU.
constexpr uint32_t kS4In = 36864, kS4Span = 32768, kS4Q = 768, kS4Slots = kS4Q / kWave;
struct Snap4Lds {
  uint64_t q[kS4Q];           // dst | len << 16 | (src or offset) << 32 | copy << 63
  uint32_t r[kS4Q];           // copies: where their bytes are (kSnRes / kSnStop / output offset)
  uint32_t tb[kS4In / 32];    // the walk's tag bitmap
  uint32_t ob[kS4Span / 32];  // the round's element starts, by output offset - the round's first
  uint16_t pf[kS4Span / 64];  // element starts before each 64-bit word of ob
  uint16_t cl[kS4Q];          // the round's copies, in order
};
// (kS4In past 32 KiB: an incompressible 32 KiB block's snappy form is a few
// bytes longer than the block; at 32 KiB such blocks fell to the one-lane
// global-memory decoder, 1/256 of a text batch's blocks taking 80 % of its time)
static_assert(8 * sizeof(Snap4Lds) <= 163840, "8 blocks per CU");
__device__ __forceinline__ bool sn4_walkable(uint32_t n, uint32_t D) {
  return n >= 8 && n <= kS4In && D >= kSnWalkMin && D <= kS4Span && D >= 16 + 4 * ((n + 31) / 32);
}
// bytes [s, s + 8) (s < n) reading nothing past p[n] (the block's indicator)
__device__ __forceinline__ uint64_t sn_load8c(gptr<const uint8_t> p, uint32_t s, uint32_t n) {
  const uint32_t a = s < n - 7 ? s : n - 7;
  return *(gptr<const sn_u64_u>)(p + a) >> (8 * (s - a));
}
// bytes [s, s + 16) (s < n; past p[n]: unspecified)
__device__ __forceinline__ uint4 sn_load16c(gptr<const uint8_t> p, uint32_t s, uint32_t n) {
  if (s + 16 <= n + 1) {
    const u32x4 v = *(gptr<const sn_u32x4_u>)(p + s);
    return make_uint4(v[0], v[1], v[2], v[3]);
  }
  const uint64_t lo = sn_load8c(p, s, n), hi = s + 8 < n ? sn_load8c(p, s + 8, n) : 0ull;
  return make_uint4(uint32_t(lo), uint32_t(lo >> 32), uint32_t(hi), uint32_t(hi >> 32));
}
#ifndef SN_EMU_SCAN
// inclusive, over the wave: DPP row shifts and row broadcasts (no LDS round trip)
__device__ __forceinline__ uint32_t sn_scan(uint32_t v) {
  v += __builtin_amdgcn_update_dpp(0u, v, 0x111, 0xf, 0xf, false);  // row_shr:1
  v += __builtin_amdgcn_update_dpp(0u, v, 0x112, 0xf, 0xf, false);  // row_shr:2
  v += __builtin_amdgcn_update_dpp(0u, v, 0x114, 0xf, 0xf, false);  // row_shr:4
  v += __builtin_amdgcn_update_dpp(0u, v, 0x118, 0xf, 0xf, false);  // row_shr:8
  v += __builtin_amdgcn_update_dpp(0u, v, 0x142, 0xa, 0xf, false);  // row_bcast:15
  v += __builtin_amdgcn_update_dpp(0u, v, 0x143, 0xc, 0xf, false);  // row_bcast:31
  return v;
}
#else  // (the host emulator: the same scan by exchanges)
__device__ __forceinline__ uint32_t sn_scan(uint32_t v) {
  const uint32_t lane = lane_id();
  for (uint32_t o = 1; o < uint32_t(kWave); o <<= 1) {
    const uint32_t t = __shfl(v, lane >= o ? int(lane - o) : int(lane), kWave);
    if (lane >= o) v += t;
  }
  return v;
}
#endif
#ifndef SN_LDS_OR
#define SN_LDS_OR(p, v) __hip_atomic_fetch_or((p), (v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)
#endif

// One lane's read window over a block's input: the 64 bytes at [wb, wb + 64)
// (wb a 16-B aligned address) in eight u64 registers, slid 16 bytes at a time;
// the granule a slide loads is first read two slides later, so the walk reads
// from registers while its loads run ~32 bytes (~10 text elements) ahead,
// instead of one dependent global load per element.  Granules past the last
// readable byte (the indicator at p[n]) read as zeros; the first may start up
// to 15 bytes before p, inside p's own 16-B granule.
struct SnWin {
  uint64_t lim;  // address of p[n]
  uint64_t wb;
  uint64_t w0, w1, w2, w3, w4, w5, w6, w7;
  __device__ __forceinline__ void ld(uint64_t a, uint64_t& x, uint64_t& y) const {
    if (a <= lim) {
      const u32x4 v = *(gptr<const u32x4>)(reinterpret_cast<const u32x4*>(a));
      x = uint64_t(v[0]) | uint64_t(v[1]) << 32;
      y = uint64_t(v[2]) | uint64_t(v[3]) << 32;
    } else {
      x = y = 0;
    }
  }
  __device__ __forceinline__ void reset(uint64_t a) {
    wb = a & ~uint64_t(15);
    ld(wb, w0, w1);
    ld(wb + 16, w2, w3);
    ld(wb + 32, w4, w5);
    ld(wb + 48, w6, w7);
  }
  __device__ __forceinline__ uint64_t sel(uint32_t k) const {  // word k of 8, selects only
    const uint64_t a = (k & 1) ? w1 : w0, b = (k & 1) ? w3 : w2, c = (k & 1) ? w5 : w4, d = (k & 1) ? w7 : w6;
    const uint64_t e = (k & 2) ? b : a, f = (k & 2) ? d : c;
    return (k & 4) ? f : e;
  }
  // bytes [a, a + 8) (a - wb <= 56)
  __device__ __forceinline__ uint64_t get8(uint64_t a) const {
    const uint32_t o = uint32_t(a - wb), k = o >> 3, sh = 8 * (o & 7);
    const uint64_t lo = sel(k);
    if (!sh) return lo;
    return (lo >> sh) | (sel(k + 1) << (64 - sh));
  }
  // make [a, a + 8) readable: slide while a is 16 or more bytes in (a load per
  // slide), jump when it is past the window
  __device__ __forceinline__ void seek(uint64_t a) {
    if (a - wb >= 64) {
      reset(a);
      return;
    }
    while (a - wb >= 16) {
      w0 = w2; w1 = w3; w2 = w4; w3 = w5; w4 = w6; w5 = w7;
      wb += 16;
      ld(wb + 48, w6, w7);
    }
  }
};

// One lane: the walk of a block (n input bytes from `used` on, D output bytes).
__device__ __forceinline__ void sn4_walk(gptr<const uint8_t> p, uint32_t n, uint32_t used, uint32_t D,
                                         gptr<uint8_t> out) {
  const gptr<uint8_t> bm = out + 16;
  const uint32_t nw = (n + 31) / 32;
  uint32_t s = used, d = 0, cnt = 0, ok = 1, cw = 0, acc = 0;
  const uint64_t pa = reinterpret_cast<uint64_t>(p);
  SnWin W;
  W.lim = pa + n;
  W.reset(pa + s);
  while (s < n) {
    const SnElem e = sn_elem(W.get8(pa + s));
    if (!sn_elem_ok(e, s, n, d, D)) { ok = 0; break; }
    const uint32_t s0 = s;
    s += e.h + (e.lit ? e.len : 0u);
    d += e.len;
    if (s < n) W.seek(pa + s);
    for (; cw < (s0 >> 5); cw++, acc = 0) *(gptr<sn_u32_u>)(bm + 4 * cw) = acc;
    acc |= 1u << (s0 & 31);
    cnt++;
  }
  if (ok)
    for (; cw < nw; cw++, acc = 0) *(gptr<sn_u32_u>)(bm + 4 * cw) = acc;
  *(gptr<sn_u32x4_u>)out = u32x4{ok && d == D ? 1u : 0u, cnt, d, s};
}

// The element holding output offset a (d0 <= a < the round's end).
__device__ __forceinline__ uint32_t sn4_find(lptr<const uint32_t> OB, lptr<const uint16_t> PF, uint32_t x) {
  const uint32_t w = x >> 6;
  const uint64_t b = uint64_t(OB[2 * w]) | uint64_t(OB[2 * w + 1]) << 32;
  return uint32_t(PF[w]) + uint32_t(__builtin_popcountll(b & (~0ull >> (63 - (x & 63))))) - 1u;
}

// Pointer jumping (as sn_resolve) with each lane's copies in registers: copy
// g of the round's list on lane g % 64, slot g / 64; every round reads the
// state it needs first and writes all new states after (the wave in lockstep).
__device__ __forceinline__ void sn4_resolve(lptr<const uint64_t> QR, lptr<uint32_t> R, lptr<const uint16_t> CL,
                                            lptr<const uint32_t> OB, lptr<const uint16_t> PF, uint32_t cc,
                                            uint32_t dr) {
  const uint32_t lane = lane_id();
  uint32_t sj[kS4Slots], sl[kS4Slots], sr[kS4Slots];
#pragma unroll
  for (uint32_t t = 0; t < kS4Slots; t++) {
    const uint32_t g = lane + kWave * t;
    sj[t] = 0;
    sl[t] = 0;
    sr[t] = kSnStop;
    if (g < cc) {
      sj[t] = CL[g];
      const uint64_t e = QR[sj[t]];
      const uint32_t o = sn_dst(e), len = sn_len(e), off = sn_src(e);
      sl[t] = len;
      sr[t] = (off < len ? kSnStop : 0u) | (o - off);
      R[sj[t]] = sr[t];
    }
  }
  wave_sync();
  for (int round = 0; round < 16; round++) {
    bool open = false;
    uint32_t nr[kS4Slots];
#pragma unroll
    for (uint32_t t = 0; t < kS4Slots; t++) {
      const uint32_t x = sr[t];
      nr[t] = x;
      if (!(x & (kSnRes | kSnStop))) {
        nr[t] = kSnStop | x;
        if (x >= dr) {
          const uint32_t k = sn4_find(OB, PF, x - dr);
          const uint64_t ek = QR[k];
          const uint32_t dk = sn_dst(ek);
          if (x + sl[t] <= dk + sn_len(ek)) {
            if (!(ek >> 63)) {
              nr[t] = kSnRes | (sn_src(ek) + (x - dk));
            } else {
              const uint32_t rk = R[k];
              if (rk & kSnRes) {
                nr[t] = rk + (x - dk);
              } else {
                nr[t] = (rk & kSnPos) + (x - dk);  // (< x: another round)
                open = true;
              }
            }
          }
        }
      }
    }
#pragma unroll
    for (uint32_t t = 0; t < kS4Slots; t++) {
      if (lane + kWave * t < cc && nr[t] != sr[t]) R[sj[t]] = nr[t];
      sr[t] = nr[t];
    }
    wave_sync();
    if (!__ballot(open)) break;
  }
}

// One block the walk covers: n input bytes at src (HBM), D output bytes to dst
// (holding the walk's header and bitmap).  Uniform result: false = corrupt.
__device__ bool sn4_decode(Snap4Lds& S, gptr<const uint8_t> src, uint32_t n, uint32_t D, gptr<uint8_t> dst,
                           uint32_t g_sn_b = 0) {
  const uint32_t lane = lane_id();
  (void)g_sn_b;
  lptr<uint64_t> Q = to_lds_ptr(S.q);
  const lptr<const uint64_t> QR = to_lds_ptr(static_cast<const uint64_t*>(S.q));
  lptr<uint32_t> R = to_lds_ptr(S.r);
  lptr<uint32_t> TB = to_lds_ptr(S.tb);
  lptr<uint32_t> OB = to_lds_ptr(S.ob);
  lptr<uint16_t> PF = to_lds_ptr(S.pf);
  lptr<uint16_t> CL = to_lds_ptr(S.cl);
  SN_T(ts);
  const u32x4 hd = *(gptr<const sn_u32x4_u>)dst;  // (read before any output is written)
  if (!hd[0]) return false;
  const uint32_t nw = (n + 31) / 32;
  for (uint32_t w = lane; w < nw; w += kWave) TB[w] = *(gptr<const sn_u32_u>)(dst + 16 + 4 * w);
  wave_sync();
  SN_ACC(0, ts);
  uint32_t wc = 0, d = 0;
  while (wc < nw) {
    const uint32_t dr = d;
    SN_T(t0);
    // 1. the round's tag offsets from the bitmap (whole words, <= kS4Q)
    uint32_t qc = 0;
    for (;;) {
      const uint32_t w = wc + lane;
      const uint32_t bits = w < nw ? TB[w] : 0u;
      const uint32_t c = uint32_t(__builtin_popcount(bits));
      const uint32_t incl = sn_scan(c);
      const bool take = w < nw && qc + incl <= kS4Q;
      const uint64_t tm = __ballot(take);
      if (take) {
        uint32_t k = qc + incl - c;
        for (uint32_t b = bits; b; b &= b - 1) Q[k++] = 32 * w + uint32_t(__builtin_ctz(b));
      }
      const uint32_t na = uint32_t(__builtin_popcountll(tm));
      if (na) qc += __builtin_amdgcn_readlane(incl, int(na - 1));
      wc += na;
      if (na < uint32_t(kWave)) break;
    }
    for (uint32_t i = lane; i < kS4Span / 32; i += kWave) OB[i] = 0;
    wave_sync();
    // 2. the elements, a lane each: decode, output offsets, output starts
    uint64_t wv[kS4Slots];
#pragma unroll
    for (uint32_t t = 0; t < kS4Slots; t++) {
      const uint32_t i = lane + kWave * t;
      wv[t] = i < qc ? sn_load8c(src, uint32_t(QR[i]), n) : 0ull;
    }
#pragma unroll
    for (uint32_t t = 0; t < kS4Slots; t++) {
      if (kWave * t >= qc) break;
      const uint32_t i = lane + kWave * t;
      SnElem e{0, 0, 0, true};
      uint32_t pos = 0;
      if (i < qc) {
        pos = uint32_t(QR[i]);
        e = sn_elem(wv[t]);
      }
      const uint32_t incl = sn_scan(e.len), o = d + incl - e.len;
      if (i < qc) {
        Q[i] = sn_qent(e, pos, o);
        SN_LDS_OR(OB + ((o - dr) >> 5), 1u << ((o - dr) & 31));
      }
      d += __builtin_amdgcn_readlane(incl, kWave - 1);
    }
    wave_sync();
    // element starts before each 64-bit word of OB (8 words a lane)
    {
      uint32_t cnt[8], tot = 0;
#pragma unroll
      for (uint32_t t = 0; t < 8; t++) {
        const uint32_t w = 8 * lane + t;
        cnt[t] = uint32_t(__builtin_popcountll(uint64_t(OB[2 * w]) | uint64_t(OB[2 * w + 1]) << 32));
        tot += cnt[t];
      }
      uint32_t run = sn_scan(tot) - tot;
#pragma unroll
      for (uint32_t t = 0; t < 8; t++) {
        PF[8 * lane + t] = uint16_t(run);
        run += cnt[t];
      }
    }
    // the round's copies, in order
    uint32_t cc = 0;
    for (uint32_t i0 = 0; i0 < qc; i0 += kWave) {
      const uint32_t i = i0 + lane;
      const bool isc = i < qc && (QR[i] >> 63);
      const uint64_t m = __ballot(isc);
      if (isc) CL[cc + uint32_t(__builtin_popcountll(m & ((1ull << lane) - 1)))] = uint16_t(i);
      cc += uint32_t(__builtin_popcountll(m));
    }
    wave_sync();
    SN_ACC(1, t0);
    SN_T(t1);
    // 3. copy sources
    sn4_resolve(QR, R, to_lds_ptr(static_cast<const uint16_t*>(S.cl)), to_lds_ptr(static_cast<const uint32_t*>(S.ob)),
                to_lds_ptr(static_cast<const uint16_t*>(S.pf)), cc, dr);
    SN_ACC(6, t1);
    SN_T(t1b);
    // 4. literals and resolved copies: lane per element, from the input
    for (uint32_t i0 = 0; i0 < qc; i0 += kWave) {
      const uint32_t i = i0 + lane;
      uint32_t len = 0, x = 0, o = 0;
      if (i < qc) {
        const uint64_t e = QR[i];
        o = sn_dst(e);
        len = sn_len(e);
        x = sn_src(e);
        if (e >> 63) {
          const uint32_t ri = R[i];
          if (ri & kSnRes) x = ri & ~kSnRes;
          else len = 0;
        }
      }
      if (len && len <= 256)
        for (uint32_t c = 0; c < len; c += 16) sn_store_n(dst + o + c, sn_load16c(src, x + c, n), len - c < 16 ? len - c : 16u);
      for (uint64_t m = __ballot(len > 256); m; m &= m - 1) {
        const int sl = __builtin_ctzll(m);
        const uint32_t lo = __builtin_amdgcn_readlane(o, sl), ls = __builtin_amdgcn_readlane(x, sl),
                       ll = __builtin_amdgcn_readlane(len, sl);
        for (uint32_t c = 16 * lane; c < ll; c += 16 * kWave)
          sn_store_n(dst + lo + c, sn_load16c(src, ls + c, n), ll - c < 16 ? ll - c : 16u);
      }
    }
    sn_fence();
    SN_ACC(2, t1b);
    SN_T(t2);
    // 5. the other copies in output order, groups of independent ones (sn_decode's)
    uint32_t g = 0;
    while (g < cc) {
      const uint32_t gi = g + lane;
      uint32_t j = 0, ri = kSnRes;
      if (gi < cc) {
        j = CL[gi];
        ri = R[j];
      }
      const bool isc = gi < cc && !(ri & kSnRes);
      const uint64_t cm = __ballot(isc);
      if (!cm) {
        g += kWave;
        continue;
      }
      const int first = __builtin_ctzll(cm);
      const uint64_t e = isc ? QR[j] : 0ull;
      const uint32_t o = sn_dst(e), len = sn_len(e), off = sn_src(e);
      const uint32_t d0 = __builtin_amdgcn_readlane(o, first);
      const bool ovl = off < len;
      const uint32_t P = ovl ? o - off : (ri & kSnPos);
      const bool indep = isc && (ovl ? o <= d0 : P + len <= d0);
      const uint64_t stop = first == 63 ? 0ull : (__ballot(isc && !indep) & ~((2ull << first) - 1));
      const uint32_t end = stop ? uint32_t(__builtin_ctzll(stop)) : uint32_t(kWave);
      if (isc && uint32_t(lane) >= uint32_t(first) && uint32_t(lane) < end) {
        const gptr<const uint8_t> sp = dst + P;
        if (!ovl || off >= 16) {
          for (uint32_t c = 0; c < len; c += 16) {
            const u32x4 v = *(gptr<const sn_u32x4_u>)(sp + c);
            sn_store_n(dst + o + c, make_uint4(v[0], v[1], v[2], v[3]), len - c < 16 ? len - c : 16u);
          }
        } else {
          uint8_t per[16];
          for (uint32_t k = 0; k < off; k++) per[k] = sp[k];
          for (uint32_t k = 0; k < len; k++) dst[o + k] = per[k % off];
        }
      }
      sn_fence();
      g += end;
#ifdef PBL_SNAP_STAMPS
      if (lane == 0 && g_sn_b < 65536) g_snap_stamps[8 * g_sn_b + 5] += 1;  // groups
#endif
    }
    SN_ACC(3, t2);
#ifdef PBL_SNAP_STAMPS
    if (lane == 0 && g_sn_b < 65536) g_snap_stamps[8 * g_sn_b + 4] += 1;  // rounds
#endif
  }
  return d == D;
}
