// snappy_dec.hip.h — the snappy block decoder of snappy2_kernel (physical.hip),
// written against a small set of wave primitives (lptr / gptr, lane_id,
// wave_sync, __shfl, __ballot, readfirstlane, alignbyte) so that
// scripts/snappy_emu.cpp can run the same code on the host with 64 threads in
// lockstep.  Included by physical.hip inside namespace pbl::phys, after
// kSnIn / kSnQ and the SN_T / SN_ACC stamp macros.
#pragma once

struct Snap2Lds {
  alignas(16) uint32_t in[(kSnIn + 64) / 4];  // compressed bytes at their 16-B phase (+ slack)
  uint64_t q[kSnQ];               // dst | len << 16 | (src or offset) << 32 | copy << 63
  uint32_t r[kSnQ];               // copies: where their bytes are (see sn_resolve)
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

// Lane 0: queue the elements starting at input offset *s (output offset *d)
// until the queue or the input is full.  Returns the count; *ok clears on a
// corrupt element (snappy.Decode's ErrCorrupt cases).
// The whole wave runs it with uniform values (the LDS words are read by every
// lane at one address and made scalar with readfirstlane), so the element
// walk's arithmetic and branches are scalar; lane 0 writes the queue.
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
    const uint32_t t = uint32_t(w) & 0xff, kind = t & 3, ext = uint32_t(w >> 8);
    uint32_t len, h;
    uint64_t e;
    if (kind == 0) {
      uint32_t x = t >> 2;
      h = 1;
      if (x >= 60) {
        const uint32_t nb = x - 59;
        h = 1 + nb;
        x = ext & (nb == 4 ? 0xffffffffu : (1u << (8 * nb)) - 1u);
      }
      len = x + 1;  // (x = 2^32 - 1 wraps to 0: rejected)
      if (h > n - s || len == 0 || len > n - s - h || len > D - d) { *ok = false; break; }
      e = uint64_t(d) | uint64_t(len) << 16 | uint64_t(s + h) << 32;
      s += h + len;
    } else {
      uint32_t off;
      if (kind == 1) {
        h = 2;
        len = 4 + ((t >> 2) & 7);
        off = ((t & 0xe0) << 3) | (ext & 0xff);
      } else {
        h = kind == 2 ? 3 : 5;
        len = 1 + (t >> 2);
        off = kind == 2 ? (ext & 0xffff) : ext;
      }
      if (h > n - s || off == 0 || off > d || len > D - d) { *ok = false; break; }
      e = uint64_t(d) | uint64_t(len) << 16 | uint64_t(off) << 32 | (1ull << 63);
      s += h;
    }
    if (l0) Q[c] = e;
    c++;
    d += len;
  }
  *s_io = s;
  *d_io = d;
  return c;
}

// Copy sources resolved to the INPUT by pointer jumping.  r[j] of copy j holds
// a position whose bytes equal the copy's source: first its output position
// o - off, then, hop by hop, the source of the element whose output contains
// that range (a literal: its input bytes -> resolved, kSnRes | input offset; a
// copy without self-overlap: that copy's own r), so a chain of copies of
// copies collapses in log rounds.  A range that straddles elements, reaches
// before this round's queue or into a self-overlapping copy stays kSnStuck and
// is copied from the output afterwards.  Races between lanes are benign: every
// value r[k] takes is a valid source of copy k's bytes.
constexpr uint32_t kSnRes = 1u << 31, kSnStuck = 1u << 30;
__device__ __forceinline__ uint32_t sn_find(const lptr<const uint64_t> Q, uint32_t qc, uint32_t a) {
  uint32_t lo = 0, hi = qc;  // the last element with dst <= a (qc when before the first)
  if ((uint32_t(Q[0]) & 0xffffu) > a) return qc;
  while (hi - lo > 1) {
    const uint32_t mid = (lo + hi) >> 1;
    if ((uint32_t(Q[mid]) & 0xffffu) <= a) lo = mid;
    else hi = mid;
  }
  return lo;
}
__device__ __forceinline__ void sn_resolve(lptr<const uint64_t> QR, lptr<uint32_t> R, uint32_t qc) {
  const uint32_t lane = lane_id();
  for (uint32_t j = lane; j < qc; j += kWave) {
    const uint64_t e = QR[j];
    if (e >> 63) {
      const uint32_t o = uint32_t(e) & 0xffffu, len = uint32_t(e >> 16) & 0xffffu, off = uint32_t(e >> 32) & 0x7fffffffu;
      R[j] = off < len ? kSnStuck : o - off;
    }
  }
  wave_sync();
  for (int round = 0; round < 12; round++) {
    bool open = false;
    for (uint32_t j = lane; j < qc; j += kWave) {
      const uint64_t e = QR[j];
      if (!(e >> 63)) continue;
      const uint32_t rj = R[j];
      if (rj & (kSnRes | kSnStuck)) continue;
      const uint32_t len = uint32_t(e >> 16) & 0xffffu;
      const uint32_t k = sn_find(QR, qc, rj);
      uint32_t nr = kSnStuck;
      if (k < qc) {
        const uint64_t ek = QR[k];
        const uint32_t dk = uint32_t(ek) & 0xffffu, lk = uint32_t(ek >> 16) & 0xffffu;
        if (rj + len <= dk + lk) {
          if (!(ek >> 63)) {
            nr = kSnRes | ((uint32_t(ek >> 32) & 0x7fffffffu) + (rj - dk));
          } else {
            const uint32_t rk = R[k];
            if (rk & kSnRes) nr = kSnRes | ((rk & ~kSnRes) + (rj - dk));
            else if (!(rk & kSnStuck)) { nr = rk + (rj - dk); open = true; }
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

// One snappy block: compressed bytes staged at byte ib of W (n bytes, the
// uvarint header included), D decoded bytes to dst.  Uniform result: false = corrupt.
__device__ bool sn_decode(Snap2Lds& S, uint32_t ib, uint32_t n, uint32_t used, uint32_t D, gptr<uint8_t> dst,
                          uint32_t g_sn_b = 0) {
  const uint32_t lane = lane_id();
  (void)g_sn_b;
  lptr<const uint32_t> W = to_lds_ptr(static_cast<const uint32_t*>(S.in));
  lptr<uint64_t> Q = to_lds_ptr(S.q);
  const lptr<const uint64_t> QR = to_lds_ptr(static_cast<const uint64_t*>(S.q));
  lptr<uint32_t> R = to_lds_ptr(S.r);
  uint32_t s = used, d = 0;
  bool ok = true;
  while (s < n) {
    uint32_t qc = 0;
    SN_T(t0);
    qc = sn_parse(W, ib, Q, n, D, &s, &d, &ok);
    if (!ok) return false;
    wave_sync();
    SN_ACC(1, t0);
    SN_T(t1);
    sn_resolve(QR, R, qc);
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
    SN_ACC(2, t1);
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
      const uint32_t d0 = __shfl(o, first, kWave);
      // bytes read below its own output: [o - off, o - off + min(len, off))
      const bool indep = isc && (o - off + (len < off ? len : off) <= d0);
      const uint64_t stop = first == 63 ? 0ull : (__ballot(isc && !indep) & ~((2ull << first) - 1));
      const uint32_t end = stop ? uint32_t(__builtin_ctzll(stop)) : uint32_t(kWave);  // lanes [first, end) run
      if (isc && uint32_t(lane) >= uint32_t(first) && uint32_t(lane) < end) {
        const gptr<const uint8_t> sp = dst + (o - off);
        if (off >= 16) {
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

