// zstd_dec.hip.h — the zstd frame decoder of zstd.hip (see there), written
// against a small set of wave primitives (lptr / gptr, lane_id, wave_sync,
// __shfl, __ballot, kWave) so that scripts/zstd_emu.cpp can run the same code
// on the host with 64 threads in lockstep for debugging.  Included by
// zstd.hip after common.hip.h.
#pragma once

namespace pbl {
namespace zstd {

constexpr uint32_t kIn = 28672;   // staged compressed bytes (LDS)
constexpr uint32_t kOut = 36864;  // decoded window (LDS)
constexpr uint32_t kSeq = 256;    // sequences decoded per execution round

enum : uint32_t { kOk = 0, kCorrupt = 1, kUnsupported = 2 };

struct Lds {
  alignas(16) uint8_t in[kIn + 48];
  uint8_t out[kOut + 32];
  uint32_t fse[3][512];  // LL, OF, ML: sym | nb << 8 | base << 16
  uint32_t wt[64];       // the Huffman weights' FSE table
  uint16_t huf[2048];    // sym | nb << 8
  uint32_t s_ll[kSeq], s_ml[kSeq], s_off[kSeq];
  uint8_t w[256];
  int16_t norm[256];
  uint16_t aux[256];
};


// ---- byte accessors ------------------------------------------------------------
struct LIn {
  lptr<const uint8_t> p;
  __device__ uint32_t operator[](uint32_t i) const { return p[i]; }
};
struct GIn {
  gptr<const uint8_t> p;
  __device__ uint32_t operator[](uint32_t i) const { return p[i]; }
};
// step(): between the 64-byte rounds of a copy whose later rounds read what
// earlier rounds wrote (or write what they read).  A wave's LDS accesses
// execute in order, so nothing is needed on the device; the host emulator
// (scripts/zstd_emu.cpp, PBL_ZSTD_EMU) runs lanes as threads and syncs them.
#ifndef PBL_ZSTD_EMU_STEP
#define PBL_ZSTD_EMU_STEP()
#endif
#ifndef PBL_ZSTD_EMU_MID  // (between a round's loads and its stores: one instruction each on the device)
#define PBL_ZSTD_EMU_MID()
#endif
struct LOut {
  lptr<uint8_t> p;
  __device__ uint32_t get(uint32_t i) const { return p[i]; }
  __device__ void set(uint32_t i, uint32_t v) const { p[i] = uint8_t(v); }
  __device__ void sync() const { wave_sync(); }
  __device__ void step() const { PBL_ZSTD_EMU_STEP(); }
};
struct GOut {
  gptr<uint8_t> p;
  __device__ uint32_t get(uint32_t i) const { return p[i]; }
  __device__ void set(uint32_t i, uint32_t v) const { p[i] = uint8_t(v); }
  __device__ void sync() const {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
  }
  __device__ void step() const { sync(); }
};

// o[dst + j] = o[src + j] for j < n, in 64-byte rounds (src < dst: a match
// whose source may overlap it at distance >= 64; src >= dst: a literal run
// moving down the window).
template <class O>
__device__ inline void copy_rounds(const O& o, uint32_t dst, uint32_t src, uint32_t n) {
  for (uint32_t j0 = 0; j0 < n; j0 += kWave) {
    const uint32_t j = j0 + lane_id();
    const uint32_t v = j < n ? o.get(src + j) : 0u;
    PBL_ZSTD_EMU_MID();
    if (j < n) o.set(dst + j, v);
    o.step();
  }
}

template <class S>
__device__ inline uint64_t le64(const S& s, uint32_t i) {
  uint64_t v = 0;
#pragma unroll
  for (int k = 0; k < 8; k++) v |= uint64_t(s[i + k]) << (8 * k);
  return v;
}
template <class S>
__device__ inline uint32_t le_n(const S& s, uint32_t i, uint32_t n) {
  uint32_t v = 0;
  for (uint32_t k = 0; k < n; k++) v |= s[i + k] << (8 * k);
  return v;
}

__device__ inline int highbit(uint32_t v) { return 31 - __builtin_clz(v); }

// Backward bitstream (RFC 8878 §4.1): unread bits [0, pos) of the stream at
// s[base, base + n); bits below 0 read as zeros.  A 64-bit container holds
// stream bits [cb, cb + 64) (it may read up to 7 bytes past the stream: the
// staging buffers and the physical trailer cover them).
template <class S>
struct BitR {
  S s;
  uint32_t base;
  int32_t pos, cb;
  uint64_t c;
  __device__ bool init(const S& src, uint32_t b, uint32_t n) {
    s = src;
    base = b;
    if (n == 0) return false;
    const uint32_t last = s[b + n - 1];
    if (last == 0) return false;
    pos = int32_t(8 * n) - 8 + highbit(last);
    refill();
    return true;
  }
  __device__ void refill() {
    int32_t b = (pos - 57) >> 3;
    if (b < 0) b = 0;
    cb = 8 * b;
    c = le64(s, base + uint32_t(b));
  }
  __device__ uint32_t read(uint32_t k) {
    if (k == 0) return 0;
    const int32_t lo = pos - int32_t(k);
    if (lo < cb && cb > 0) refill();  // (afterwards lo >= cb, or cb == 0 and lo < 0)
    uint64_t v;
    if (lo >= cb) v = c >> (lo - cb);
    else if (pos <= 0) v = 0;  // past the start: zeros
    else v = c << (-lo);       // cb == 0: the low bits are below the stream
    pos = lo;
    return uint32_t(v & ((1ull << k) - 1));
  }
  __device__ uint32_t peek(uint32_t k) {
    const int32_t p0 = pos;
    const uint32_t v = read(k);
    pos = p0;
    return v;
  }
};

// forward bits [bit, bit + k) of s[base, base + n) (zeros past its end), k <= 25
template <class S>
__device__ inline uint32_t fwd(const S& s, uint32_t base, uint32_t n, uint32_t bit, uint32_t k) {
  const uint32_t byte = bit >> 3;
  uint32_t v = 0;
  for (uint32_t i = 0; i < 4; i++) {
    const uint32_t q = byte + i;
    v |= (q < n ? s[base + q] : 0u) << (8 * i);
  }
  return (v >> (bit & 7)) & ((1u << k) - 1);
}

// FSE decoding table from norm[0, nsym) (lane 0).  T entries: sym | nb << 8 | base << 16.
// kSpread: stop after the symbol spread (T[u] = sym, next[] = the counts): the
// batch path finishes the table with the whole wave (zstd_fast.hip.h).
template <bool kSpread = false>
__device__ inline bool fse_build(lptr<uint32_t> T, lptr<const int16_t> norm, lptr<uint16_t> next, uint32_t nsym,
                                 uint32_t al) {
  const uint32_t size = 1u << al;
  int32_t high = int32_t(size) - 1;
  for (uint32_t s = 0; s < nsym; s++) {
    if (norm[s] == -1) {
      T[high--] = s;
      next[s] = 1;
    } else {
      next[s] = uint16_t(norm[s]);
    }
  }
  uint32_t pos = 0;
  const uint32_t step = (size >> 1) + (size >> 3) + 3, mask = size - 1;
  for (uint32_t s = 0; s < nsym; s++)
    for (int32_t i = 0; i < norm[s]; i++) {
      T[pos] = s;
      do pos = (pos + step) & mask;
      while (int32_t(pos) > high);
    }
  if (pos != 0) return false;
  if (kSpread) return true;
  for (uint32_t u = 0; u < size; u++) {
    const uint32_t s = T[u] & 0xff;
    const uint32_t x = next[s]++;
    const uint32_t nb = al - highbit(x);
    T[u] = s | nb << 8 | ((x << nb) - size) << 16;
  }
  return true;
}

// FSE_readNCount + build (lane 0).  Returns bytes used, or -1.
template <bool kSpread = false, class S, class LT>
__device__ inline int32_t fse_desc(lptr<uint32_t> T, LT& L, const S& s, uint32_t base, uint32_t n, uint32_t max_al,
                                   uint32_t max_sym, uint32_t* al_out) {
  lptr<int16_t> norm = to_lds_ptr(L.norm);
  uint32_t bit = 0;
  const uint32_t al = fwd(s, base, n, bit, 4) + 5;
  bit += 4;
  if (al > max_al) return -1;
  int32_t remaining = (1 << al) + 1, threshold = 1 << al, nbits = al + 1;
  uint32_t sym = 0;
  while (remaining > 1 && sym <= max_sym) {
    const int32_t mx = (2 * threshold - 1) - remaining;
    int32_t v;
    const int32_t low = int32_t(fwd(s, base, n, bit, nbits - 1));
    if (low < mx) {
      v = low;
      bit += nbits - 1;
    } else {
      v = int32_t(fwd(s, base, n, bit, nbits));
      if (v >= threshold) v -= mx;
      bit += nbits;
    }
    const int32_t prob = v - 1;
    remaining -= prob < 0 ? -prob : prob;
    norm[sym++] = int16_t(prob);
    if (prob == 0) {
      for (;;) {
        const uint32_t r = fwd(s, base, n, bit, 2);
        bit += 2;
        for (uint32_t i = 0; i < r && sym <= max_sym; i++) norm[sym++] = 0;
        if (r != 3 || bit > 8 * n) break;
      }
    }
    while (remaining < threshold && nbits > 1) {
      nbits--;
      threshold >>= 1;
    }
  }
  if (remaining != 1 || bit > 8 * n || sym > max_sym + 1) return -1;
  if (!fse_build<kSpread>(T, norm, to_lds_ptr(L.aux), sym, al)) return -1;
  *al_out = al;
  return int32_t((bit + 7) / 8);
}

__constant__ int16_t kLLDef[36] = {4, 3, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 1, 1, 1, 2, 2,
                                   2, 2, 2, 2, 2, 2, 2, 3, 2, 1, 1, 1, 1, 1, -1, -1, -1, -1};
__constant__ int16_t kMLDef[53] = {1, 4, 3, 2, 2, 2, 2, 2, 2, 1, 1, 1, 1, 1, 1, 1, 1, 1,
                                   1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1,
                                   1, 1, 1, 1, 1, 1, 1, 1, 1, 1, -1, -1, -1, -1, -1, -1, -1};
__constant__ int16_t kOFDef[29] = {1, 1, 1, 1, 1, 1, 2, 2, 2, 1, 1, 1, 1, 1, 1,
                                   1, 1, 1, 1, 1, 1, 1, 1, 1, -1, -1, -1, -1, -1};
__constant__ uint32_t kLLBase[36] = {0,  1,  2,  3,  4,  5,  6,   7,   8,   9,   10,   11,   12,   13,   14,    15,    16,    18,
                                     20, 22, 24, 28, 32, 40, 48, 64, 128, 256, 512, 1024, 2048, 4096, 8192, 16384, 32768, 65536};
__constant__ uint8_t kLLBits[36] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0,  0,  1,  1,
                                    1, 1, 2, 2, 3, 3, 4, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16};
__constant__ uint32_t kMLBase[53] = {3,  4,  5,  6,  7,  8,  9,  10, 11,  12,  13,  14,   15,   16,   17,   18,    19,    20,
                                     21, 22, 23, 24, 25, 26, 27, 28, 29,  30,  31,  32,   33,   34,   35,   37,    39,    41,
                                     43, 47, 51, 59, 67, 83, 99, 131, 259, 515, 1027, 2051, 4099, 8195, 16387, 32771, 65539};
__constant__ uint8_t kMLBits[53] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0,  0,  0,  0,  0,  0,  0,  0, 0,
                                    0, 0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 3, 3, 4, 4, 5, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16};

// Sequence table for mode m (lane 0): predefined / RLE / FSE / repeat.
// Returns bytes used or -1.
template <bool kSpread = false, class S, class LT>
__device__ inline int32_t seq_table(lptr<uint32_t> T, LT& L, uint32_t mode, const int16_t* def, uint32_t ndef,
                                    uint32_t def_al, uint32_t max_al, uint32_t max_sym, const S& s, uint32_t base,
                                    uint32_t n, uint32_t* al, bool* have) {
  if (mode == 0) {
    lptr<int16_t> norm = to_lds_ptr(L.norm);
    for (uint32_t i = 0; i < ndef; i++) norm[i] = def[i];
    fse_build<kSpread>(T, norm, to_lds_ptr(L.aux), ndef, def_al);
    *al = def_al;
    *have = true;
    return 0;
  }
  if (mode == 1) {
    if (n < 1 || s[base] > max_sym) return -1;
    T[0] = s[base];
    *al = 0;
    *have = true;
    return 1;
  }
  if (mode == 2) {
    const int32_t d = fse_desc<kSpread>(T, L, s, base, n, max_al, max_sym, al);
    if (d < 0) return -1;
    *have = true;
    return d;
  }
  return *have ? 0 : -1;
}

// Huffman tree description at s[base, base + n) -> L.huf (wave).  Returns bytes
// used or -1 (uniform).
template <class S, class LT>
__device__ inline int32_t huf_read(LT& L, const S& s, uint32_t base, uint32_t n, uint32_t* log_out) {
  const uint32_t lane = lane_id();
  if (n < 1) return -1;
  const uint32_t hb = s[base];
  int32_t used = -1;
  uint32_t nw = 0, log = 0;
  lptr<uint8_t> w = to_lds_ptr(L.w);
  if (lane == 0) {
    bool ok = true;
    if (hb >= 128) {
      nw = hb - 127;
      used = int32_t(1 + (nw + 1) / 2);
      if (uint32_t(used) > n) ok = false;
      for (uint32_t i = 0; ok && i < nw; i++) {
        const uint32_t x = s[base + 1 + i / 2];
        w[i] = uint8_t((i & 1) ? (x & 15) : (x >> 4));
      }
    } else {
      used = int32_t(1 + hb);
      if (uint32_t(used) > n || hb == 0) ok = false;
      uint32_t al = 0;
      const int32_t d = ok ? fse_desc(to_lds_ptr(L.wt), L, s, base + 1, hb, 6, 255, &al) : -1;
      if (d < 0 || uint32_t(d) >= hb) ok = false;
      BitR<S> br;
      if (ok && !br.init(s, base + 1 + d, hb - d)) ok = false;
      if (ok) {
        lptr<const uint32_t> T = to_lds_ptr(static_cast<const uint32_t*>(L.wt));
        uint32_t s1 = br.read(al), s2 = br.read(al);
        for (;;) {
          if (nw > 253) {
            ok = false;
            break;
          }
          uint32_t e = T[s1];
          w[nw++] = uint8_t(e);
          s1 = (e >> 16) + br.read((e >> 8) & 0xff);
          if (br.pos < 0) {
            w[nw++] = uint8_t(T[s2]);
            break;
          }
          e = T[s2];
          w[nw++] = uint8_t(e);
          s2 = (e >> 16) + br.read((e >> 8) & 0xff);
          if (br.pos < 0) {
            w[nw++] = uint8_t(T[s1]);
            break;
          }
        }
      }
    }
    uint32_t sum = 0;
    for (uint32_t i = 0; ok && i < nw; i++) {
      if (w[i] > 11) ok = false;
      else if (w[i]) sum += 1u << (w[i] - 1);
    }
    if (ok && sum == 0) ok = false;
    if (ok) {
      log = highbit(sum) + 1;
      const uint32_t rest = (1u << log) - sum;
      if (log > 11 || (rest & (rest - 1))) ok = false;
      else w[nw++] = uint8_t(highbit(rest) + 1);
    }
    if (ok) {
      // HUF_readDTableX1: weight 1 first, symbols in order within a weight
      uint32_t cnt[13] = {0}, start[13] = {0};
      for (uint32_t i = 0; i < nw; i++) cnt[w[i]]++;
      uint32_t acc = 0;
      for (uint32_t k = 1; k <= log; k++) {
        start[k] = acc;
        acc += cnt[k] << (k - 1);
      }
      lptr<uint16_t> st = to_lds_ptr(L.aux);
      for (uint32_t i = 0; i < nw; i++) {
        const uint32_t k = w[i];
        st[i] = uint16_t(k ? start[k] : 0);
        if (k) start[k] += 1u << (k - 1);
      }
    }
    if (!ok) used = -1;
  }
  used = __shfl(used, 0, kWave);
  nw = __shfl(nw, 0, kWave);
  log = __shfl(log, 0, kWave);
  wave_sync();
  if (used < 0) return -1;
  lptr<uint16_t> H = to_lds_ptr(L.huf);
  lptr<const uint16_t> st = to_lds_ptr(static_cast<const uint16_t*>(L.aux));
  for (uint32_t i = lane; i < nw; i += kWave) {
    const uint32_t k = w[i];
    if (!k) continue;
    const uint32_t e = i | (log + 1 - k) << 8, s0 = st[i], len = 1u << (k - 1);
    for (uint32_t u = 0; u < len; u++) H[s0 + u] = uint16_t(e);
  }
  wave_sync();
  *log_out = log;
  return used;
}

// Decoder state carried across the blocks of a frame (uniform registers).
struct ZState {
  uint32_t huf_log, al_ll, al_of, al_ml;
  bool have_ll, have_of, have_ml;
  uint32_t rep0, rep1, rep2;
};

// One compressed block at s[base, base + n); output window o[0, D); the frame
// starts at o[start]; *pos advances.  Uniform return: kOk / kCorrupt.
template <class S, class O>
__device__ uint32_t comp_block(Lds& L, ZState& Z, const S& s, uint32_t base, uint32_t n, const O& o, uint32_t D,
                               uint32_t start, uint32_t* pos_io) {
  const uint32_t lane = lane_id();
  if (n < 1) return kCorrupt;
  const uint32_t b0 = s[base], ltype = b0 & 3, sf = (b0 >> 2) & 3;
  uint32_t h, regen, csize = 0, streams = 1;
  if (ltype < 2) {
    if (sf == 0 || sf == 2) {
      h = 1;
      regen = b0 >> 3;
    } else if (sf == 1) {
      h = 2;
      if (n < 2) return kCorrupt;
      regen = (b0 >> 4) + (s[base + 1] << 4);
    } else {
      h = 3;
      if (n < 3) return kCorrupt;
      regen = (b0 >> 4) + (s[base + 1] << 4) + (s[base + 2] << 12);
    }
  } else {
    if (sf < 2) {
      h = 3;
      if (n < 3) return kCorrupt;
      regen = (b0 >> 4) + ((s[base + 1] & 0x3f) << 4);
      csize = (s[base + 1] >> 6) + (s[base + 2] << 2);
      streams = sf == 0 ? 1 : 4;
    } else if (sf == 2) {
      h = 4;
      if (n < 4) return kCorrupt;
      regen = (b0 >> 4) + (s[base + 1] << 4) + ((s[base + 2] & 3) << 12);
      csize = (s[base + 2] >> 2) + (s[base + 3] << 6);
      streams = 4;
    } else {
      h = 5;
      if (n < 5) return kCorrupt;
      regen = (b0 >> 4) + (s[base + 1] << 4) + ((s[base + 2] & 0x3f) << 12);
      csize = (s[base + 2] >> 6) + (s[base + 3] << 2) + (s[base + 4] << 10);
      streams = 4;
    }
  }
  uint32_t pos = *pos_io;
  if (regen > (1u << 17) || regen > D - pos) return kCorrupt;
  const uint32_t lit0 = D - regen;  // literals at the end of the window
  uint32_t q = base + h;
  if (ltype == 0) {
    if (h + regen > n) return kCorrupt;
    for (uint32_t i = lane; i < regen; i += kWave) o.set(lit0 + i, s[q + i]);
    q += regen;
  } else if (ltype == 1) {
    if (h + 1 > n) return kCorrupt;
    const uint32_t v = s[q];
    for (uint32_t i = lane; i < regen; i += kWave) o.set(lit0 + i, v);
    q += 1;
  } else {
    if (h + csize > n) return kCorrupt;
    uint32_t c = q, cn = csize;
    if (ltype == 2) {
      const int32_t t = huf_read(L, s, c, cn, &Z.huf_log);
      if (t < 0) return kCorrupt;
      c += t;
      cn -= t;
    } else if (!Z.huf_log) {
      return kCorrupt;
    }
    uint32_t so = c, sl = cn, cnt = regen, d0 = lit0;
    bool bad = false;
    if (streams == 4) {
      if (cn < 6) return kCorrupt;
      const uint32_t l1 = s[c] | s[c + 1] << 8, l2 = s[c + 2] | s[c + 3] << 8, l3 = s[c + 4] | s[c + 5] << 8;
      if (6 + l1 + l2 + l3 > cn) return kCorrupt;
      const uint32_t seg = (regen + 3) / 4;
      if (3 * seg > regen) return kCorrupt;
      const uint32_t ls[4] = {l1, l2, l3, cn - 6 - l1 - l2 - l3};
      so = c + 6;
      for (uint32_t i = 0; i < 4 && i < lane; i++) so += ls[i];
      sl = lane < 4 ? ls[lane < 4 ? lane : 0] : 0;
      cnt = lane < 3 ? seg : regen - 3 * seg;
      d0 = lit0 + (lane < 4 ? lane : 0) * seg;
    }
    if (lane < streams) {
      BitR<S> br;
      if (!br.init(s, so, sl)) {
        bad = true;
      } else {
        lptr<const uint16_t> H = to_lds_ptr(static_cast<const uint16_t*>(L.huf));
        const uint32_t lg = Z.huf_log;
        for (uint32_t i = 0; i < cnt; i++) {
          const uint32_t e = H[br.peek(lg)];
          o.set(d0 + i, e & 0xff);
          br.pos -= int32_t(e >> 8);
        }
        if (br.pos != 0) bad = true;
      }
    }
    if (__ballot(bad)) return kCorrupt;
    q += csize;
  }
  o.sync();
  // sequences section
  const uint32_t end = base + n;
  if (q >= end) return kCorrupt;
  uint32_t nseq = s[q];
  if (nseq < 128) {
    q += 1;
  } else if (nseq < 255) {
    if (q + 2 > end) return kCorrupt;
    nseq = ((nseq - 128) << 8) + s[q + 1];
    q += 2;
  } else {
    if (q + 3 > end) return kCorrupt;
    nseq = s[q + 1] + (s[q + 2] << 8) + 0x7F00;
    q += 3;
  }
  uint32_t lp = 0;  // literals consumed
  if (nseq > 0) {
    if (q >= end) return kCorrupt;
    const uint32_t modes = s[q++];
    if (modes & 3) return kCorrupt;
    int32_t u = 0;
    if (lane == 0) {
      u = seq_table(to_lds_ptr(L.fse[0]), L, modes >> 6, kLLDef, 36, 6, 9, 35, s, q, end - q, &Z.al_ll, &Z.have_ll);
      int32_t u2 = u < 0 ? -1
                         : seq_table(to_lds_ptr(L.fse[1]), L, (modes >> 4) & 3, kOFDef, 29, 5, 8, 31, s, q + u,
                                     end - q - u, &Z.al_of, &Z.have_of);
      int32_t u3 = u2 < 0 ? -1
                          : seq_table(to_lds_ptr(L.fse[2]), L, (modes >> 2) & 3, kMLDef, 53, 6, 9, 52, s,
                                      q + u + u2, end - q - u - u2, &Z.al_ml, &Z.have_ml);
      u = u3 < 0 ? -1 : u + u2 + u3;
    }
    u = __shfl(u, 0, kWave);
    Z.al_ll = __shfl(Z.al_ll, 0, kWave);
    Z.al_of = __shfl(Z.al_of, 0, kWave);
    Z.al_ml = __shfl(Z.al_ml, 0, kWave);
    Z.have_ll = __shfl(int(Z.have_ll), 0, kWave);
    Z.have_of = __shfl(int(Z.have_of), 0, kWave);
    Z.have_ml = __shfl(int(Z.have_ml), 0, kWave);
    wave_sync();
    if (u < 0) return kCorrupt;
    q += u;
    // lane 0's bit reader and states persist across rounds
    BitR<S> br;
    uint32_t stl = 0, sto = 0, stm = 0;
    bool okb = true;
    if (lane == 0) {
      okb = br.init(s, q, end - q);
      if (okb) {
        stl = br.read(Z.al_ll);
        sto = br.read(Z.al_of);
        stm = br.read(Z.al_ml);
      }
    }
    if (!__shfl(int(okb), 0, kWave)) return kCorrupt;
    lptr<const uint32_t> TL = to_lds_ptr(static_cast<const uint32_t*>(L.fse[0]));
    lptr<const uint32_t> TO = to_lds_ptr(static_cast<const uint32_t*>(L.fse[1]));
    lptr<const uint32_t> TM = to_lds_ptr(static_cast<const uint32_t*>(L.fse[2]));
    for (uint32_t r0 = 0; r0 < nseq; r0 += kSeq) {
      const uint32_t m = min(kSeq, nseq - r0);
      bool bad = false;
      if (lane == 0) {
        for (uint32_t i = 0; i < m; i++) {
          const uint32_t el = TL[stl], eo = TO[sto], em = TM[stm];
          const uint32_t oc = eo & 0xff, mc = em & 0xff, lc = el & 0xff;
          if (oc > 31) {
            bad = true;
            break;
          }
          const uint32_t ofv = (1u << oc) + br.read(oc);  // (oc = 31 wraps only on corrupt input)
          const uint32_t ml = kMLBase[mc] + br.read(kMLBits[mc]);
          const uint32_t ll = kLLBase[lc] + br.read(kLLBits[lc]);
          if (r0 + i + 1 < nseq) {
            stl = (el >> 16) + br.read((el >> 8) & 0xff);
            stm = (em >> 16) + br.read((em >> 8) & 0xff);
            sto = (eo >> 16) + br.read((eo >> 8) & 0xff);
          }
          uint32_t off;
          if (ofv > 3) {
            off = ofv - 3;
            Z.rep2 = Z.rep1;
            Z.rep1 = Z.rep0;
            Z.rep0 = off;
          } else {
            const uint32_t k = ofv - 1 + (ll == 0);
            if (k == 0) {
              off = Z.rep0;
            } else {
              off = k == 3 ? Z.rep0 - 1u : (k == 1 ? Z.rep1 : Z.rep2);
              if (k != 1) Z.rep2 = Z.rep1;
              Z.rep1 = Z.rep0;
              Z.rep0 = off;
            }
          }
          L.s_ll[i] = ll;
          L.s_ml[i] = ml;
          L.s_off[i] = off;
        }
        if (r0 + m == nseq && !bad && br.pos != 0) bad = true;
      }
      if (__shfl(int(bad), 0, kWave)) return kCorrupt;
      wave_sync();
      for (uint32_t i = 0; i < m; i++) {
        const uint32_t ll = L.s_ll[i], ml = L.s_ml[i], off = L.s_off[i];
        if (ll > regen - lp || ml > D - pos || ll > D - pos - ml) return kCorrupt;
        // literal run: the window's literal bytes sit at or after the output
        // (dst <= src), so a forward copy by 64-byte rounds never overwrites
        // bytes a later round still reads
        copy_rounds(o, pos, lit0 + lp, ll);
        lp += ll;
        pos += ll;
        o.sync();
        if (off == 0 || off > pos - start) return kCorrupt;
        if (off >= kWave) {
          copy_rounds(o, pos, pos - off, ml);
        } else {
          for (uint32_t j = lane; j < ml; j += kWave) o.set(pos + j, o.get(pos - off + (j % off)));
        }
        pos += ml;
        o.sync();
      }
    }
    Z.rep0 = __shfl(Z.rep0, 0, kWave);
    Z.rep1 = __shfl(Z.rep1, 0, kWave);
    Z.rep2 = __shfl(Z.rep2, 0, kWave);
  } else if (q != end) {
    return kCorrupt;
  }
  const uint32_t rest = regen - lp;
  if (rest > D - pos) return kCorrupt;
  copy_rounds(o, pos, lit0 + lp, rest);
  o.sync();
  *pos_io = pos + rest;
  return kOk;
}

// XXH64 of o[a, a + n) by lane 0 (content checksum).
template <class O>
__device__ inline uint32_t xxh64_lo(const O& o, uint32_t a, uint32_t n) {
  constexpr uint64_t P1 = 11400714785074694791ull, P2 = 14029467366897019727ull, P3 = 1609587929392839161ull,
                     P4 = 9650029242287828579ull, P5 = 2870177450012600261ull;
  auto rotl = [](uint64_t x, int r) { return (x << r) | (x >> (64 - r)); };
  auto rd = [&](uint32_t i, uint32_t k) {
    uint64_t v = 0;
    for (uint32_t t = 0; t < k; t++) v |= uint64_t(o.get(i + t)) << (8 * t);
    return v;
  };
  auto round = [&](uint64_t acc, uint64_t in) { return rotl(acc + in * P2, 31) * P1; };
  uint64_t h;
  uint32_t p = a;
  const uint32_t e = a + n;
  if (n >= 32) {
    uint64_t v1 = P1 + P2, v2 = P2, v3 = 0, v4 = 0 - P1;
    for (; p + 32 <= e; p += 32) {
      v1 = round(v1, rd(p, 8));
      v2 = round(v2, rd(p + 8, 8));
      v3 = round(v3, rd(p + 16, 8));
      v4 = round(v4, rd(p + 24, 8));
    }
    h = rotl(v1, 1) + rotl(v2, 7) + rotl(v3, 12) + rotl(v4, 18);
    h = (h ^ round(0, v1)) * P1 + P4;
    h = (h ^ round(0, v2)) * P1 + P4;
    h = (h ^ round(0, v3)) * P1 + P4;
    h = (h ^ round(0, v4)) * P1 + P4;
  } else {
    h = P5;
  }
  h += n;
  for (; p + 8 <= e; p += 8) {
    h ^= round(0, rd(p, 8));
    h = rotl(h, 27) * P1 + P4;
  }
  if (p + 4 <= e) {
    h ^= rd(p, 4) * P1;
    h = rotl(h, 23) * P2 + P3;
    p += 4;
  }
  for (; p < e; p++) {
    h ^= o.get(p) * P5;
    h = rotl(h, 11) * P1;
  }
  h ^= h >> 33;
  h *= P2;
  h ^= h >> 29;
  h *= P3;
  h ^= h >> 32;
  return uint32_t(h);
}

// ZSTD_decompressDCtx of s[base, base + n) into o[0, D): every frame (skippable
// ones passed over) back to back, exactly D bytes.  Uniform status.
template <class S, class O>
__device__ uint32_t decode_frames(Lds& L, const S& s, uint32_t base, uint32_t n, const O& o, uint32_t D) {
  const uint32_t lane = lane_id();
  uint32_t q = base, pos = 0;
  const uint32_t end = base + n;
  if (n == 0) return kCorrupt;
  while (q < end) {
    if (end - q < 4) return kCorrupt;
    const uint32_t magic = le_n(s, q, 4);
    if ((magic & 0xFFFFFFF0u) == 0x184D2A50u) {
      if (end - q < 8) return kCorrupt;
      const uint32_t sz = le_n(s, q + 4, 4);
      if (sz > end - q - 8) return kCorrupt;
      q += 8 + sz;
      continue;
    }
    if (magic != 0xFD2FB528u) return kCorrupt;
    q += 4;
    if (q >= end) return kCorrupt;
    const uint32_t fhd = s[q++];
    const uint32_t fcs_flag = fhd >> 6, single = (fhd >> 5) & 1, cksum = (fhd >> 2) & 1, did = fhd & 3;
    if (fhd & 8) return kCorrupt;
    if (!single) {
      if (q >= end) return kCorrupt;
      q++;  // window descriptor (the whole block is resident: no window limit applies)
    }
    const uint32_t dl = did == 0 ? 0 : did == 1 ? 1 : did == 2 ? 2 : 4;
    if (end - q < dl) return kCorrupt;
    const uint32_t dict = le_n(s, q, dl);
    q += dl;
    if (dict) return kUnsupported;
    const uint32_t fl = fcs_flag == 0 ? (single ? 1 : 0) : fcs_flag == 1 ? 2 : fcs_flag == 2 ? 4 : 8;
    if (end - q < fl) return kCorrupt;
    uint64_t fcs = 0;
    for (uint32_t i = 0; i < fl; i++) fcs |= uint64_t(s[q + i]) << (8 * i);
    if (fl == 2) fcs += 256;
    q += fl;
    ZState Z{0, 0, 0, 0, false, false, false, 1, 4, 8};
    const uint32_t start = pos;
    for (;;) {
      if (end - q < 3) return kCorrupt;
      const uint32_t bh = s[q] | s[q + 1] << 8 | s[q + 2] << 16;
      q += 3;
      const uint32_t last = bh & 1, type = (bh >> 1) & 3, bs = bh >> 3;
      if (type == 3) return kCorrupt;
      if (type == 1) {
        if (q + 1 > end || bs > D - pos) return kCorrupt;
        const uint32_t v = s[q];
        for (uint32_t i = lane; i < bs; i += kWave) o.set(pos + i, v);
        o.sync();
        pos += bs;
        q += 1;
      } else {
        if (bs > end - q || bs > (1u << 17)) return kCorrupt;
        if (type == 0) {
          if (bs > D - pos) return kCorrupt;
          for (uint32_t i = lane; i < bs; i += kWave) o.set(pos + i, s[q + i]);
          o.sync();
          pos += bs;
        } else {
          const uint32_t r = comp_block(L, Z, s, q, bs, o, D, start, &pos);
          if (r != kOk) return r;
        }
        q += bs;
      }
      if (last) break;
    }
    if (fl && uint64_t(pos - start) != fcs) return kCorrupt;
    if (cksum) {
      if (end - q < 4) return kCorrupt;
      uint32_t h = 0;
      if (lane == 0) h = xxh64_lo(o, start, pos - start);
      h = __shfl(h, 0, kWave);
      if (h != le_n(s, q, 4)) return kCorrupt;
      q += 4;
    }
  }
  return pos == D ? kOk : kCorrupt;
}

}  // namespace zstd
}  // namespace pbl
