// physical.hip — the physical-block step before data-block decode, on the
// device: checksum validation and decompression of blocks
// as they sit in an SST file, [block bytes][compression indicator u8]
// [checksum LE32] (sstable/block/block.go:539-571).
//
//   checksum_crc_kernel   CRC32C (internal/crc/crc.go): one wave per block;
//                         lane l CRCs the 16-B granules l, l+64, ... (coalesced
//                         1 KiB wave loads, slicing-by-16 tables in LDS), carrying
//                         its state across the 1008-B gaps by a constant GF(2)
//                         multiply; the lane states combine by shift and XOR
//                         (the CRC is linear), then Value()'s rotation + delta
//   checksum_xxh_kernel   XXH64 truncated to 32 bits (cespare/xxhash/v2, the
//                         ChecksumTypeXXHash64 of block.go:155-160): one lane
//                         per block (XXH64's stripes are sequential)
//   snappy_len_kernel     the decoded length (uvarint header, snappy.DecodedLen)
//   snappy_walk_kernel    snappy.Decode (golang/snappy block format), step 1:
//                         each block's element chain walked and validated on
//                         one lane (64 blocks a wave), a tag bitmap left in
//                         the block's output region (snappy_dec.hip.h)
//   snappy4_kernel        step 2, a wave per walked block, nothing staged:
//                         elements decoded a lane each, copy chains resolved
//                         by pointer jumping (to the input where they lead to
//                         a literal), literals and resolved copies written in
//                         parallel, the rest in groups of independent copies
//   snappy2_kernel        the other blocks (uncompressed copies, snappy blocks
//                         the walk does not cover): one wave per block, the
//                         input staged in LDS, the elements walked by the wave
//                         with scalar arithmetic, then snappy4's phases
//   zstd_kernel           (zstd.hip) the blocks whose indicator is zstd
//   minlz_kernel          (minlz_dec.hip.h) MinLZ blocks in the MinLZ form; a
//                         MinLZ-indicated block in the Snappy form (first byte
//                         not 0: minlz_test.go:31-36) takes the snappy kernels
// Unknown indicators report PBL_UNSUPPORTED.
#include <algorithm>

#include "common.hip.h"
#include "colblk_block.hip.h"

namespace pbl {
hipError_t launch_zstd(const pbl_phys_batch& batch, uint8_t* out, const uint64_t* out_off, const uint32_t* out_cap,
                       uint32_t* out_len, uint32_t* status, hipStream_t st);
namespace phys {

constexpr uint32_t kPoly = 0x82F63B78u;  // reflected Castagnoli

// GF(2) polynomial product a*b mod P, reflected (zlib's multmodp)
__device__ inline uint32_t multmodp(uint32_t a, uint32_t b) {
  uint32_t m = 1u << 31, p = 0;
  for (;;) {
    if (a & m) {
      p ^= b;
      if ((a & (m - 1)) == 0) break;
    }
    m >>= 1;
    b = (b & 1) ? (b >> 1) ^ kPoly : b >> 1;
  }
  return p;
}

// Tables: slicing-by-16 (T[k][b] = CRC of byte b followed by k zero bytes) and
// multiplication by the constant K = x^(8*1008) mod P split by byte.
constexpr uint32_t kGap = 63 * 16;  // bytes between a lane's consecutive granules
struct CrcLds {
  uint32_t t[16][256];
  uint32_t m[4][256];
  uint32_t x2n[32];  // x^(2^k) mod P
};

__device__ inline void crc_tables(CrcLds& L) {
  for (uint32_t i = threadIdx.x; i < 256; i += blockDim.x) {
    uint32_t c = i;
    for (int k = 0; k < 8; k++) c = (c & 1) ? (c >> 1) ^ kPoly : c >> 1;
    L.t[0][i] = c;
  }
  if (threadIdx.x == 0) {
    uint32_t p = 1u << 30;  // x^1
    L.x2n[0] = p;
    for (int k = 1; k < 32; k++) L.x2n[k] = p = multmodp(p, p);
  }
  __syncthreads();
  for (uint32_t i = threadIdx.x; i < 256; i += blockDim.x) {
    uint32_t c = L.t[0][i];
    for (int k = 1; k < 16; k++) {
      c = L.t[0][c & 0xff] ^ (c >> 8);
      L.t[k][i] = c;
    }
  }
  __syncthreads();
}

// x^(8n) mod P
__device__ inline uint32_t x8nmodp(const CrcLds& L, uint64_t n) {
  uint32_t p = 1u << 31;  // x^0
  int k = 3;
  while (n) {
    if (n & 1) p = multmodp(L.x2n[k & 31], p);
    n >>= 1;
    k++;
  }
  return p;
}

__device__ inline void crc_mul_tables(CrcLds& L) {
  __shared__ uint32_t K;
  if (threadIdx.x == 0) K = x8nmodp(L, kGap);
  __syncthreads();
  for (uint32_t e = threadIdx.x; e < 1024; e += blockDim.x) L.m[e >> 8][e & 255] = multmodp(K, (e & 255u) << (8 * (e >> 8)));
  __syncthreads();
}

// raw (unconditioned) CRC update of state s by 16 bytes w (slicing-by-16)
__device__ __forceinline__ uint32_t crc16(const CrcLds& L, uint32_t s, const uint4& w) {
  const uint32_t a = w.x ^ s;
  return L.t[15][a & 0xff] ^ L.t[14][(a >> 8) & 0xff] ^ L.t[13][(a >> 16) & 0xff] ^ L.t[12][a >> 24] ^
         L.t[11][w.y & 0xff] ^ L.t[10][(w.y >> 8) & 0xff] ^ L.t[9][(w.y >> 16) & 0xff] ^ L.t[8][w.y >> 24] ^
         L.t[7][w.z & 0xff] ^ L.t[6][(w.z >> 8) & 0xff] ^ L.t[5][(w.z >> 16) & 0xff] ^ L.t[4][w.z >> 24] ^
         L.t[3][w.w & 0xff] ^ L.t[2][(w.w >> 8) & 0xff] ^ L.t[1][(w.w >> 16) & 0xff] ^ L.t[0][w.w >> 24];
}
// s * x^(8*kGap) mod P
__device__ __forceinline__ uint32_t crc_gap(const CrcLds& L, uint32_t s) {
  return L.m[0][s & 0xff] ^ L.m[1][(s >> 8) & 0xff] ^ L.m[2][(s >> 16) & 0xff] ^ L.m[3][s >> 24];
}

// Data granule j (bytes [16j, 16j+16) of the block) from global memory: one
// aligned load, or two and a funnel shift when the block is not 16-B aligned
// (the batch is readable to the next 16-B boundary past every block's trailer).
__device__ __forceinline__ uint4 granule(gptr<const uint8_t> base, uint32_t sh, uint32_t j) {
  const gptr<const u32x4> a = (gptr<const u32x4>)(base - sh + 16ull * j);
  const u32x4 x = a[0];
  const uint4 x4 = make_uint4(x.x, x.y, x.z, x.w);
  if (!sh) return x4;
  const u32x4 y = a[1];
  return col::funnel16(x4, make_uint4(y.x, y.y, y.z, y.w), sh);
}

// One wave per block.  Lane l takes the 16-B granules l, l+64, l+128, ... (each
// wave load is 1 KiB contiguous); its raw CRC is carried across the 1008-byte
// gaps by the constant multiply, the 64 lane states are shifted to the end of
// the data and XORed, the < 16-byte tail is added by lane 0, and the init ~0
// enters as x^(8n) * ~0 (linearity of the CRC).  Then Go's final complement and
// crc.CRC.Value()'s rotation and delta.
__global__ void __launch_bounds__(kTPB) checksum_crc_kernel(const pbl_phys_batch B, uint32_t* status,
                                                            uint32_t* computed) {
  __shared__ CrcLds L;
  crc_tables(L);
  crc_mul_tables(L);
  const uint32_t lane = lane_id(), wpb = kTPB / kWave;
  for (uint32_t b = blockIdx.x * wpb + wave_id(); b < B.n_blocks; b += gridDim.x * wpb) {
    const uint64_t n = uint64_t(B.block_len[b]) + 1;  // the block and its compression indicator
    const uint64_t off = B.block_off[b];
    const gptr<const uint8_t> p = to_glb(B.bytes + off);
    const uint32_t sh = uint32_t(off & 15);
    const uint64_t G = n >> 4;  // full granules
    uint32_t s = 0;
    uint64_t j = lane;
    // four granules in flight per lane
    for (; j + 3 * kWave < G; j += 4 * kWave) {
      const uint4 g0 = granule(p, sh, uint32_t(j)), g1 = granule(p, sh, uint32_t(j + kWave)),
                  g2 = granule(p, sh, uint32_t(j + 2 * kWave)), g3 = granule(p, sh, uint32_t(j + 3 * kWave));
      s = crc16(L, j == lane ? s : crc_gap(L, s), g0);
      s = crc16(L, crc_gap(L, s), g1);
      s = crc16(L, crc_gap(L, s), g2);
      s = crc16(L, crc_gap(L, s), g3);
    }
    for (; j < G; j += kWave) {
      const uint4 g = granule(p, sh, uint32_t(j));
      s = crc16(L, j == lane ? s : crc_gap(L, s), g);
    }
    // shift to the end of the full granules (16*G): the lane's last ends at 16*(jl+1)
    if (uint64_t(lane) < G) {
      const uint64_t jl = lane + ((G - 1 - lane) / kWave) * kWave;
      const uint64_t after = 16 * (G - jl - 1);
      if (after) s = multmodp(x8nmodp(L, after), s);
    }
#pragma unroll
    for (int d = kWave / 2; d >= 1; d >>= 1) s ^= __shfl_xor(s, d, kWave);
    if (lane == 0) {
      uint32_t t = s;
      for (uint64_t i = 16 * G; i < n; i++) t = L.t[0][(t ^ p[i]) & 0xff] ^ (t >> 8);  // the tail, raw
      const uint32_t c = ~(t ^ multmodp(x8nmodp(L, n), ~0u));
      const uint32_t v = ((c >> 15) | (c << 17)) + 0xa282ead8u;  // crc.CRC.Value()
      const gptr<const uint8_t> tr = p + n;
      const uint32_t want = uint32_t(tr[0]) | uint32_t(tr[1]) << 8 | uint32_t(tr[2]) << 16 | uint32_t(tr[3]) << 24;
      status[b] = v == want ? PBL_OK : PBL_CORRUPT_CHECKSUM;
      if (computed) computed[b] = v;
    }
  }
}

// ---- XXH64 (the XXH64 specification; cespare/xxhash/v2 implements it) ---------
constexpr uint64_t P1 = 11400714785074694791ull, P2 = 14029467366897019727ull, P3 = 1609587929392839161ull,
                   P4 = 9650029242287828579ull, P5 = 2870177450012600261ull;
__device__ inline uint64_t rotl(uint64_t x, int r) { return (x << r) | (x >> (64 - r)); }
__device__ inline uint64_t xround(uint64_t acc, uint64_t in) { return rotl(acc + in * P2, 31) * P1; }
__device__ inline uint64_t xmerge(uint64_t acc, uint64_t v) { return (acc ^ xround(0, v)) * P1 + P4; }
__device__ inline uint64_t ld64(gptr<const uint8_t> p) {
  uint64_t v = 0;
  for (int i = 7; i >= 0; i--) v = v << 8 | p[i];
  return v;
}

__device__ inline uint64_t xxh64(gptr<const uint8_t> p, uint64_t n) {
  uint64_t h, i = 0;
  if (n >= 32) {
    uint64_t v1 = P1 + P2, v2 = P2, v3 = 0, v4 = 0ull - P1;
    for (; i + 32 <= n; i += 32) {
      v1 = xround(v1, ld64(p + i));
      v2 = xround(v2, ld64(p + i + 8));
      v3 = xround(v3, ld64(p + i + 16));
      v4 = xround(v4, ld64(p + i + 24));
    }
    h = rotl(v1, 1) + rotl(v2, 7) + rotl(v3, 12) + rotl(v4, 18);
    h = xmerge(h, v1);
    h = xmerge(h, v2);
    h = xmerge(h, v3);
    h = xmerge(h, v4);
  } else {
    h = P5;
  }
  h += n;
  for (; i + 8 <= n; i += 8) h = rotl(h ^ xround(0, ld64(p + i)), 27) * P1 + P4;
  if (i + 4 <= n) {
    const uint64_t w = uint64_t(p[i]) | uint64_t(p[i + 1]) << 8 | uint64_t(p[i + 2]) << 16 | uint64_t(p[i + 3]) << 24;
    h = rotl(h ^ (w * P1), 23) * P2 + P3;
    i += 4;
  }
  for (; i < n; i++) h = rotl(h ^ (uint64_t(p[i]) * P5), 11) * P1;
  h ^= h >> 33;
  h *= P2;
  h ^= h >> 29;
  h *= P3;
  h ^= h >> 32;
  return h;
}

__global__ void __launch_bounds__(kTPB) checksum_xxh_kernel(const pbl_phys_batch B, uint32_t* status,
                                                            uint32_t* computed) {
  for (uint32_t b = blockIdx.x * kTPB + threadIdx.x; b < B.n_blocks; b += gridDim.x * kTPB) {
    const uint64_t n = uint64_t(B.block_len[b]) + 1;
    const gptr<const uint8_t> p = to_glb(B.bytes + B.block_off[b]);
    const uint32_t v = uint32_t(xxh64(p, n));
    const gptr<const uint8_t> t = p + n;
    const uint32_t want = uint32_t(t[0]) | uint32_t(t[1]) << 8 | uint32_t(t[2]) << 16 | uint32_t(t[3]) << 24;
    status[b] = v == want ? PBL_OK : PBL_CORRUPT_CHECKSUM;
    if (computed) computed[b] = v;
  }
}

// ---- snappy ---------------------------------------------------------------------
constexpr uint32_t kSnapCap = 32768;  // staged compressed bytes / decoded bytes per block (LDS)

__device__ inline bool uvarint32(gptr<const uint8_t> p, uint64_t n, uint32_t* v, uint32_t* used) {
  uint64_t x = 0;
  for (uint32_t i = 0; i < n && i < 10; i++) {
    x |= uint64_t(p[i] & 0x7f) << (7 * i);
    if (p[i] < 0x80) {
      if (x > 0xffffffffull) return false;
      *v = uint32_t(x);
      *used = i + 1;
      return true;
    }
  }
  return false;
}

// ---- MinLZ (minlz_dec.hip.h decodes the MinLZ form) ------------------------------
constexpr uint32_t kMinlzMaxBlock = 8u << 20;  // minlz.MaxBlockSize

// The MinLZ form's header (src[0] == 0): decoded length, header bytes, stored.
// False on a corrupt header (minlz.DecodedLen's errors).
__device__ inline bool minlz_header(gptr<const uint8_t> p, uint32_t n, uint32_t* dlen, uint32_t* hdr, bool* stored) {
  *stored = false;
  if (n == 1) {  // the empty block
    *dlen = 0;
    *hdr = 1;
    return true;
  }
  uint32_t v = 0, u = 0;
  if (!uvarint32(p + 1, n - 1, &v, &u) || v > kMinlzMaxBlock) return false;
  const uint32_t rest = n - 1 - u;
  if (rest == 0) return false;
  *hdr = 1 + u;
  if (v == 0) {
    *stored = true;
    *dlen = rest;
    return true;
  }
  if (v < rest) return false;  // a compressed block is never longer than its output
  *dlen = v;
  return true;
}

// Whether a block with indicator `ind` is decoded by the snappy kernels:
// snappy blocks, and MinLZ-indicated blocks in the Snappy form.
__device__ __forceinline__ bool snappy_form(uint32_t ind, gptr<const uint8_t> p, uint32_t n) {
  return ind == PBL_COMPRESSION_SNAPPY || (ind == PBL_COMPRESSION_MINLZ && n > 0 && p[0] != 0);
}

__global__ void __launch_bounds__(kTPB) snappy_len_kernel(const pbl_phys_batch B, uint32_t* out_len, uint32_t* status) {
  for (uint32_t b = blockIdx.x * kTPB + threadIdx.x; b < B.n_blocks; b += gridDim.x * kTPB) {
    const uint32_t n = B.block_len[b];
    const gptr<const uint8_t> p = to_glb(B.bytes + B.block_off[b]);
    const uint32_t ind = p[n];
    uint32_t st = PBL_OK, len = 0, used = 0;
    bool stored = false;
    if (ind == PBL_COMPRESSION_NONE) len = n;
    else if (snappy_form(ind, p, n) || ind == PBL_COMPRESSION_ZSTD)  // (zstd_cgo.go:111-119)
      st = uvarint32(p, n, &len, &used) ? PBL_OK : PBL_CORRUPT_COMPRESSION;
    else if (ind == PBL_COMPRESSION_MINLZ)  // minlz.DecodedLen
      st = n > 0 && minlz_header(p, n, &len, &used, &stored) ? PBL_OK : PBL_CORRUPT_COMPRESSION;
    else st = PBL_UNSUPPORTED;
    out_len[b] = st == PBL_OK ? len : 0u;
    status[b] = st;
  }
}

// Staged block bytes sit at their global 16-B phase (byte j of the block at
// src[(block address & 15) + j]) so the staging loads and the output stores
// are aligned 16-B accesses; 32 bytes of slack cover the phase and the 16-B
// literal copies that run past an element's end.
// LDS staging of one block for the one-wave decoders (minlz_kernel): the
// compressed bytes and the decoded bytes, each at its global 16-B phase.
struct SnapLds {
  uint4 src4[(kSnapCap + 32) / 16];
  uint4 dst4[(kSnapCap + 32) / 16];
};

typedef uint32_t su32x4_u __attribute__((ext_vector_type(4), aligned(1)));
struct LdsBytes {
  lptr<uint8_t> p;
  static constexpr bool kVec = true;
  __device__ uint8_t operator[](uint32_t i) const { return p[i]; }
  __device__ su32x4_u get16(uint32_t i) const { return *(lptr<const su32x4_u>)(p + i); }
};
struct LdsBytesW {
  lptr<uint8_t> p;
  __device__ uint8_t get(uint32_t i) const { return p[i]; }
  __device__ void set(uint32_t i, uint8_t v) const { p[i] = v; }
  __device__ su32x4_u get16(uint32_t i) const { return *(lptr<const su32x4_u>)(p + i); }
  __device__ void set16(uint32_t i, su32x4_u v) const { *(lptr<su32x4_u>)(p + i) = v; }
};
struct GlbBytes {
  gptr<const uint8_t> p;
  static constexpr bool kVec = false;
  __device__ uint8_t operator[](uint32_t i) const { return p[i]; }
  __device__ su32x4_u get16(uint32_t) const { return su32x4_u{0, 0, 0, 0}; }
};
struct GlbBytesW {
  gptr<uint8_t> p;
  __device__ uint8_t get(uint32_t i) const { return p[i]; }
  __device__ void set(uint32_t i, uint8_t v) const { p[i] = v; }
};

#include "minlz_dec.hip.h"

// Decode one snappy block.  Lane 0 reads element headers; the wave copies.
// Returns the decoded length, or ~0u when the input is corrupt.
// (lane, step): the wave's lanes (lane_id(), 64) or one lane alone (0, 1).
template <class Src, class Dst>
__device__ inline uint32_t snappy_wave(Src src, uint32_t n, Dst dst, uint32_t cap, uint32_t lane, uint32_t step) {
  uint32_t dlen = 0, s = 0;
  bool ok = true;
  {  // uvarint decoded length
    uint64_t x = 0;
    bool done = false;
    for (uint32_t i = 0; i < n && i < 10 && !done; i++) {
      x |= uint64_t(src[i] & 0x7f) << (7 * i);
      if (src[i] < 0x80) {
        done = true;
        s = i + 1;
      }
    }
    ok = done && x <= cap;
    dlen = uint32_t(x);
  }
  uint32_t d = 0;
  while (ok && s < n) {
    // element header (every lane reads the same bytes: uniform control flow)
    const uint32_t t = src[s];
    uint32_t kind = t & 3, len = 0, off = 0, lit = 0;
    if (kind == 0) {
      uint32_t x = t >> 2;
      if (x < 60) {
        s += 1;
      } else {
        const uint32_t nb = x - 59;
        if (s + 1 + nb > n) { ok = false; break; }
        x = 0;
        for (uint32_t i = 0; i < nb; i++) x |= uint32_t(src[s + 1 + i]) << (8 * i);
        s += 1 + nb;
      }
      len = x + 1;
      if (len > n - s || len > dlen - d) { ok = false; break; }
      lit = s;
      s += len;
    } else if (kind == 1) {
      if (s + 2 > n) { ok = false; break; }
      len = 4 + ((t >> 2) & 7);
      off = ((t & 0xe0) << 3) | src[s + 1];
      s += 2;
    } else if (kind == 2) {
      if (s + 3 > n) { ok = false; break; }
      len = 1 + (t >> 2);
      off = uint32_t(src[s + 1]) | uint32_t(src[s + 2]) << 8;
      s += 3;
    } else {
      if (s + 5 > n) { ok = false; break; }
      len = 1 + (t >> 2);
      off = uint32_t(src[s + 1]) | uint32_t(src[s + 2]) << 8 | uint32_t(src[s + 3]) << 16 | uint32_t(src[s + 4]) << 24;
      s += 5;
    }
    if (kind != 0 && (off == 0 || off > d || len > dlen - d)) { ok = false; break; }
    if constexpr (Src::kVec) {
      // LDS -> LDS (the wave): 16 bytes per lane per step.  A chunk may write
      // up to 15 bytes past the element's end: later elements rewrite them, and
      // copies read only below d.  A copy whose offset is at least one step's
      // span (64 x 16 B) never reads what the same step writes.
      if (kind == 0) {
        for (uint32_t i = 16 * lane; i < len; i += 16 * step) dst.set16(d + i, src.get16(lit + i));
      } else if (off >= 16 * kWave) {
        for (uint32_t i = 16 * lane; i < len; i += 16 * step) dst.set16(d + i, dst.get16(d - off + i));
      } else {
        for (uint32_t i = lane; i < len; i += step) dst.set(d + i, dst.get(d - off + (i % off)));
      }
    } else {
      if (kind == 0) {
        for (uint32_t i = lane; i < len; i += step) dst.set(d + i, src[lit + i]);
      } else {
        for (uint32_t i = lane; i < len; i += step) dst.set(d + i, dst.get(d - off + (i % off)));
      }
    }
    wave_sync();
    d += len;
  }
  return ok && d == dlen ? d : ~0u;
}

// ---- snappy: snappy2_kernel (also the path for blocks the walk does not cover) ----
// One wave per block, four blocks per CU (38 KB of LDS each: the compressed
// bytes and a queue of element descriptors; the output goes straight to HBM):
//   parse     lane 0 walks the element tags from LDS (8 bytes per element in
//             one LDS round trip) and queues up to kSnQ descriptors {kind,
//             length, literal source / copy offset, output offset}
//   literals  lane per queued literal, 16-B chunks LDS -> global (literals
//             longer than 256 B by the whole wave)
//   copies    in groups: the pending copies whose source bytes below their
//             own output all lie below the group's first output offset are
//             independent (their sources are final), one lane each; a copy
//             with offset < 16 writes its period (byte i = src[i % off], read
//             once), others 16-B chunks.  A workgroup fence between groups.
// Blocks past the LDS stage (or decoding past 64 KiB) take snappy_wave on one
// lane from global memory.
constexpr uint32_t kSnIn = 32768;
constexpr uint32_t kSnQ = 592;  // (4 blocks per CU: 40 KB of LDS each)
#ifdef PBL_SNAP_STAMPS  // diagnostic builds: per-block phase cycles (scripts/snap_stamps.py)
__device__ uint64_t g_snap_stamps[65536 * 8];
#define SN_T(v) const uint64_t v = __builtin_amdgcn_s_memtime()
#define SN_ACC(i, v) if (lane_id() == 0 && g_sn_b < 65536) g_snap_stamps[8 * g_sn_b + (i)] += __builtin_amdgcn_s_memtime() - (v)
__device__ uint32_t g_sn_dummy;
#else
#define SN_T(v)
#define SN_ACC(i, v)
#endif
#include "snappy_dec.hip.h"

// The element walk of the blocks snappy4_kernel decodes, a lane per block.
__global__ void __launch_bounds__(kTPB) snappy_walk_kernel(const pbl_phys_batch B, uint8_t* out,
                                                           const uint64_t* out_off, const uint32_t* out_cap) {
  const uint32_t b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B.n_blocks) return;
  const uint32_t n = to_glb(B.block_len)[b];
  const gptr<const uint8_t> src = to_glb(B.bytes + to_glb(B.block_off)[b]);
  if (!snappy_form(src[n], src, n)) return;
  uint32_t dl = 0, used = 0;
  if (!uvarint32(src, n, &dl, &used) || dl > to_glb(out_cap)[b] || !sn4_walkable(n, dl)) return;
  sn4_walk(src, n, used, dl, to_glb(out + to_glb(out_off)[b]));
}

// A wave per walked block (sn4_decode); snappy2_kernel takes the others.
__global__ void __launch_bounds__(kWave) snappy4_kernel(const pbl_phys_batch B, uint8_t* out, const uint64_t* out_off,
                                                        const uint32_t* out_cap, uint32_t* out_len, uint32_t* status) {
  __shared__ Snap4Lds S;
  for (uint32_t b = blockIdx.x; b < B.n_blocks; b += gridDim.x) {
    const uint32_t n = to_glb(B.block_len)[b];
    const gptr<const uint8_t> src = to_glb(B.bytes + to_glb(B.block_off)[b]);
    if (!snappy_form(src[n], src, n)) continue;
    uint32_t dl = 0, used = 0;
    if (!uvarint32(src, n, &dl, &used) || dl > to_glb(out_cap)[b] || !sn4_walkable(n, dl)) continue;
    const bool ok = sn4_decode(S, src, n, dl, to_glb(out + to_glb(out_off)[b]), b);
    if (lane_id() == 0) {
      to_glb(out_len)[b] = ok ? dl : 0u;
      to_glb(status)[b] = ok ? uint32_t(PBL_OK) : uint32_t(PBL_CORRUPT_COMPRESSION);
    }
    wave_sync();
  }
}

__global__ void __launch_bounds__(kWave) snappy2_kernel(const pbl_phys_batch B, uint8_t* out, const uint64_t* out_off,
                                                        const uint32_t* out_cap, uint32_t* out_len, uint32_t* status) {
  __shared__ Snap2Lds S;
  const uint32_t lane = lane_id();
  for (uint32_t b = blockIdx.x; b < B.n_blocks; b += gridDim.x) {
    const uint32_t n = to_glb(B.block_len)[b];
    const uint64_t boff = to_glb(B.block_off)[b];
    const gptr<const uint8_t> src = to_glb(B.bytes + boff);
    const uint32_t ind = src[n];
    if (ind == PBL_COMPRESSION_ZSTD) continue;  // zstd_kernel's
    if (ind == PBL_COMPRESSION_MINLZ && !snappy_form(ind, src, n)) continue;  // minlz_kernel's
    gptr<uint8_t> dst = to_glb(out + to_glb(out_off)[b]);
    const uint32_t cap = to_glb(out_cap)[b];
    uint32_t st = PBL_OK, len = 0;
    if (ind == PBL_COMPRESSION_NONE) {
      if (n > cap) {
        st = PBL_OVERFLOW;
      } else {
        // 16-B chunks, the tail byte-wise (nothing read past the block)
        const uint32_t nf = n & ~15u;
        for (uint32_t c = 16 * lane; c < nf; c += 16 * kWave)
          *(gptr<sn_u32x4_u>)(dst + c) = *(gptr<const sn_u32x4_u>)(src + c);
        for (uint32_t c = nf + lane; c < n; c += kWave) dst[c] = src[c];
      }
      len = n;
    } else if (snappy_form(ind, src, n)) {
      uint32_t dl = 0, used = 0;
      if (!uvarint32(src, n, &dl, &used)) st = PBL_CORRUPT_COMPRESSION;
      else if (dl > cap) st = PBL_OVERFLOW;
      else if (sn4_walkable(n, dl)) continue;  // snappy4_kernel's
      else if (n <= kSnIn && dl <= 0xffffu) {
        const uint64_t sa = reinterpret_cast<uint64_t>(B.bytes + boff);
        const uint32_t ssh = uint32_t(sa & 15), ng = (ssh + n + 15) / 16;
        const gptr<const u32x4> sg = to_glb(reinterpret_cast<const u32x4*>(sa - ssh));
        SN_T(ts);
        lds_stage16(to_lds_ptr(reinterpret_cast<u32x4*>(S.in)), sg, ng);
        {
          const uint32_t g_sn_b = b;
          SN_ACC(0, ts);
          (void)g_sn_b;
        }
        len = dl;
        if (!sn_decode(S, ssh, n, used, dl, dst, b)) st = PBL_CORRUPT_COMPRESSION;
      } else {
        len = ~0u;
        if (lane == 0) len = snappy_wave(GlbBytes{src}, n, GlbBytesW{dst}, dl, 0, 1);
        len = __shfl(len, 0, kWave);
        if (len == ~0u) st = PBL_CORRUPT_COMPRESSION;
      }
    } else {
      st = PBL_UNSUPPORTED;
    }
    if (lane == 0) {
      to_glb(out_len)[b] = st == PBL_OK ? len : 0u;
      to_glb(status)[b] = st;
    }
    wave_sync();
  }
}

}  // namespace phys
}  // namespace pbl

extern "C" {

#ifdef PBL_SNAP_STAMPS
int pbl_diag_snap_stamps(uint64_t* host, uint64_t n, int clear) {
  if (clear) {
    static uint64_t zero[65536 * 8];
    return hipMemcpyToSymbol(HIP_SYMBOL(pbl::phys::g_snap_stamps), zero, sizeof(zero)) == hipSuccess ? 0 : 8;
  }
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(pbl::phys::g_snap_stamps), n * 8) == hipSuccess ? 0 : 8;
}
#endif

int pbl_verify_checksums(const pbl_phys_batch* batch, uint32_t checksum_type, uint32_t* status, uint32_t* computed,
                         void* stream) {
  if (!batch || !status) return PBL_INVALID_ARG;
  if (batch->n_blocks == 0) return PBL_OK;
  if (!batch->bytes || !batch->block_off || !batch->block_len) return PBL_INVALID_ARG;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const uint32_t n = batch->n_blocks;
  if (checksum_type == PBL_CHECKSUM_CRC32C) {
    const uint32_t wpb = pbl::kTPB / pbl::kWave;
    const uint32_t grid = uint32_t(std::min<uint64_t>((n + wpb - 1) / wpb, 4096));
    hipLaunchKernelGGL(pbl::phys::checksum_crc_kernel, dim3(grid), dim3(pbl::kTPB), 0, st, *batch, status, computed);
  } else if (checksum_type == PBL_CHECKSUM_XXHASH64) {
    const uint32_t grid = uint32_t(std::min<uint64_t>((n + pbl::kTPB - 1) / pbl::kTPB, 4096));
    hipLaunchKernelGGL(pbl::phys::checksum_xxh_kernel, dim3(grid), dim3(pbl::kTPB), 0, st, *batch, status, computed);
  } else {
    return PBL_UNSUPPORTED;  // ChecksumTypeNone has nothing to validate; ChecksumTypeXXHash is unsupported (block.go:161)
  }
  return hipGetLastError() == hipSuccess ? PBL_OK : PBL_DEVICE_ERROR;
}

int pbl_decompressed_lengths(const pbl_phys_batch* batch, uint32_t* out_len, uint32_t* status, void* stream) {
  if (!batch || !out_len || !status) return PBL_INVALID_ARG;
  if (batch->n_blocks == 0) return PBL_OK;
  if (!batch->bytes || !batch->block_off || !batch->block_len) return PBL_INVALID_ARG;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const uint32_t grid = uint32_t(std::min<uint64_t>((batch->n_blocks + pbl::kTPB - 1) / pbl::kTPB, 4096));
  hipLaunchKernelGGL(pbl::phys::snappy_len_kernel, dim3(grid), dim3(pbl::kTPB), 0, st, *batch, out_len, status);
  return hipGetLastError() == hipSuccess ? PBL_OK : PBL_DEVICE_ERROR;
}

int pbl_decompress_blocks(const pbl_phys_batch* batch, uint8_t* out, const uint64_t* out_off, const uint32_t* out_cap,
                          uint32_t* out_len, uint32_t* status, void* stream) {
  if (!batch || !out || !out_off || !out_cap || !out_len || !status) return PBL_INVALID_ARG;
  if (batch->n_blocks == 0) return PBL_OK;
  if (!batch->bytes || !batch->block_off || !batch->block_len) return PBL_INVALID_ARG;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  hipLaunchKernelGGL(pbl::phys::snappy_walk_kernel, dim3((batch->n_blocks + pbl::kTPB - 1) / pbl::kTPB),
                     dim3(pbl::kTPB), 0, st, *batch, out, out_off, out_cap);
  hipLaunchKernelGGL(pbl::phys::snappy4_kernel, dim3(std::min<uint32_t>(batch->n_blocks, 8192)), dim3(pbl::kWave), 0,
                     st, *batch, out, out_off, out_cap, out_len, status);
  const uint32_t grid = std::min<uint32_t>(batch->n_blocks, 4096);
  hipLaunchKernelGGL(pbl::phys::snappy2_kernel, dim3(grid), dim3(pbl::kWave), 0, st, *batch, out, out_off, out_cap,
                     out_len, status);
  hipLaunchKernelGGL(pbl::phys::minlz_kernel, dim3(std::min<uint32_t>(batch->n_blocks, 2048)), dim3(pbl::kWave), 0, st,
                     *batch, out, out_off, out_cap, out_len, status);
  if (hipGetLastError() != hipSuccess) return PBL_DEVICE_ERROR;
  return pbl::launch_zstd(*batch, out, out_off, out_cap, out_len, status, st) == hipSuccess ? PBL_OK
                                                                                              : PBL_DEVICE_ERROR;
}

}  // extern "C"
