// sstable.hip — from whole tables to batches of blocks:
//
//   pbl_parse_footer       parseFooter (sstable/table.go:328-404), host code:
//                          LevelDB / RocksDBv2 / Pebblev1-v8 footers, the
//                          Pebblev6+ footer checksum, Pebblev7+ attributes
//   pbl_index_handles_row  rowblk.IndexIter.BlockHandleWithProperties over a
//                          decoded batch of row index blocks: one wave per block,
//                          lane per entry, block.DecodeHandleWithProperties
//                          (block/block.go:80-104) of each value
//   pbl_index_handles_col  colblk.IndexBlockDecoder.Init + IndexIter over raw
//                          columnar index blocks: size kernel (wave per block:
//                          column checks, rows), one-workgroup scan, write kernel
//                          (thread per row: offsets.At, lengths.At, blockProps.At)
//   pbl_kv_blocks          colblk.KeyValueBlockDecoder (metaindex, properties)
//   pbl_valblk_index       valblk.DecodeIndex: the value-block handles
//   pbl_resolve_values     valueBlockFetcher.Fetch for every value-block handle
//                          of a decoded batch (size / scan / copy)
//
// The handles of a table's index are its data blocks: with the file's bytes in
// HBM they become a pbl_phys_batch (checksums, decompression) and then a
// pbl_block_batch for pbl_decode_batch, without the host reading the index.
#include <cstring>

#include "common.hip.h"
#include "colblk_block.hip.h"

namespace pbl {
namespace sst {
using namespace col;

// Go binary.Uvarint over [o, end): bytes used (> 0), 0 when the input ends
// first, -1 on a 64-bit overflow (a 10th byte > 1, or more than 10 bytes).
__device__ inline int uvarint64(gptr<const uint8_t> p, uint64_t o, uint64_t end, uint64_t* v) {
  uint64_t x = 0;
  uint32_t s = 0;
  for (int i = 0; i < 10; i++) {
    if (o + i >= end) return 0;
    const uint32_t b = p[o + i];
    if (b < 0x80) {
      if (i == 9 && b > 1) return -1;
      *v = x | uint64_t(b) << s;
      return i + 1;
    }
    x |= uint64_t(b & 0x7f) << s;
    s += 7;
  }
  return -1;
}

__global__ void __launch_bounds__(kTPB) index_row_kernel(pbl_decode_out D, uint32_t nb, pbl_index_out O) {
  const uint32_t wpb = kTPB / kWave;
  for (uint32_t b = blockIdx.x * wpb + wave_id(); b < nb; b += gridDim.x * wpb) {
    const uint64_t k0 = to_glb(D.blk_kv_base)[b], k1 = to_glb(D.blk_kv_base)[b + 1];
    const uint64_t vb = to_glb(D.blk_val_base)[b];
    uint32_t st = to_glb(D.blk_status)[b];
    const gptr<const uint8_t> vals = to_glb(static_cast<const uint8_t*>(D.val_bytes));
    bool bad = false;
    if (st == PBL_OK) {
      for (uint64_t k = k0 + lane_id(); k < k1; k += kWave) {
        const uint64_t j = k - k0;
        const uint64_t v0 = vb + to_glb(D.val_off)[k0 + b + j], v1 = vb + to_glb(D.val_off)[k0 + b + j + 1];
        uint64_t off = 0, len = 0;
        const int n = uvarint64(vals, v0, v1, &off);
        const int m = n > 0 ? uvarint64(vals, v0 + n, v1, &len) : 0;
        if (n <= 0 || m <= 0) {
          bad = true;
          continue;
        }
        if (k < O.cap) {
          to_glb(O.handle_off)[k] = off;
          to_glb(O.handle_len)[k] = len;
          if (O.props_off) to_glb(O.props_off)[k] = v0 + n + m;
          if (O.props_len) to_glb(O.props_len)[k] = uint32_t(v1 - (v0 + n + m));
        }
      }
      if (__ballot(bad)) st = PBL_CORRUPT_INDEX;
      else if (k1 > O.cap) st = PBL_OVERFLOW;
    }
    if (lane_id() == 0) {
      to_glb(O.blk_status)[b] = st;
      to_glb(O.blk_base)[b] = k0;
      if (b + 1 == nb) to_glb(O.blk_base)[nb] = k1;
    }
  }
}

// Column layout of a colblk index block (custom header size 0).
struct IdxDesc {
  uint32_t rows;
  UCol sep_off, offs, lens, prop_off;
  uint32_t sep_data, prop_data;
};

__device__ inline uint32_t index_desc(const Src& S, IdxDesc* D) {
  Dir dir;
  dir.custom = 0;
  if (S.len < 7) return PBL_CORRUPT_COLBLK_HEADER;
  dir.ncols = uint32_t(S.le_u(1, 2));
  D->rows = uint32_t(S.le_u(3, 4));
  const uint32_t rows = D->rows;
  uint64_t s, nx, e;
  if (!dir.column(S, 0, kDtBytes, &s, &nx) || !dec_rawbytes(S, s, rows, &D->sep_off, &D->sep_data, &e) || e != nx)
    return PBL_CORRUPT_COLBLK_HEADER;
  if (!dir.column(S, 1, kDtUint, &s, &nx) || !dec_uints(S, s, rows, &D->offs, &e) || e != nx)
    return PBL_CORRUPT_COLBLK_HEADER;
  if (!dir.column(S, 2, kDtUint, &s, &nx) || !dec_uints(S, s, rows, &D->lens, &e) || e != nx)
    return PBL_CORRUPT_COLBLK_HEADER;
  if (!dir.column(S, 3, kDtBytes, &s, &nx) || !dec_rawbytes(S, s, rows, &D->prop_off, &D->prop_data, &e) ||
      e != nx)
    return PBL_CORRUPT_COLBLK_HEADER;
  return PBL_OK;
}

__device__ inline Src glb_src(const uint8_t* blk, uint32_t len, lds_cu8 dummy) {
  return Src{dummy, dummy, (glb_cu8)blk, 0u, len, len};
}

// Pass 1: each index block's entry count into blk_base[b] (status alongside).
__global__ void __launch_bounds__(kTPB) index_col_size_kernel(pbl_block_batch B, pbl_index_out O) {
  __shared__ uint8_t dummy[16];
  for (uint32_t b = blockIdx.x * kTPB + threadIdx.x; b < B.n_blocks; b += gridDim.x * kTPB) {
    IdxDesc D;
    const Src S = glb_src(B.blocks + to_glb(B.block_off)[b], to_glb(B.block_len)[b], (lds_cu8)to_lds(dummy));
    const uint32_t st = index_desc(S, &D);
    to_glb(O.blk_status)[b] = st;
    to_glb(O.blk_base)[b] = st == PBL_OK ? D.rows : 0u;
  }
}

// Pass 2 (one workgroup): blk_base becomes the exclusive prefix; blocks past
// cap become PBL_OVERFLOW (sizes kept, entries not written).
__global__ void __launch_bounds__(1024) index_col_scan_kernel(uint32_t nb, pbl_index_out O) {
  __shared__ uint64_t part[1024];
  __shared__ uint64_t carry;
  if (threadIdx.x == 0) carry = 0;
  __syncthreads();
  for (uint32_t c0 = 0; c0 < nb; c0 += 1024) {
    const uint32_t i = c0 + threadIdx.x;
    const uint64_t v = i < nb ? to_glb(O.blk_base)[i] : 0;
    part[threadIdx.x] = v;
    __syncthreads();
    for (uint32_t d = 1; d < 1024; d <<= 1) {
      const uint64_t x = threadIdx.x >= d ? part[threadIdx.x - d] : 0;
      __syncthreads();
      part[threadIdx.x] += x;
      __syncthreads();
    }
    const uint64_t excl = carry + part[threadIdx.x] - v;
    if (i < nb) {
      to_glb(O.blk_base)[i] = excl;
      if (excl + v > O.cap && to_glb(O.blk_status)[i] == PBL_OK) to_glb(O.blk_status)[i] = PBL_OVERFLOW;
    }
    __syncthreads();
    if (threadIdx.x == 1023) carry += part[1023];
    __syncthreads();
  }
  if (threadIdx.x == 0) to_glb(O.blk_base)[nb] = carry;
}

// Pass 3: one workgroup per index block, thread per row.
__global__ void __launch_bounds__(kTPB) index_col_write_kernel(pbl_block_batch B, pbl_index_out O) {
  __shared__ uint8_t dummy[16];
  for (uint32_t b = blockIdx.x; b < B.n_blocks; b += gridDim.x) {
    if (to_glb(O.blk_status)[b] != PBL_OK) continue;
    const uint64_t boff = to_glb(B.block_off)[b];
    const Src S = glb_src(B.blocks + boff, to_glb(B.block_len)[b], (lds_cu8)to_lds(dummy));
    IdxDesc D;
    (void)index_desc(S, &D);
    const uint64_t base = to_glb(O.blk_base)[b];
    for (uint32_t r = threadIdx.x; r < D.rows; r += kTPB) {
      to_glb(O.handle_off)[base + r] = u_at<false>(S, D.offs, r);
      to_glb(O.handle_len)[base + r] = u_at<false>(S, D.lens, r);
      const UCol& po = D.prop_off;
      const uint64_t p0 = po.w ? S.le(po.at + r * po.w, po.w) : 0, p1 = po.w ? S.le(po.at + (r + 1) * po.w, po.w) : 0;
      if (O.props_off) to_glb(O.props_off)[base + r] = boff + D.prop_data + p0;
      if (O.props_len) to_glb(O.props_len)[base + r] = uint32_t(p1 - p0);
    }
  }
}

// ---- colblk.KeyValueBlockDecoder (metaindex / properties of Pebblev6+ / v7+) ----
// key_value_block.go:76-89: no custom header; column 0 the keys and column 1 the
// values, both RawBytes.  Entries point into the batch's block bytes (KeyAt /
// ValueAt are zero-copy slices there too).
struct KvDesc {
  uint32_t rows;
  UCol koff, voff;
  uint32_t kdata, vdata;
};

__device__ inline uint32_t kv_desc(const Src& S, KvDesc* D) {
  Dir dir;
  dir.custom = 0;
  if (S.len < 7) return PBL_CORRUPT_COLBLK_HEADER;
  dir.ncols = uint32_t(S.le_u(1, 2));
  D->rows = uint32_t(S.le_u(3, 4));
  uint64_t s, nx, e;
  if (!dir.column(S, 0, kDtBytes, &s, &nx) || !dec_rawbytes(S, s, D->rows, &D->koff, &D->kdata, &e) || e != nx)
    return PBL_CORRUPT_COLBLK_HEADER;
  if (!dir.column(S, 1, kDtBytes, &s, &nx) || !dec_rawbytes(S, s, D->rows, &D->voff, &D->vdata, &e) || e != nx)
    return PBL_CORRUPT_COLBLK_HEADER;
  return PBL_OK;
}

__device__ inline bool kv_slice(const Src& S, const UCol& o, uint32_t data, uint32_t r, uint64_t* at, uint32_t* n) {
  const uint64_t p0 = o.w ? S.le(o.at + r * o.w, o.w) : 0, p1 = o.w ? S.le(o.at + (r + 1) * o.w, o.w) : 0;
  if (p1 < p0 || data + p1 > S.len) return false;  // (Go would slice past the column: corrupt)
  *at = data + p0;
  *n = uint32_t(p1 - p0);
  return true;
}

// Pass 1: each block's row count into blk_base[b] (status alongside), every
// row's slices checked.
__global__ void __launch_bounds__(kTPB) kv_size_kernel(pbl_block_batch B, pbl_kv_out O) {
  __shared__ uint8_t dummy[16];
  const uint32_t wpb = kTPB / kWave;
  for (uint32_t b = blockIdx.x * wpb + wave_id(); b < B.n_blocks; b += gridDim.x * wpb) {
    KvDesc D;
    const Src S = glb_src(B.blocks + to_glb(B.block_off)[b], to_glb(B.block_len)[b], (lds_cu8)to_lds(dummy));
    uint32_t st = kv_desc(S, &D);
    bool bad = false;
    if (st == PBL_OK)
      for (uint32_t r = lane_id(); r < D.rows; r += kWave) {
        uint64_t a;
        uint32_t n;
        bad |= !kv_slice(S, D.koff, D.kdata, r, &a, &n) || !kv_slice(S, D.voff, D.vdata, r, &a, &n);
      }
    if (__ballot(bad)) st = PBL_CORRUPT_BOUNDS;
    if (lane_id() == 0) {
      to_glb(O.blk_status)[b] = st;
      to_glb(O.blk_base)[b] = st == PBL_OK ? D.rows : 0u;
    }
  }
}

// Pass 2 (one workgroup): exclusive prefix of blk_base; blocks past cap become
// PBL_OVERFLOW (sizes kept, entries not written).
__global__ void __launch_bounds__(1024) kv_scan_kernel(uint32_t nb, uint64_t* blk_base, uint32_t* blk_status,
                                                       uint64_t cap) {
  __shared__ uint64_t part[1024];
  __shared__ uint64_t carry;
  if (threadIdx.x == 0) carry = 0;
  __syncthreads();
  for (uint32_t c0 = 0; c0 < nb; c0 += 1024) {
    const uint32_t i = c0 + threadIdx.x;
    const uint64_t v = i < nb ? to_glb(blk_base)[i] : 0;
    part[threadIdx.x] = v;
    __syncthreads();
    for (uint32_t d = 1; d < 1024; d <<= 1) {
      const uint64_t x = threadIdx.x >= d ? part[threadIdx.x - d] : 0;
      __syncthreads();
      part[threadIdx.x] += x;
      __syncthreads();
    }
    const uint64_t excl = carry + part[threadIdx.x] - v;
    if (i < nb) {
      to_glb(blk_base)[i] = excl;
      if (excl + v > cap && to_glb(blk_status)[i] == PBL_OK) to_glb(blk_status)[i] = PBL_OVERFLOW;
    }
    __syncthreads();
    if (threadIdx.x == 1023) carry += part[1023];
    __syncthreads();
  }
  if (threadIdx.x == 0) to_glb(blk_base)[nb] = carry;
}

// Pass 3: one workgroup per block, thread per row.
__global__ void __launch_bounds__(kTPB) kv_write_kernel(pbl_block_batch B, pbl_kv_out O) {
  __shared__ uint8_t dummy[16];
  for (uint32_t b = blockIdx.x; b < B.n_blocks; b += gridDim.x) {
    if (to_glb(O.blk_status)[b] != PBL_OK) continue;
    const uint64_t boff = to_glb(B.block_off)[b];
    const Src S = glb_src(B.blocks + boff, to_glb(B.block_len)[b], (lds_cu8)to_lds(dummy));
    KvDesc D;
    (void)kv_desc(S, &D);
    const uint64_t base = to_glb(O.blk_base)[b];
    for (uint32_t r = threadIdx.x; r < D.rows; r += kTPB) {
      uint64_t a;
      uint32_t n;
      kv_slice(S, D.koff, D.kdata, r, &a, &n);
      to_glb(O.key_off)[base + r] = boff + a;
      to_glb(O.key_len)[base + r] = n;
      kv_slice(S, D.voff, D.vdata, r, &a, &n);
      to_glb(O.val_off)[base + r] = boff + a;
      to_glb(O.val_len)[base + r] = n;
    }
  }
}


// ---- value blocks (sstable/valblk) ----------------------------------------------
__device__ inline uint64_t le_n(gptr<const uint8_t> p, uint64_t o, uint32_t n) {
  uint64_t v = 0;
  for (uint32_t i = 0; i < n; i++) v |= uint64_t(p[o + i]) << (8 * i);
  return v;
}

// DecodeIndex (valblk.go:338-368) with one workgroup: row i = (block num, offset,
// length) little-endian in the IndexHandle's widths.
__global__ void __launch_bounds__(kTPB) valblk_index_kernel(const uint8_t* vbi, uint64_t len, uint32_t nw,
                                                            uint32_t ow, uint32_t lw, uint64_t* ho, uint64_t* hl,
                                                            uint32_t cap, uint32_t* n_out, uint32_t* status) {
  const uint32_t w = nw + ow + lw;
  const bool bad_w = nw == 0 || ow == 0 || lw == 0 || nw > 8 || ow > 8 || lw > 8;
  const uint64_t rows = bad_w ? 0 : len / w;
  bool bad = bad_w || len % w != 0;
  const gptr<const uint8_t> p = to_glb(vbi);
  for (uint64_t i = threadIdx.x; i < rows; i += kTPB) {
    const uint64_t o = i * w;
    if (le_n(p, o, nw) != i) bad = true;
    if (i < cap) {
      to_glb(ho)[i] = le_n(p, o + nw, ow);
      to_glb(hl)[i] = le_n(p, o + nw + ow, lw);
    }
  }
  bad = __syncthreads_or(bad);
  if (threadIdx.x == 0) {
    to_glb(n_out)[0] = uint32_t(rows);
    to_glb(status)[0] = bad ? PBL_CORRUPT_VALUE_HANDLE : PBL_OK;
  }
}

// One KV's resolved value: its slice of the decoded values, or the value-block
// bytes its valblk.Handle names (prefix byte, then uvarint ValueLen, BlockNum,
// OffsetInBlock: valblk.go:218-279).  Returns false when the handle is malformed
// or past its block (valueBlockFetcher.getValueInternal, valblk/reader.go:280-302).
struct ValSrc {
  const uint8_t* p;
  uint32_t n;
};
__device__ inline bool kv_value(const pbl_decode_out& D, const pbl_block_batch& V, uint32_t b, uint64_t k0,
                                uint64_t vb, uint64_t k, ValSrc* out) {
  const uint64_t j = k - k0;
  const uint64_t v0 = vb + to_glb(D.val_off)[k0 + b + j], v1 = vb + to_glb(D.val_off)[k0 + b + j + 1];
  const gptr<const uint8_t> vals = to_glb(static_cast<const uint8_t*>(D.val_bytes));
  if (!(to_glb(D.kv_flags)[k] & PBL_KV_VALBLK_HANDLE)) {
    *out = ValSrc{D.val_bytes + v0, uint32_t(v1 - v0)};
    return true;
  }
  uint64_t vlen = 0, bn = 0, oib = 0;
  const int a = v1 > v0 ? uvarint64(vals, v0 + 1, v1, &vlen) : 0;
  const int c = a > 0 ? uvarint64(vals, v0 + 1 + a, v1, &bn) : 0;
  const int d = c > 0 ? uvarint64(vals, v0 + 1 + a + c, v1, &oib) : 0;
  if (d <= 0 || bn >= V.n_blocks || vlen > 0xffffffffull) return false;
  const uint64_t blen = to_glb(V.block_len)[bn];
  if (oib > blen || vlen > blen - oib) return false;
  *out = ValSrc{V.blocks + to_glb(V.block_off)[bn] + oib, uint32_t(vlen)};
  return true;
}

// Pass 1 (wave per block): resolved lengths -> block-relative val_off (N+1 per
// block) and the block's total in blk_val_base[b].
__global__ void __launch_bounds__(kTPB) resolve_size_kernel(pbl_decode_out D, uint32_t nb, pbl_block_batch V,
                                                            pbl_value_out O) {
  const uint32_t wpb = kTPB / kWave;
  for (uint32_t b = blockIdx.x * wpb + wave_id(); b < nb; b += gridDim.x * wpb) {
    const uint64_t k0 = to_glb(D.blk_kv_base)[b], k1 = to_glb(D.blk_kv_base)[b + 1];
    const uint64_t vb = to_glb(D.blk_val_base)[b];
    uint32_t st = to_glb(D.blk_status)[b];
    uint64_t carry = 0;
    bool bad = false;
    if (st == PBL_OK) {
      for (uint64_t c0 = k0; c0 < k1; c0 += kWave) {
        const uint64_t k = c0 + lane_id();
        uint64_t n = 0;
        if (k < k1) {
          ValSrc v;
          if (kv_value(D, V, b, k0, vb, k, &v)) n = v.n;
          else bad = true;
        }
        const uint64_t incl = wave_incl_scan(n);
        if (k < k1) to_glb(O.val_off)[k0 + b + (k - k0) + 1] = uint32_t(carry + incl);
        carry += __shfl(incl, kWave - 1, kWave);
      }
      if (__ballot(bad)) st = PBL_CORRUPT_VALUE_HANDLE;
      else if (carry > 0xffffffffull) st = PBL_UNSUPPORTED;
    }
    if (lane_id() == 0) {
      to_glb(O.val_off)[k0 + b] = 0;
      to_glb(O.blk_status)[b] = st;
      to_glb(O.blk_val_base)[b] = st == PBL_OK ? carry : 0;
    }
  }
}

// Pass 3: workgroup per block, a wave per KV, lanes over its bytes.
__global__ void __launch_bounds__(kTPB) resolve_write_kernel(pbl_decode_out D, uint32_t nb, pbl_block_batch V,
                                                             pbl_value_out O) {
  const uint32_t wpb = kTPB / kWave;
  for (uint32_t b = blockIdx.x; b < nb; b += gridDim.x) {
    if (to_glb(O.blk_status)[b] != PBL_OK) continue;
    const uint64_t k0 = to_glb(D.blk_kv_base)[b], k1 = to_glb(D.blk_kv_base)[b + 1];
    const uint64_t vb = to_glb(D.blk_val_base)[b], ob = to_glb(O.blk_val_base)[b];
    for (uint64_t k = k0 + wave_id(); k < k1; k += wpb) {
      ValSrc v;
      (void)kv_value(D, V, b, k0, vb, k, &v);
      const uint64_t dst = ob + to_glb(O.val_off)[k0 + b + (k - k0)];
      const gptr<const uint8_t> src = to_glb(v.p);
      for (uint32_t i = lane_id(); i < v.n; i += kWave) to_glb(O.val_bytes)[dst + i] = src[i];
    }
  }
}

}  // namespace sst
}  // namespace pbl

namespace {
// ---- host: parseFooter --------------------------------------------------------------
constexpr uint64_t kMagicLen = 8, kVersionLen = 4, kChecksumLen = 4, kAttrLen = 4;
constexpr uint64_t kLevelDBFooterLen = 48;
constexpr uint64_t kRocksDBFooterLen = 1 + 2 * 20 + kVersionLen + kMagicLen;  // 53
constexpr uint64_t kCheckedFooterLen = kRocksDBFooterLen + kChecksumLen;       // 57
constexpr uint64_t kV7FooterLen = kCheckedFooterLen + kAttrLen;                // 61
const uint8_t kLevelDBMagic[8] = {0x57, 0xfb, 0x80, 0x8b, 0x24, 0x75, 0x47, 0xdb};
const uint8_t kRocksDBMagic[8] = {0xf7, 0xcf, 0xf4, 0x85, 0xb7, 0x41, 0xe2, 0x88};
const uint8_t kPebbleDBMagic[8] = {0xf0, 0x9f, 0xaa, 0xb3, 0xf0, 0x9f, 0xaa, 0xb3};

uint32_t le32h(const uint8_t* p) {
  return uint32_t(p[0]) | uint32_t(p[1]) << 8 | uint32_t(p[2]) << 16 | uint32_t(p[3]) << 24;
}

// crc.New(b).Value() (internal/crc/crc.go:21-40) over two pieces
uint32_t crc_update(uint32_t crc, const uint8_t* p, uint64_t n) {
  static uint32_t tab[256];
  static bool ready = false;
  if (!ready) {
    for (uint32_t i = 0; i < 256; i++) {
      uint32_t c = i;
      for (int k = 0; k < 8; k++) c = (c & 1) ? (c >> 1) ^ 0x82F63B78u : c >> 1;
      tab[i] = c;
    }
    ready = true;
  }
  uint32_t c = ~crc;
  for (uint64_t i = 0; i < n; i++) c = tab[(c ^ p[i]) & 0xff] ^ (c >> 8);
  return ~c;
}

// block.DecodeHandle: Go binary.Uvarint twice; 0 = invalid
int decode_handle(const uint8_t* p, uint64_t n, uint64_t* off, uint64_t* len) {
  auto uv = [](const uint8_t* q, uint64_t m, uint64_t* v) -> int {
    uint64_t x = 0;
    uint32_t s = 0;
    for (uint64_t i = 0; i < m && i < 10; i++) {
      const uint8_t b = q[i];
      if (b < 0x80) {
        if (i == 9 && b > 1) return -1;
        *v = x | uint64_t(b) << s;
        return int(i) + 1;
      }
      x |= uint64_t(b & 0x7f) << s;
      s += 7;
    }
    return m >= 10 ? -1 : 0;
  };
  const int a = uv(p, n, off);
  if (a <= 0) return 0;
  const int b = uv(p + a, n - uint64_t(a), len);
  if (b <= 0) return 0;
  return a + b;
}
}  // namespace

extern "C" {

int pbl_parse_footer(const uint8_t* buf, uint64_t buf_len, uint64_t file_size, pbl_footer* out) {
  if (!buf || !out) return PBL_INVALID_ARG;
  std::memset(out, 0, sizeof(*out));
  if (buf_len < kMagicLen || buf_len > file_size) return PBL_CORRUPT_FOOTER;
  const uint64_t off = file_size - buf_len;  // file offset of buf[0]
  const uint8_t* magic = buf + buf_len - kMagicLen;
  const uint8_t* f;
  uint64_t flen;
  if (!std::memcmp(magic, kLevelDBMagic, 8)) {
    if (buf_len < kLevelDBFooterLen) return PBL_CORRUPT_FOOTER;
    flen = kLevelDBFooterLen;
    f = buf + buf_len - flen;
    out->table_format = PBL_TABLE_LEVELDB;
    out->checksum_type = PBL_CHECKSUM_CRC32C;
  } else if (!std::memcmp(magic, kRocksDBMagic, 8) || !std::memcmp(magic, kPebbleDBMagic, 8)) {
    if (buf_len < kRocksDBFooterLen) return PBL_CORRUPT_FOOTER;
    const uint32_t version = le32h(buf + buf_len - kMagicLen - kVersionLen);
    uint32_t fmt;
    if (!std::memcmp(magic, kRocksDBMagic, 8)) {
      if (version != 2) return PBL_CORRUPT_FOOTER;  // parseTableFormat (format.go:261-295)
      fmt = PBL_TABLE_ROCKSDBV2;
    } else {
      if (version < 1 || version > 8) return PBL_CORRUPT_FOOTER;
      fmt = PBL_TABLE_PEBBLEV1 + (version - 1);
    }
    flen = fmt >= PBL_TABLE_PEBBLEV7 ? kV7FooterLen : fmt >= PBL_TABLE_PEBBLEV6 ? kCheckedFooterLen
                                                                                : kRocksDBFooterLen;
    if (buf_len < flen) return PBL_CORRUPT_FOOTER;
    f = buf + buf_len - flen;
    out->table_format = fmt;
    if (f[0] != PBL_CHECKSUM_CRC32C && f[0] != PBL_CHECKSUM_XXHASH64) return PBL_CORRUPT_FOOTER;
    out->checksum_type = f[0];
    if (fmt >= PBL_TABLE_PEBBLEV6) {
      const uint64_t co = fmt >= PBL_TABLE_PEBBLEV7 ? kV7FooterLen - kMagicLen - kVersionLen - kChecksumLen
                                                     : kCheckedFooterLen - kMagicLen - kVersionLen - kChecksumLen;
      if (fmt >= PBL_TABLE_PEBBLEV7) out->attributes = le32h(f + co - kAttrLen);
      const uint32_t want = le32h(f + co);
      uint32_t c = crc_update(0, f, co);
      c = crc_update(c, f + co + kChecksumLen, flen - co - kChecksumLen);
      const uint32_t v = ((c >> 15) | (c << 17)) + 0xa282ead8u;
      if (v != want) return PBL_CORRUPT_FOOTER;
    }
    f += 1;  // past the checksum type
  } else {
    return PBL_CORRUPT_FOOTER;
  }
  out->footer_off = off + buf_len - flen;
  out->footer_len = flen;
  const uint64_t avail = (buf + buf_len) - f;
  const int n = decode_handle(f, avail, &out->metaindex_off, &out->metaindex_len);
  if (n == 0 || out->metaindex_off + out->metaindex_len > file_size) return PBL_CORRUPT_FOOTER;
  const int m = decode_handle(f + n, avail - uint64_t(n), &out->index_off, &out->index_len);
  if (m == 0 || out->index_off + out->index_len > file_size) return PBL_CORRUPT_FOOTER;
  return PBL_OK;
}

int pbl_index_handles_row(const pbl_decode_out* decoded, uint32_t n_blocks, pbl_index_out* out, void* stream) {
  if (!decoded || !out || !out->blk_base || !out->blk_status) return PBL_INVALID_ARG;
  if (n_blocks == 0) return PBL_OK;
  if (!decoded->val_off || !decoded->val_bytes || !decoded->blk_kv_base || !decoded->blk_val_base ||
      !decoded->blk_status || (out->cap && (!out->handle_off || !out->handle_len)))
    return PBL_INVALID_ARG;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const uint32_t wpb = pbl::kTPB / pbl::kWave;
  const uint32_t grid = uint32_t(std::min<uint64_t>((n_blocks + wpb - 1) / wpb, 4096));
  hipLaunchKernelGGL(pbl::sst::index_row_kernel, dim3(grid), dim3(pbl::kTPB), 0, st, *decoded, n_blocks, *out);
  return hipGetLastError() == hipSuccess ? PBL_OK : PBL_DEVICE_ERROR;
}

int pbl_index_handles_col(const pbl_block_batch* batch, pbl_index_out* out, void* stream) {
  if (!batch || !out || !out->blk_base || !out->blk_status) return PBL_INVALID_ARG;
  if (batch->n_blocks == 0) return PBL_OK;
  if (!batch->blocks || !batch->block_off || !batch->block_len || (out->cap && (!out->handle_off || !out->handle_len)))
    return PBL_INVALID_ARG;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const uint32_t nb = batch->n_blocks;
  hipLaunchKernelGGL(pbl::sst::index_col_size_kernel, dim3(std::min<uint32_t>((nb + pbl::kTPB - 1) / pbl::kTPB, 4096)),
                     dim3(pbl::kTPB), 0, st, *batch, *out);
  hipLaunchKernelGGL(pbl::sst::index_col_scan_kernel, dim3(1), dim3(1024), 0, st, nb, *out);
  hipLaunchKernelGGL(pbl::sst::index_col_write_kernel, dim3(std::min<uint32_t>(nb, 4096)), dim3(pbl::kTPB), 0, st,
                     *batch, *out);
  return hipGetLastError() == hipSuccess ? PBL_OK : PBL_DEVICE_ERROR;
}

int pbl_kv_blocks(const pbl_block_batch* batch, pbl_kv_out* out, void* stream) {
  if (!batch || !out || !out->blk_base || !out->blk_status) return PBL_INVALID_ARG;
  if (batch->n_blocks == 0) return PBL_OK;
  if (!batch->blocks || !batch->block_off || !batch->block_len ||
      (out->cap && (!out->key_off || !out->key_len || !out->val_off || !out->val_len)))
    return PBL_INVALID_ARG;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const uint32_t nb = batch->n_blocks;
  const uint32_t wpb = pbl::kTPB / pbl::kWave;
  hipLaunchKernelGGL(pbl::sst::kv_size_kernel, dim3(std::min<uint32_t>((nb + wpb - 1) / wpb, 4096)), dim3(pbl::kTPB),
                     0, st, *batch, *out);
  hipLaunchKernelGGL(pbl::sst::kv_scan_kernel, dim3(1), dim3(1024), 0, st, nb, out->blk_base, out->blk_status,
                     out->cap);
  hipLaunchKernelGGL(pbl::sst::kv_write_kernel, dim3(std::min<uint32_t>(nb, 4096)), dim3(pbl::kTPB), 0, st, *batch,
                     *out);
  return hipGetLastError() == hipSuccess ? PBL_OK : PBL_DEVICE_ERROR;
}

int pbl_valblk_index(const uint8_t* vbi, uint64_t vbi_len, uint32_t num_w, uint32_t off_w, uint32_t len_w,
                     uint64_t* handle_off, uint64_t* handle_len, uint32_t cap, uint32_t* n_blocks,
                     uint32_t* status, void* stream) {
  if ((!vbi && vbi_len) || !n_blocks || !status || (cap && (!handle_off || !handle_len))) return PBL_INVALID_ARG;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  hipLaunchKernelGGL(pbl::sst::valblk_index_kernel, dim3(1), dim3(pbl::kTPB), 0, st, vbi, vbi_len, num_w, off_w,
                     len_w, handle_off, handle_len, cap, n_blocks, status);
  return hipGetLastError() == hipSuccess ? PBL_OK : PBL_DEVICE_ERROR;
}

int pbl_resolve_values(const pbl_decode_out* decoded, uint32_t n_blocks, const pbl_block_batch* value_blocks,
                       pbl_value_out* out, void* stream) {
  if (!decoded || !value_blocks || !out || !out->val_off || !out->blk_val_base || !out->blk_status)
    return PBL_INVALID_ARG;
  if (n_blocks == 0) return PBL_OK;
  if (!decoded->kv_flags || !decoded->val_off || !decoded->val_bytes || !decoded->blk_kv_base ||
      !decoded->blk_val_base || !decoded->blk_status || (out->val_cap && !out->val_bytes) ||
      (value_blocks->n_blocks && (!value_blocks->blocks || !value_blocks->block_off || !value_blocks->block_len)))
    return PBL_INVALID_ARG;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const uint32_t wpb = pbl::kTPB / pbl::kWave;
  hipLaunchKernelGGL(pbl::sst::resolve_size_kernel, dim3(std::min<uint32_t>((n_blocks + wpb - 1) / wpb, 4096)),
                     dim3(pbl::kTPB), 0, st, *decoded, n_blocks, *value_blocks, *out);
  hipLaunchKernelGGL(pbl::sst::kv_scan_kernel, dim3(1), dim3(1024), 0, st, n_blocks, out->blk_val_base,
                     out->blk_status, out->val_cap);
  hipLaunchKernelGGL(pbl::sst::resolve_write_kernel, dim3(std::min<uint32_t>(n_blocks, 4096)), dim3(pbl::kTPB), 0,
                     st, *decoded, n_blocks, *value_blocks, *out);
  return hipGetLastError() == hipSuccess ? PBL_OK : PBL_DEVICE_ERROR;
}

}  // extern "C"
